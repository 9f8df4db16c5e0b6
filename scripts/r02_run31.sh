#!/bin/bash
# dW v2: tests, C2 and C3 microbench (default plan vs BN=64 forced), C2 / C3 bench lines.
export TMPDIR=/tmp
M="python scripts/microbench.py --only gemm:dW --reps 50"
MB="python scripts/microbench.py --only base --reps 20"
B="python bench.py --no-cpu-baseline --profile-steps 0 --steps 40 --warmup 10"
B3="python bench.py --no-cpu-baseline --profile-steps 0 --steps 10 --warmup 3 --model vmae_video --neurons 512 --lr 5e-8"
scripts/gpu_steps.sh \
  "dw_tests|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k 'dw or splitk'" \
  "dw_c2|90|$M" \
  "base_def|120|$MB" \
  "base_bn64|120|VSPIKE_DW_BN=64 $MB" \
  "bench_c2|150|$B" \
  "bench_c3|200|$B3" \
  "bench_c3_bn64|200|VSPIKE_DW_BN=64 $B3" || exit $?
for f in dw_c2 base_def base_bn64; do echo "== $f"; grep "dW" gpurun_out/$f.log; done
for f in bench_c2 bench_c3 bench_c3_bn64; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
