#!/bin/bash
export TMPDIR=/tmp
set -e
scripts/gpu_steps.sh \
  "t_big|300|python -u -m pytest tests/test_gpu_ops.py -q -x -k 'big_tile or gemm_layouts or epilogues' --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "mb_big|200|python scripts/microbench.py --only base --reps 10" \
  "mb_old|200|VSPIKE_NO_BIG=1 python scripts/microbench.py --only base --reps 10" \
  "t_models|400|python -u -m pytest tests/test_gpu_models.py tests/test_gpu_parity_bench.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "c3|300|python bench.py --model vmae_video --neurons 512 --lr 5e-8 --no-cpu-baseline --steps 20 --warmup 5 --profile-steps 3" \
  "c2|120|python bench.py --no-cpu-baseline --profile-steps 0"
for f in c3 c2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/$f.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log | head -1)"; done
cat gpurun_out/mb_big.log gpurun_out/mb_old.log | grep base
