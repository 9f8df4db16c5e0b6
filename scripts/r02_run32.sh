#!/bin/bash
# W-resident K = 192 kernel: tests, microbench (on / off), bench A/B.
export TMPDIR=/tmp
M="python scripts/microbench.py --only gemm --reps 50"
B="python bench.py --no-cpu-baseline --profile-steps 0 --steps 40 --warmup 10"
scripts/gpu_steps.sh \
  "wres_tests|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k 'w_resident or wide_row_slab'" \
  "mb_wres|90|$M" \
  "mb_nowres|90|VSPIKE_NO_WRES=1 $M" \
  "bench_wres|150|$B" \
  "bench_nowres|150|VSPIKE_NO_WRES=1 $B" \
  "bench_wres_b|150|$B" || exit $?
for f in mb_wres mb_nowres; do echo "== $f"; grep -E "^fwd|^bwd da" gpurun_out/$f.log; done
for f in bench_wres bench_nowres bench_wres_b; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
