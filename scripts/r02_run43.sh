#!/bin/bash
export TMPDIR=/tmp
M="python scripts/microbench.py --only gemm:fwd --reps 50"
scripts/gpu_steps.sh \
  "t|300|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k 'w_resident'" \
  "mb|90|$M" "mb2|90|$M" || exit $?
for f in mb mb2; do echo "== $f"; grep -E "^fwd" gpurun_out/$f.log; done
