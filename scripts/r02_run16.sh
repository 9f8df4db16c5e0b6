#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t_ops|300|python -u -m pytest tests/test_gpu_ops.py -q -x -k 'slab or panel' --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "mb|200|python scripts/microbench.py --only gemm --reps 20" \
  "mb_g768|200|VSPIKE_WSLAB_G=768 python scripts/microbench.py --only gemm --reps 20" \
  "mb_old|200|VSPIKE_NO_WSLAB=1 python scripts/microbench.py --only gemm --reps 20"
