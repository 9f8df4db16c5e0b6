#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t_ops|300|python -u -m pytest tests/test_gpu_ops.py -q -x -k 'slab or panel or gemm' --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "mb|200|python scripts/microbench.py --only copy --reps 20" \
  "bench|200|python bench.py --no-cpu-baseline --profile-steps 5" \
  "bench2|200|python bench.py --no-cpu-baseline --profile-steps 0"
