#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "tests|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "mb|200|python scripts/microbench.py --reps 20" \
  "prof_dw|200|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dw6 -o run -- python3 scripts/microbench.py --only gemm:dW --reps 20" \
  "bench|300|python bench.py"
