#!/bin/bash
# dW kernel checkpoint: op tests first (new kernel), then the full GPU suite, microbench old vs new, bench
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t_dw|300|python -u -m pytest tests/test_gpu_ops.py -x -q -k 'splitk or dw_kernel' --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "tests|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "mb_old|120|VSPIKE_DW_OLD=1 python scripts/microbench.py --only gemm:dW --reps 30" \
  "mb_new|120|python scripts/microbench.py --only gemm --reps 30" \
  "bench_old|200|VSPIKE_DW_OLD=1 python bench.py --no-cpu-baseline" \
  "bench|300|python bench.py"
