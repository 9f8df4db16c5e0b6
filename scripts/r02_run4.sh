#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t_ops|300|python -u -m pytest tests/test_gpu_ops.py -x -q -k 'splitk or dw_kernel or skinny' --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "mb_dma8|120|python scripts/microbench.py --only gemm:dW --reps 30" \
  "mb_dma8_192|120|VSPIKE_DW_BM=192 python scripts/microbench.py --only gemm:dW --reps 30" \
  "mb_reg|120|VSPIKE_DW_MODE=0 python scripts/microbench.py --only gemm:dW --reps 30" \
  "prof_dw|200|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dw4 -o run -- python3 scripts/microbench.py --only gemm:dW --reps 20" \
  "tests|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench|300|python bench.py --no-cpu-baseline"
