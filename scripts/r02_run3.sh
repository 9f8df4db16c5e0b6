#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t_dw|300|python -u -m pytest tests/test_gpu_ops.py -x -q -k 'splitk or dw_kernel' --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "mb_reg|120|python scripts/microbench.py --only gemm:dW --reps 30" \
  "mb_reg64|120|VSPIKE_DW_BM=64 python scripts/microbench.py --only gemm:dW --reps 30" \
  "mb_reg192|120|VSPIKE_DW_BM=192 python scripts/microbench.py --only gemm:dW --reps 30" \
  "mb_dma|120|VSPIKE_DW_MODE=1 python scripts/microbench.py --only gemm:dW --reps 30" \
  "prof_dw|200|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dw -o run -- python3 scripts/microbench.py --only gemm:dW --reps 20"
