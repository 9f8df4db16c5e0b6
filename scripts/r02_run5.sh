#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t_ops|300|python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "mb_def|120|python scripts/microbench.py --only gemm:dW --reps 30" \
  "mb_s8|120|VSPIKE_DW_SPLITS=8 python scripts/microbench.py --only gemm:dW --reps 30" \
  "mb_s12|120|VSPIKE_DW_SPLITS=12 python scripts/microbench.py --only gemm:dW --reps 30" \
  "mb_s16_192|120|VSPIKE_DW_BM=192 VSPIKE_DW_SPLITS=16 python scripts/microbench.py --only gemm:dW --reps 30" \
  "prof_dw|200|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dw5 -o run -- python3 scripts/microbench.py --only gemm:dW --reps 20" \
  "pmc_attn|400|ONLY=attn scripts/pmc_attn.sh gpurun_out/pmc_attn" \
  "bench|300|python bench.py --no-cpu-baseline"
