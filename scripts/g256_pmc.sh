#!/bin/bash
# PMC of the C3 fwd_qkv / dx_qkv products: 256 x 128 big tile vs the opt-in 256 x 256 persistent kernel
set -e
bash scripts/pmc_cmd.sh gpurun_out/pmc_big gemm_bf16 python3 scripts/gemm_c3_bench.py --no-torch --only fwd_qkv --reps 3 > gpurun_out/pmc_big.txt 2>&1
VSPIKE_G256=1 bash scripts/pmc_cmd.sh gpurun_out/pmc_g256 gemm_bf16 python3 scripts/gemm_c3_bench.py --no-torch --only fwd_qkv --reps 3 > gpurun_out/pmc_g256.txt 2>&1
