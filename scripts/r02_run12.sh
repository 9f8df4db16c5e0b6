#!/bin/bash
# Isolated per-op microbenchmark + PMC: HBM traffic per bench kernel class, MFMA/VALU/LDS counters
# for attention and the dW GEMMs.
export TMPDIR=/tmp
set -e
timeout -k 10 200 python scripts/microbench.py --reps 20 > gpurun_out/mb.log 2>&1
scripts/pmc_traffic.sh r02_v1
ONLY=attn scripts/pmc_attn.sh gpurun_out/pmc_attn
ONLY=gemm:dW scripts/pmc_attn.sh gpurun_out/pmc_dw
python3 scripts/pmc_summary.py gpurun_out/pmc_attn attn_ > gpurun_out/pmc_attn_summary.txt
python3 scripts/pmc_summary.py gpurun_out/pmc_dw gemm_dw > gpurun_out/pmc_dw_summary.txt
cat gpurun_out/mb.log
