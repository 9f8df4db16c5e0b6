#!/bin/bash
# PMC passes over the attention microbenchmark (one rocprofv3 run per counter group).
# usage: scripts/pmc_attn.sh [outdir]   (env ONLY=attn|gemm|ln, MB_ARGS="--batch 128 ...", VSPIKE_LIB to pick a build)
export TMPDIR=/tmp
set -e
out=${1:-gpurun_out/pmc}
mkdir -p $out
run() { timeout -k 10 180 rocprofv3 --pmc $2 -d $out -o $1 --output-format csv -- python3 scripts/microbench.py --only "${ONLY:-attn}" --reps 5 $MB_ARGS > $out/$1.log 2>&1; }
run a "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES"
run b "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"
run c "GRBM_GUI_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA"
run d "FETCH_SIZE"
run e "WRITE_SIZE"
run f "SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM"
echo done
