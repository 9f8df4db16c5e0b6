#!/bin/bash
# SQ counter passes + HBM bytes over the fused MLP kernels (scripts/mlp_bench.py), one rocprofv3 run
# per pass, then the per-kernel JSON summary.   usage: scripts/pmc_mlp.sh <outdir>
export TMPDIR=/tmp
out=$1
mkdir -p "$out"
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES"
B="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"
C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA"
for g in a b c d e; do
  case $g in a) CNT=$A;; b) CNT=$B;; c) CNT=$C;; d) CNT=FETCH_SIZE;; e) CNT=WRITE_SIZE;; esac
  timeout -s KILL 150 rocprofv3 --pmc $CNT -d "$out" -o $g --output-format csv -- python3 scripts/mlp_bench.py > "$out/$g.log" 2>&1 || { echo "pass $g failed"; exit 1; }
done
python3 scripts/pmc_json.py "$out" "$out.json" mlp_ && echo "wrote $out.json"
