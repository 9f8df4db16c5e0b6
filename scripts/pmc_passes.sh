#!/bin/bash
# SQ counter passes (a: wave-cycle split, b: instruction / LDS mix, c: clock + co-issue) over
# scripts/microbench.py, one rocprofv3 run per pass, then the per-kernel JSON summary.
# usage: scripts/pmc_passes.sh <outdir> <microbench --only value> [extra microbench args]
export TMPDIR=/tmp
out=$1; only=$2; shift 2
mkdir -p "$out"
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES"
B="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"
C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA"
for g in a b c; do
  case $g in a) CNT=$A;; b) CNT=$B;; c) CNT=$C;; esac
  timeout -s KILL 150 rocprofv3 --pmc $CNT -d "$out" -o $g --output-format csv -- python3 scripts/microbench.py --only "$only" --reps 5 "$@" > "$out/$g.log" 2>&1 || { echo "pass $g failed"; exit 1; }
done
python3 scripts/pmc_json.py "$out" "$out.json" && echo "wrote $out.json"
