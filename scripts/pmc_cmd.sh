#!/bin/bash
# rocprofv3 PMC passes (one run per pass: SQ issue/wait, MFMA/VALU/LDS, L2 hit/miss, HBM read,
# HBM write) over an arbitrary python command, then the per-kernel JSON summary (scripts/pmc_json.py).
# usage: scripts/pmc_cmd.sh <outdir> <kernel-substring> python3 <script> [args...]
export TMPDIR=/tmp
out=$1; filt=$2; shift 2
mkdir -p "$out"
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES"
B="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"
C="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
# address path and L2 request side: TA busy, L2 requests / memory-side reads, TCP -> L2 read latency
F="GRBM_GUI_ACTIVE TA_BUSY_avr TCC_REQ_sum TCC_EA0_RDREQ_sum"
G="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
for g in ${PMC_PASSES:-a b c d e f g}; do
  case $g in a) CNT=$A;; b) CNT=$B;; c) CNT=$C;; d) CNT=FETCH_SIZE;; e) CNT=WRITE_SIZE;; f) CNT=$F;; g) CNT=$G;; esac
  timeout -s KILL 120 rocprofv3 --pmc $CNT -d "$out" -o $g --output-format csv -- "$@" > "$out/$g.log" 2>&1 || { echo "pass $g failed"; exit 1; }
done
python3 scripts/pmc_json.py "$out" "$out.json" "$filt" && echo "wrote $out.json"
