#!/bin/bash
# dW product sweep: ring/register modes, tile heights, split counts (isolated microbench), plus a
# rocprof split of kernel vs reduce time at the default plan.
export TMPDIR=/tmp
M="python scripts/microbench.py --only gemm:dW --reps 50"
scripts/gpu_steps.sh \
  "dw_def|90|$M" \
  "dw_reg|90|VSPIKE_DW_MODE=0 $M" \
  "dw_s8|90|VSPIKE_DW_SPLITS=8 $M" \
  "dw_s12|90|VSPIKE_DW_SPLITS=12 $M" \
  "dw_s42|90|VSPIKE_DW_SPLITS=42 $M" \
  "dw_bm64|90|VSPIKE_DW_BM=64 $M" \
  "dw_bm128|90|VSPIKE_DW_BM=128 $M" \
  "dw_prof|120|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dw_prof -o run -- python3 scripts/microbench.py --only gemm:dW --reps 50" || exit $?
for f in dw_def dw_reg dw_s8 dw_s12 dw_s42 dw_bm64 dw_bm128; do echo "== $f"; grep "^dW" gpurun_out/$f.log; done
f=$(find gpurun_out/dw_prof -name '*kernel_stats.csv' | head -1); python3 scripts/kstats.py "$f" 1 12
