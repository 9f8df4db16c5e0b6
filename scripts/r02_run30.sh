#!/bin/bash
# dW kernel v2 (BN in {64,128}, step-invariant DMA offsets, split-order reduce): tests + sweep.
export TMPDIR=/tmp
M="python scripts/microbench.py --only gemm:dW --reps 50"
scripts/gpu_steps.sh \
  "dw_tests|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k 'dw or splitk'" \
  "dw_def|90|$M" \
  "dw_bn64|90|VSPIKE_DW_BN=64 $M" \
  "dw_bn128|90|VSPIKE_DW_BN=128 $M" \
  "dw_bn128_s16|90|VSPIKE_DW_BN=128 VSPIKE_DW_SPLITS=16 $M" \
  "dw_bn128_s24|90|VSPIKE_DW_BN=128 VSPIKE_DW_SPLITS=24 $M" \
  "dw_prof|120|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dw_prof -o run -- python3 scripts/microbench.py --only gemm:dW --reps 50" || exit $?
for f in dw_def dw_bn64 dw_bn128 dw_bn128_s16 dw_bn128_s24; do echo "== $f"; grep "^dW" gpurun_out/$f.log; done
f=$(find gpurun_out/dw_prof -name '*kernel_stats.csv' | head -1); python3 scripts/kstats.py "$f" 1 12
