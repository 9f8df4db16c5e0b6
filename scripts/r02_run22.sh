#!/bin/bash
export TMPDIR=/tmp
set -e
scripts/gpu_steps.sh \
  "t_attn2|300|VSPIKE_ATTN_BWD=2 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity_bench.py -q -x -k 'attention or attn' --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "mb1|120|python scripts/microbench.py --only attn --reps 20" \
  "mb2|120|VSPIKE_ATTN_BWD=2 python scripts/microbench.py --only attn --reps 20" \
  "mb1b|120|python scripts/microbench.py --only attn --reps 20" \
  "mb2b|120|VSPIKE_ATTN_BWD=2 python scripts/microbench.py --only attn --reps 20"
grep -h "attn bwd" gpurun_out/mb1.log gpurun_out/mb2.log gpurun_out/mb1b.log gpurun_out/mb2b.log
