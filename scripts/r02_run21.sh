#!/bin/bash
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --profile-steps 0 --steps 40 --warmup 10"
set -e; scripts/gpu_steps.sh \
  "t_dw|200|VSPIKE_DW_STAGES=3 python -u -m pytest tests/test_gpu_ops.py -q -x -k 'dw or splitk' --timeout 100 --timeout-method thread -p no:cacheprovider" \
  "s4|120|$B" \
  "s3|120|VSPIKE_DW_STAGES=3 $B" \
  "s4_fuse|120|VSPIKE_LN_FUSE=1 $B" \
  "s3_fuse|120|VSPIKE_DW_STAGES=3 VSPIKE_LN_FUSE=1 $B" \
  "s4b|120|$B" \
  "s3b|120|VSPIKE_DW_STAGES=3 $B" \
  "s3_fuse_b|120|VSPIKE_DW_STAGES=3 VSPIKE_LN_FUSE=1 $B" \
  "mb3|120|VSPIKE_DW_STAGES=3 python scripts/microbench.py --only gemm:dW --reps 20" \
  "mb4|120|python scripts/microbench.py --only gemm:dW --reps 20"
for f in s4 s3 s4_fuse s3_fuse s4b s3b s3_fuse_b; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
cat gpurun_out/mb3.log gpurun_out/mb4.log | grep dW
