#!/bin/bash
# A/B of the backward schedule: fused LN' or not x side stream or not x deferral
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --profile-steps 0 --steps 40 --warmup 10"
scripts/gpu_steps.sh \
  "fused_side|120|$B" \
  "unfused_side|120|VSPIKE_NO_LN_FUSE=1 $B" \
  "fused_noside|120|VSPIKE_SIDE=0 $B" \
  "unfused_noside|120|VSPIKE_NO_LN_FUSE=1 VSPIKE_SIDE=0 $B" \
  "fused_d1|120|VSPIKE_DEFER=1 $B" \
  "fused_d0|120|VSPIKE_DEFER=0 $B" \
  "fused_side_b|120|$B" \
  "unfused_side_b|120|VSPIKE_NO_LN_FUSE=1 $B"
for f in fused_side unfused_side fused_noside unfused_noside fused_d1 fused_d0 fused_side_b unfused_side_b; do
  echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
