#!/bin/bash
# schedule knobs re-measured with the r02_v4 kernels: fused dX + LN' (VSPIKE_LN_FUSE=1), join modes
export TMPDIR=/tmp
timeout -k 10 800 scripts/ab_env.sh 3 "VSPIKE_X=0|base" "VSPIKE_LN_FUSE=1|lnfuse" "VSPIKE_DEFER=1|defer1" "VSPIKE_DEFER=0|defer0" -- --profile-steps 0 --steps 40 --warmup 10
