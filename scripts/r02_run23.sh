#!/bin/bash
export TMPDIR=/tmp
ST=video-spike_amd/vspike/_build/libvspike_stamp.so
scripts/gpu_steps.sh \
  "st_qkv|120|VSPIKE_LIB=$ST python scripts/stamp_gemm.py" \
  "st_fc1|120|VSPIKE_LIB=$ST N=768 EPI=gelu python scripts/stamp_gemm.py"
