#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "tests|600|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "t_dp2|400|python -u -m pytest tests/test_gpu_dp.py -q -s -k 'bf16' --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "stamp576|120|VSPIKE_LIB=video-spike_amd/vspike/_build/libvspike_stamp.so N=576 python scripts/stamp_gemm.py" \
  "stamp768|120|VSPIKE_LIB=video-spike_amd/vspike/_build/libvspike_stamp.so N=768 python scripts/stamp_gemm.py" \
  "mb_lin|100|python scripts/microbench.py --only linear --reps 10"
