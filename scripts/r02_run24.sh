#!/bin/bash
# dQ-body fragment prefetch (default build) vs none (libvspike_pf0.so)
export TMPDIR=/tmp
set -e
P0=video-spike_amd/vspike/_build/libvspike_pf0.so
scripts/gpu_steps.sh \
  "t_attn|300|python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity_bench.py -q -x -k 'attention or attn' --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "mb1|120|python scripts/microbench.py --only attn --reps 20" \
  "mb0|120|VSPIKE_LIB=$P0 python scripts/microbench.py --only attn --reps 20" \
  "mb1b|120|python scripts/microbench.py --only attn --reps 20" \
  "mb0b|120|VSPIKE_LIB=$P0 python scripts/microbench.py --only attn --reps 20" \
  "b1|120|python bench.py --no-cpu-baseline --profile-steps 0 --steps 40" \
  "b0|120|VSPIKE_LIB=$P0 python bench.py --no-cpu-baseline --profile-steps 0 --steps 40"
grep -h "attn bwd" gpurun_out/mb1.log gpurun_out/mb0.log gpurun_out/mb1b.log gpurun_out/mb0b.log
for f in b1 b0; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
