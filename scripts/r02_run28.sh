#!/bin/bash
# Side-stream cost: bench with and without the dW side stream, rocprof kernel stats of the serialised step.
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --profile-steps 0 --steps 40 --warmup 10"
scripts/gpu_steps.sh \
  "side_a|150|$B" \
  "noside_a|150|VSPIKE_SIDE=0 $B" \
  "side_b|150|$B" \
  "noside_b|150|VSPIKE_SIDE=0 $B" \
  "prof_noside|240|VSPIKE_SIDE=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_noside -o run -- python3 bench.py --no-cpu-baseline --profile-steps 0 --steps 5 --warmup 2" || exit $?
for f in side_a noside_a side_b noside_b; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
f=$(find gpurun_out/prof_noside -name '*kernel_stats.csv' | head -1); python3 scripts/kstats.py "$f" 7 30
