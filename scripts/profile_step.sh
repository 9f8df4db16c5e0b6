#!/bin/bash
# The benched train step under rocprofv3: kernel trace + stats of 5 timed steps (the real,
# side-stream-overlapped schedule), the per-step timeline summary, then the HBM traffic passes.
# usage: scripts/profile_step.sh <tag>     (outputs under gpurun_out/)
export TMPDIR=/tmp
tag=${1:-rXX}
mkdir -p gpurun_out/tl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tl -o run -- \
  python3 bench.py --steps 5 --warmup 3 --profile-steps 0 --no-cpu-baseline > gpurun_out/tl/bench.log 2>&1 || exit $?
python3 scripts/timeline.py "$(ls gpurun_out/tl/*kernel_trace.csv | head -1)" 2 > gpurun_out/tl/timeline.txt
python3 scripts/kstats.py "$(ls gpurun_out/tl/*kernel_stats.csv | head -1)" 8 30 > gpurun_out/tl/kstats.txt
scripts/pmc_traffic.sh "$tag"
