#!/bin/bash
# HBM traffic per launch for every kernel of the bench step, per MI355X_MICROARCH.md "HBM":
# two separate --pmc passes (FETCH_SIZE, WRITE_SIZE cannot share a pass), FETCH_SIZE doubled (gfx950
# tallies 128-B requests of 16-B/lane streams at 64 B).  Output: profiles/<tag>_traffic.json
# usage: scripts/pmc_traffic.sh <tag>     (run on the GPU box)
export TMPDIR=/tmp
set -e
tag=${1:-r01}
out=gpurun_out/pmc_traffic
mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d $out -o $c --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-steps 0 --no-c3 --no-c4 > $out/$c.log 2>&1
done
python3 scripts/traffic_summary.py $out gpurun_out/${tag}_traffic.json 4
