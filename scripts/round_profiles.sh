#!/bin/bash
# Round-end evidence for the bench line's roofline (run on the GPU box):
#   1. rocprofv3 --kernel-trace --stats of the C2 bench command (its average attn_bwd duration must agree
#      with bench.py's hipEvent figure)
#   2. HBM traffic per kernel class (separate FETCH_SIZE / WRITE_SIZE passes, scripts/pmc_traffic.sh)
#   3. attention PMC passes at the benched 128 clips (scripts/pmc_attn.sh -> scripts/pmc_json.py)
# usage: scripts/round_profiles.sh <tag>
set -e
tag=${1:-r05}
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-c3 --no-c4 --steps 20 --warmup 5 --profile-steps 5 > gpurun_out/prof_bench.log 2>&1
bash scripts/pmc_traffic.sh $tag
MB_ARGS="--batch 128" bash scripts/pmc_attn.sh gpurun_out/pmc_attn_$tag
python3 scripts/pmc_json.py gpurun_out/pmc_attn_$tag gpurun_out/${tag}_pmc_attn.json attn
