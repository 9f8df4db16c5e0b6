#!/bin/bash
# Charged vs PMC bytes per bench timer class (scripts/bytes_check.py): two rocprofv3 --pmc passes
# (FETCH_SIZE, WRITE_SIZE cannot share a pass) over one block at the bench batch.
# usage: scripts/pmc_bytes_check.sh <tag>     (on the GPU box; output gpurun_out/<tag>_bytes_check.json)
export TMPDIR=/tmp
set -e
tag=${1:-rXX}
out=gpurun_out/pmc_bytes
mkdir -p $out
timeout -k 10 120 python3 scripts/bytes_check.py run $out/charged.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $c -d $out/$c -o $c --output-format csv -- \
    python3 scripts/bytes_check.py run $out/charged_$c.json > $out/$c.log 2>&1
done
python3 scripts/bytes_check.py parse $out $out/charged.json gpurun_out/${tag}_bytes_check.json
