#!/bin/bash
# GPU checkpoint at HEAD: full GPU tests, smoke, default bench, rocprof kernel stats, PMC passes.
# usage: scripts/gpu_checkpoint.sh <tag>     (outputs under gpurun_out/, traffic as <tag>_traffic.json)
export TMPDIR=/tmp
set -e
tag=${1:-rXX}
scripts/gpu_steps.sh \
  "tests|700|python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py" \
  "prof|240|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --profile-steps 0 --no-cpu-baseline" \
  "prof_serial|240|VSPIKE_SIDE=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_serial -o run -- python3 bench.py --steps 5 --warmup 2 --profile-steps 0 --no-cpu-baseline"
timeout -k 10 90 python3 scripts/store_rate.py > gpurun_out/${tag}_store_rate.txt 2>&1
scripts/pmc_traffic.sh $tag
ONLY=attn MB_ARGS="--batch 128 --attn-scale 0.5" scripts/pmc_attn.sh gpurun_out/pmc_attn
ONLY=gemm:dW MB_ARGS="--batch 128" scripts/pmc_attn.sh gpurun_out/pmc_dw
python3 scripts/pmc_json.py gpurun_out/pmc_attn gpurun_out/${tag}_pmc_attn.json
python3 scripts/pmc_json.py gpurun_out/pmc_dw gpurun_out/${tag}_pmc_dw.json
