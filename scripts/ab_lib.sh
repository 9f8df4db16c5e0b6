#!/bin/bash
# A/B two builds of libvspike on one box: alternating bench runs, the second with VSPIKE_LIB.
# usage: scripts/ab_lib.sh <variant .so> <pairs> [bench args...]
V=$1; P=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $P); do
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_new$i.log 2>&1 || exit 1
  VSPIKE_LIB=$V timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_var$i.log 2>&1 || exit 1
done
python - "$P" <<'PY'
import json, sys
for i in range(1, int(sys.argv[1]) + 1):
    r = [json.loads(open(f"gpurun_out/ab_{k}{i}.log").read().strip().splitlines()[-1]) for k in ("new", "var")]
    print(f"pair {i}: new {r[0]['ms_per_step']} ms  variant {r[1]['ms_per_step']} ms")
PY
