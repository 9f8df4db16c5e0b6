#!/bin/bash
# A/B of one build under different environment settings on one box: round-robin bench runs.
# usage: scripts/ab_env.sh <rounds> "<ENV=val ...>|<label>" ... -- [bench args...]
R=$1; shift
specs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do specs+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for s in "${specs[@]}"; do
    envs="${s%%|*}"; lab="${s#*|}"
    env $envs timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > "gpurun_out/abenv_${lab}_$i.log" 2>&1 || exit 1
  done
done
python - "$R" "${specs[@]}" <<'PY'
import json, sys
R = int(sys.argv[1]); labs = [s.split("|", 1)[1] for s in sys.argv[2:]]
for lab in labs:
    v = [json.loads(open(f"gpurun_out/abenv_{lab}_{i}.log").read().strip().splitlines()[-1])["ms_per_step"] for i in range(1, R + 1)]
    print(f"{lab:10s} ms/step {v}  mean {sum(v) / len(v):.3f}")
PY
