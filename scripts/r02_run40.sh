#!/bin/bash
export TMPDIR=/tmp
M="python scripts/microbench.py --only gemm --reps 50"
scripts/gpu_steps.sh "mb|90|$M" "mb_nowres|90|VSPIKE_NO_WRES=1 $M" \
  "prof_serial|240|VSPIKE_SIDE=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_serial2 -o run -- python3 bench.py --steps 5 --warmup 2 --profile-steps 0 --no-cpu-baseline" || exit $?
for f in mb mb_nowres; do echo "== $f"; grep -E "^fwd|^bwd da" gpurun_out/$f.log; done
f=$(find gpurun_out/prof_serial2 -name '*kernel_stats.csv' | head -1); python3 scripts/kstats.py "$f" 7 14
