#!/bin/bash
# input-walking im2col: tests + rocprof of the step
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t|400|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_preprocess.py -k 'im2col or patch or vit_small or tiny or preprocess'" \
  "prof|200|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p48 -o run -- python3 bench.py --steps 5 --warmup 2 --profile-steps 0 --no-cpu-baseline" || exit $?
f=$(find gpurun_out/p48 -name '*kernel_stats.csv' | head -1); python3 scripts/kstats.py "$f" 7 40 | grep -i "im2col\|total"
