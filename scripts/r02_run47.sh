#!/bin/bash
# patch embedding GEMM (BIAS | POS) on the row-slab kernel: tests, same-box A/B
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t|400|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py -k 'patch or epilogue or row_slab or vit_small or tiny'" \
  "prof|200|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p47 -o run -- python3 bench.py --steps 5 --warmup 2 --profile-steps 0 --no-cpu-baseline" || exit $?
f=$(find gpurun_out/p47 -name '*kernel_stats.csv' | head -1); python3 scripts/kstats.py "$f" 7 40 | grep -i "slab\|ring\|im2col"
timeout -k 10 900 scripts/ab_env.sh 3 "VSPIKE_X=0|new" "VSPIKE_NO_SLAB=1|noslab" -- --profile-steps 0 --steps 40 --warmup 10
