#!/bin/bash
# bench with the serialised instrumented pass + serialised rocprof stats (same HEAD as r02_v4 kernels)
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "bench|300|python bench.py" \
  "prof_serial|240|VSPIKE_SIDE=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_serial -o run -- python3 bench.py --steps 5 --warmup 2 --profile-steps 0 --no-cpu-baseline" || exit $?
