#!/bin/bash
# side-stream toggle test, bench with the serialised instrumented pass, serialised rocprof stats
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "side_test|200|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_ops.py -k 'side_stream or im2col or patch'" \
  "bench|300|python bench.py" \
  "prof_serial|240|VSPIKE_SIDE=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_serial -o run -- python3 bench.py --steps 5 --warmup 2 --profile-steps 0 --no-cpu-baseline" || exit $?
B="python bench.py --no-cpu-baseline --profile-steps 0 --steps 40 --warmup 10"
scripts/gpu_steps.sh \
  "ln1024|150|$B" "ln512|150|VSPIKE_LN_BLOCKS=512 $B" "ln256|150|VSPIKE_LN_BLOCKS=256 $B" \
  "ln1024b|150|$B" "ln512b|150|VSPIKE_LN_BLOCKS=512 $B" "ln256b|150|VSPIKE_LN_BLOCKS=256 $B" || exit $?
for f in ln1024 ln512 ln256 ln1024b ln512b ln256b; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
