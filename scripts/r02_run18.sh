#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t_ln|300|python -u -m pytest tests/test_gpu_ops.py -q -x -k 'ln_bwd or layernorm or slab' --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "t_models|400|python -u -m pytest tests/test_gpu_models.py tests/test_gpu_parity_bench.py tests/test_gpu_dp.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "bench|200|python bench.py --no-cpu-baseline --profile-steps 5" \
  "bench_old|200|VSPIKE_NO_LN_FUSE=1 python bench.py --no-cpu-baseline --profile-steps 0" \
  "bench2|200|python bench.py --no-cpu-baseline --profile-steps 0"
