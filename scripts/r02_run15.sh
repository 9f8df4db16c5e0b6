#!/bin/bash
# wide row-slab GEMM: parity, microbench A/B, bench
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t_ops|300|python -u -m pytest tests/test_gpu_ops.py -q -x -k 'slab or gemm or panel' --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "t_models|300|python -u -m pytest tests/test_gpu_models.py tests/test_gpu_parity_bench.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "mb|200|python scripts/microbench.py --only gemm --reps 20" \
  "mb_g768|200|VSPIKE_WSLAB_G=768 python scripts/microbench.py --only gemm:fwd --reps 20" \
  "mb_g256|200|VSPIKE_WSLAB_G=256 python scripts/microbench.py --only gemm:fwd --reps 20" \
  "bench|200|python bench.py --no-cpu-baseline --profile-steps 5" \
  "bench_old|200|VSPIKE_NO_WSLAB=1 python bench.py --no-cpu-baseline --profile-steps 0" \
  "bench2|200|python bench.py --no-cpu-baseline --profile-steps 0"
