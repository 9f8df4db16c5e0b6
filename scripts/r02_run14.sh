#!/bin/bash
# row-slab GEMM: parity, microbench, bench A/B (VSPIKE_NO_SLAB=1 = previous path)
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t_slab|300|python -u -m pytest tests/test_gpu_ops.py -q -x -k 'slab or gemm_layouts or epilogues' --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "t_models|300|python -u -m pytest tests/test_gpu_models.py tests/test_gpu_parity_bench.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "mb|200|python scripts/microbench.py --only gemm --reps 20" \
  "mb_old|200|VSPIKE_NO_SLAB=1 python scripts/microbench.py --only gemm --reps 20" \
  "bench|200|python bench.py --no-cpu-baseline --profile-steps 5" \
  "bench_old|200|VSPIKE_NO_SLAB=1 python bench.py --no-cpu-baseline --profile-steps 5" \
  "bench2|200|python bench.py --no-cpu-baseline --profile-steps 0"
