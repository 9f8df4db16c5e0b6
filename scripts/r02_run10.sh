#!/bin/bash
# A/B: write-through (sc1) epilogue stores vs plain, interleaved.
export TMPDIR=/tmp
WT=video-spike_amd/vspike/_build/libvspike_wt.so
scripts/gpu_steps.sh \
  "t_wt|300|VSPIKE_LIB=$WT python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity_bench.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "mb_wt|200|VSPIKE_LIB=$WT python scripts/microbench.py --reps 10" \
  "mb_plain|200|python scripts/microbench.py --reps 10" \
  "bench_wt|200|VSPIKE_LIB=$WT python bench.py --steps 30 --warmup 10 --profile-steps 5 --no-cpu-baseline" \
  "bench_plain|200|python bench.py --steps 30 --warmup 10 --profile-steps 5 --no-cpu-baseline" \
  "bench_wt2|200|VSPIKE_LIB=$WT python bench.py --steps 30 --warmup 10 --profile-steps 0 --no-cpu-baseline" \
  "bench_plain2|200|python bench.py --steps 30 --warmup 10 --profile-steps 0 --no-cpu-baseline"
