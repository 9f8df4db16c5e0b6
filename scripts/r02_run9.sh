#!/bin/bash
# A/B: write-through (sc1) epilogue stores vs plain; DP bf16 determinism with/without deferred joins.
export TMPDIR=/tmp
WT=video-spike_amd/vspike/_build/libvspike_wt.so
scripts/gpu_steps.sh \
  "mb_plain|200|python scripts/microbench.py --reps 10" \
  "mb_wt|200|VSPIKE_LIB=$WT python scripts/microbench.py --reps 10" \
  "bench_plain|200|python bench.py --steps 30 --warmup 10 --profile-steps 5 --no-cpu-baseline" \
  "bench_wt|200|VSPIKE_LIB=$WT python bench.py --steps 30 --warmup 10 --profile-steps 5 --no-cpu-baseline" \
  "bench_plain2|200|python bench.py --steps 30 --warmup 10 --profile-steps 0 --no-cpu-baseline" \
  "bench_wt2|200|VSPIKE_LIB=$WT python bench.py --steps 30 --warmup 10 --profile-steps 0 --no-cpu-baseline" \
  "dp_d0a|300|VSPIKE_DEFER=0 python -u -m pytest tests/test_gpu_dp.py -q -s -k 'bf16' --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "dp_d0b|300|VSPIKE_DEFER=0 python -u -m pytest tests/test_gpu_dp.py -q -s -k 'bf16' --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "dp_dla|300|python -u -m pytest tests/test_gpu_dp.py -q -s -k 'bf16' --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "dp_dlb|300|python -u -m pytest tests/test_gpu_dp.py -q -s -k 'bf16' --timeout 200 --timeout-method thread -p no:cacheprovider"
