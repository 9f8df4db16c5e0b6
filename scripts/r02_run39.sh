#!/bin/bash
# stored gelu' (fc1 forward writes gelu'(pre), the GELU' product multiplies): tests, microbench, bench A/B
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --profile-steps 0 --steps 40 --warmup 10"
scripts/gpu_steps.sh \
  "gg_tests|600|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_parity_bench.py -k 'w_resident or wide_row_slab or epilogue or bf16 or parity or side_stream or vit'" \
  "bench_a|150|$B" "bench_b|150|$B" "bench_wres_gbwd|150|VSPIKE_WRES_GBWD=1 $B" || exit $?
for f in bench_a bench_b bench_wres_gbwd; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
tail -3 gpurun_out/gg_tests.log
