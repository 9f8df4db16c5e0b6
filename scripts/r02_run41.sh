#!/bin/bash
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --profile-steps 0 --steps 40 --warmup 10"
scripts/gpu_steps.sh \
  "t|300|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py -k 'w_resident or wide_row_slab or bf16'" \
  "b1|150|$B" "b2|150|$B" "b3|150|$B" || exit $?
for f in b1 b2 b3; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log)"; done
