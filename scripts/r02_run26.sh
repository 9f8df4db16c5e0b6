#!/bin/bash
export TMPDIR=/tmp
set -e
scripts/gpu_steps.sh \
  "t_dw|300|python -u -m pytest tests/test_gpu_ops.py -q -x -k 'dw or splitk' --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "t_models|400|python -u -m pytest tests/test_gpu_models.py tests/test_gpu_parity_bench.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "c3|300|python bench.py --model vmae_video --neurons 512 --no-cpu-baseline --steps 20 --warmup 5 --profile-steps 3" \
  "c2|120|python bench.py --no-cpu-baseline --profile-steps 0"
for f in c3 c2; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$f.log | head -1)"; done
