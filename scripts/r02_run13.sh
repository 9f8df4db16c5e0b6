#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t_timer|200|python -u -m pytest tests/test_gpu_models.py -q -x -k timers --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "bench|300|python bench.py --no-cpu-baseline"
