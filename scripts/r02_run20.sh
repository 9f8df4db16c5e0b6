#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t_models|400|python -u -m pytest tests/test_gpu_models.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "bench|120|python bench.py --no-cpu-baseline --profile-steps 0"
