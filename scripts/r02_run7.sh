#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t_dp|400|python -u -m pytest tests/test_gpu_dp.py -q -s --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "tests|600|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "mb_ln|100|python scripts/microbench.py --only ln --reps 30"
