#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "c3_curve_frozen|300|python scripts/c3_curve.py 12 --freeze" \
  "c3_curve|300|python scripts/c3_curve.py 12"
