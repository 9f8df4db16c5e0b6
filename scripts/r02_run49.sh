#!/bin/bash
# final HEAD check: full GPU tests, smoke, default bench
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "tests|700|python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|300|python bench.py" || exit $?
