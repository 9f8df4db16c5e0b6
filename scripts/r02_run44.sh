#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh "tests|700|python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
