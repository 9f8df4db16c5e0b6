#!/bin/bash
# final round-2 checkpoint (scripts/gpu_checkpoint.sh r02_v8) + C3 bench line
export TMPDIR=/tmp
scripts/gpu_checkpoint.sh r02_v8 || exit $?
scripts/gpu_steps.sh "c3|300|python bench.py --model vmae_video --neurons 512 --lr 5e-8 --steps 10 --warmup 3 --profile-steps 3 --no-cpu-baseline" || exit $?
