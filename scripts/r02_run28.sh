#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "c3_curve_lr|300|python scripts/c3_curve.py 12 --lr 5e-8" \
  "c3|300|python bench.py --model vmae_video --neurons 512 --lr 5e-8 --no-cpu-baseline --steps 20 --warmup 5 --profile-steps 3"
grep -o '"ms_per_step": [0-9.]*\|"final_loss": [^,]*' gpurun_out/c3.log
