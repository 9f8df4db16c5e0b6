#!/bin/bash
# C3 (ViT-Base, 512 neurons) and the reference-default frozen-encoder mode on one GPU
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "c3|300|python bench.py --model vmae_video --neurons 512 --no-cpu-baseline --steps 20 --warmup 5 --profile-steps 3" \
  "c3_frozen|300|python bench.py --model vmae_video --neurons 512 --freeze --no-cpu-baseline --steps 20 --warmup 5 --profile-steps 3" \
  "c2_frozen|200|python bench.py --freeze --no-cpu-baseline --steps 30 --warmup 5 --profile-steps 3" \
  "c3_prof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 bench.py --model vmae_video --neurons 512 --steps 3 --warmup 1 --profile-steps 0 --no-cpu-baseline"
