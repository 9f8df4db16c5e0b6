#!/bin/bash
# Round-4 measurement lines beyond the checkpoint: C3 (ViT-Base, the reference plugin's width) at 16
# and 128 clips, C5 (ViT-Base at 32 frames, n = 1024) in fp8 and bf16, the charged-vs-PMC bytes
# check.  usage: scripts/r04_extra.sh <tag>     (outputs under gpurun_out/)
export TMPDIR=/tmp
tag=${1:-r04}
scripts/gpu_steps.sh \
  "c3_b16|300|python -u bench.py --model vmae_video --neurons 512 --lr 5e-8 --batch 16 --no-cpu-baseline --steps 20 --warmup 5" \
  "c3_b128|500|python -u bench.py --model vmae_video --neurons 512 --lr 5e-8 --batch 128 --no-cpu-baseline --steps 10 --warmup 3 --profile-steps 3" \
  "c5_fp8|400|python -u bench.py --model vmae_video --frames 32 --dtype fp8 --neurons 1024 --lr 5e-8 --batch 16 --no-cpu-baseline --steps 20 --warmup 5" \
  "c5_bf16|400|python -u bench.py --model vmae_video --frames 32 --dtype bf16 --neurons 1024 --lr 5e-8 --batch 16 --no-cpu-baseline --steps 20 --warmup 5" \
  "bytes|600|scripts/pmc_bytes_check.sh $tag"
