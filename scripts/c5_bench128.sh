#!/bin/bash
# BASELINE C5 encoder geometry (ViT-Base, 32 frames = 3,136 tokens, n = 1024) at the reference's
# 128-clip batch: fp8 (MX-FP8 block forward products) vs bf16, main line only (no sub-records)
set -e
for dt in fp8 bf16; do
  timeout -k 10 400 python -u bench.py --model vmae_video --frames 32 --neurons 1024 --dtype $dt --batch 128 \
    --lr 5e-8 --steps 5 --warmup 2 --profile-steps 2 --no-cpu-baseline --no-c3 --no-c4 > gpurun_out/c5_${dt}_b128.json 2> gpurun_out/c5_${dt}_b128.err
done
