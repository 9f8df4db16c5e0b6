#!/bin/bash
# bf16 dh1 / dh2 into the LayerNorm backward: tests, same-box round-robin A/B vs f32 dh (VSPIKE_DH_F32=1)
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t|600|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_parity_bench.py tests/test_gpu_dp.py -k 'layernorm or bf16 or parity or vit or two_ranks or accelerate or side'" || exit $?
timeout -k 10 900 scripts/ab_env.sh 3 "VSPIKE_X=0|bf16dh" "VSPIKE_DH_F32=1|f32dh" -- --profile-steps 0 --steps 40 --warmup 10
