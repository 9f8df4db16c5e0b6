#!/bin/bash
# proj product + LayerNorm2 forward in one launch (vs_gemm_ln_fwd): tests, same-box A/B
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "t|600|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_models.py tests/test_gpu_parity_bench.py -k 'ln_fwd or layernorm or bf16 or parity or vit or timers or side'" || exit $?
timeout -k 10 900 scripts/ab_env.sh 3 "VSPIKE_X=0|lnf" "VSPIKE_NO_LNF_FUSE=1|nolnf" -- --profile-steps 0 --steps 40 --warmup 10
