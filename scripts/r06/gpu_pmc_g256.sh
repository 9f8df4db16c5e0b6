set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "g256" > gpurun_out/r06_a3v1_tests.log 2>&1
timeout -k 10 300 python -u scripts/gemm_c3_ab.py --knob g256_a3 --values 2,1 --rounds 5 --reps 5 --json gpurun_out/r06_g256_a3v1_ab.json > gpurun_out/r06_g256_a3v1_ab.log 2>&1
bash scripts/pmc_cmd.sh gpurun_out/r06_pmc_g256_qkv gemm_bf16_g256 python3 scripts/gemm_c3_ab.py --only fwd_qkv --values 0 --rounds 1 --reps 3
bash scripts/pmc_cmd.sh gpurun_out/r06_pmc_g256_dxfc1 gemm_bf16_g256 python3 scripts/gemm_c3_ab.py --only dx_fc1 --values 0 --rounds 1 --reps 3
tail -2 gpurun_out/r06_a3v1_tests.log; cat gpurun_out/r06_g256_a3v1_ab.log
