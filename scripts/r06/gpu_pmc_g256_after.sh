set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PMC_PASSES="a b c" bash scripts/pmc_cmd.sh gpurun_out/r06_pmc_g256_qkv_after gemm_bf16_g256 python3 scripts/gemm_c3_ab.py --only fwd_qkv --values 0 --rounds 1 --reps 3
PMC_PASSES="a b c" bash scripts/pmc_cmd.sh gpurun_out/r06_pmc_g256_dxfc1_after gemm_bf16_g256 python3 scripts/gemm_c3_ab.py --only dx_fc1 --values 0 --rounds 1 --reps 3
