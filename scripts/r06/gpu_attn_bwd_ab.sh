set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/attn_ab.py --variants 0x0,0x60,0x90 --only bwd --heads 12 --rounds 5 --reps 5 --json gpurun_out/r06_attn_bwd_ab_c3.json > gpurun_out/r06_attn_bwd_ab_c3.log 2>&1
timeout -k 10 400 python -u scripts/attn_ab.py --variants 0x0,0x60,0x90 --only bwd --heads 3 --rounds 5 --reps 5 --json gpurun_out/r06_attn_bwd_ab_c2.json > gpurun_out/r06_attn_bwd_ab_c2.log 2>&1
grep variant gpurun_out/r06_attn_bwd_ab_c3.log gpurun_out/r06_attn_bwd_ab_c2.log
