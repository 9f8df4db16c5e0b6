set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ln_ab.py --fwd --knob ln_fwd_blocks --values 2048,0,512,384 --json gpurun_out/r06_lnf_ab2.json > gpurun_out/r06_lnf_ab2.log 2>&1
timeout -k 10 300 python -u scripts/ln_ab.py --fwd --knob ln_fwd_blocks --values 2048,0,512 --cols 192 --json gpurun_out/r06_lnf_ab_c2.json > gpurun_out/r06_lnf_ab_c2.log 2>&1
timeout -k 10 300 python -u scripts/ln_ab.py --knob ln_blocks --values 1024,0,256 --cols 192 --json gpurun_out/r06_ln_ab_c2b.json > gpurun_out/r06_ln_ab_c2b.log 2>&1
cat gpurun_out/r06_lnf_ab2.log gpurun_out/r06_lnf_ab_c2.log gpurun_out/r06_ln_ab_c2b.log
