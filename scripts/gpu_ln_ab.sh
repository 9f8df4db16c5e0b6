set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ln_ab.py --knob ln_blocks --values 1024,0,384,640 --json gpurun_out/r06_ln_ab2.json > gpurun_out/r06_ln_ab2.log 2>&1
timeout -k 10 300 python -u scripts/ln_ab.py --fwd --knob ln_fwd_blocks --values 0,1792,1536,1024,768 --json gpurun_out/r06_lnf_ab.json > gpurun_out/r06_lnf_ab.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "layernorm or ln_" > gpurun_out/r06_ln_tests.log 2>&1
cat gpurun_out/r06_ln_ab2.log gpurun_out/r06_lnf_ab.log; tail -2 gpurun_out/r06_ln_tests.log
