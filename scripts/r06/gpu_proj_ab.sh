set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/gemm_c3_ab.py --knob g256 --values 0,1 --only fwd_proj --rounds 7 --reps 5 --json gpurun_out/r06_proj_g256_ab.json > gpurun_out/r06_proj_g256_ab.log 2>&1
timeout -k 10 300 python -u scripts/gemm_c3_ab.py --knob dw256_all --values 0,1 --only dw_proj --dw --rounds 7 --reps 5 --json gpurun_out/r06_dwproj_ab.json > gpurun_out/r06_dwproj_ab.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "dw_bench128" > gpurun_out/r06_dwproj_tests.log 2>&1
cat gpurun_out/r06_proj_g256_ab.log gpurun_out/r06_dwproj_ab.log; tail -2 gpurun_out/r06_dwproj_tests.log
