set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-x}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "g256 or big_tile or dw_bench128" > gpurun_out/r06_${tag}_tests.log 2>&1
timeout -k 10 300 python -u scripts/gemm_c3_ab.py --knob g256_a3 --values 2,1 --rounds 5 --reps 5 --dw --json gpurun_out/r06_g256_${tag}_ab.json > gpurun_out/r06_g256_${tag}_ab.log 2>&1
tail -2 gpurun_out/r06_${tag}_tests.log; cat gpurun_out/r06_g256_${tag}_ab.log
