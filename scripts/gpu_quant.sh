set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_c5.py > gpurun_out/r06_quant_tests.log 2>&1
timeout -k 10 300 python -u scripts/quant_bench.py > gpurun_out/r06_quant_bench.txt 2>&1
tail -2 gpurun_out/r06_quant_tests.log; cat gpurun_out/r06_quant_bench.txt
