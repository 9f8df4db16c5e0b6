# fp8 quantisation check and timing, then the full GPU suite and smoke on the final tree
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fp8.py > gpurun_out/r06_quant_tests.log 2>&1 || { tail -20 gpurun_out/r06_quant_tests.log; exit 1; }
timeout -k 10 300 python -u scripts/quant_bench.py > gpurun_out/r06_quant_bench.txt 2>&1 || exit 1
cat gpurun_out/r06_quant_bench.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_tests_final.log 2>&1
rc=$?
tail -3 gpurun_out/r06_gpu_tests_final.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_smoke_final.log 2>&1
rc=$?
tail -2 gpurun_out/r06_smoke_final.log
exit $rc
