cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1120 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r06_gpu_tests.log
exit $rc
