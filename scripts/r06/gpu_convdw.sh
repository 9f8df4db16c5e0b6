set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_r3d.py > gpurun_out/r06_convdw_tests.log 2>&1
timeout -k 10 400 python -u scripts/r3d_ab.py --knob conv_mfma --values 0,1 --batch 16 --rounds 3 --steps 5 --json gpurun_out/r06_convdw_pf2.json > gpurun_out/r06_convdw_pf2.log 2>&1
tail -2 gpurun_out/r06_convdw_tests.log; grep conv_mfma gpurun_out/r06_convdw_pf2.log
