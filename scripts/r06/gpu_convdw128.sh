set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/r3d_ab.py --knob conv_dw128 --values 0,1 --batch 16 --rounds 3 --steps 5 --json gpurun_out/r06_convdw128_ab.json > gpurun_out/r06_convdw128_ab.log 2>&1
grep conv_dw128 gpurun_out/r06_convdw128_ab.log
