set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "slab or ln_fwd_fused or ln_bwd_fused or patch_embed" > gpurun_out/r06_slab_tests.log 2>&1
timeout -k 10 900 python -u bench.py --no-c3 --no-c4 --no-cpu-baseline > gpurun_out/r06_slab_bench.json 2> gpurun_out/r06_slab_bench.log
tail -2 gpurun_out/r06_slab_tests.log
python3 -c "
import json; d=json.load(open('gpurun_out/r06_slab_bench.json'))
print('C2', d['value'], d['ms_per_step'])
for k in ('fwd_qkv','fwd_proj','dx_fc1','dx_proj','dx_qkv','fwd_mlp','dx_mlp'): print(k, d['roofline']['all'][k]['ms_per_step'], d['roofline']['all'][k]['avg_launch_us'])
"
