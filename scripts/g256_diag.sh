export VSPIKE_LIB=$PWD/video-spike_amd/vspike/_build/libvspike_dbg.so
for d in 0 1 2 3; do
  VSPIKE_G256_DBG=$d timeout -k 10 120 python -u scripts/gemm_c3_bench.py --no-torch --only fwd > gpurun_out/diag_$d.log 2>&1 || exit 1
  VSPIKE_G256_DBG=$d timeout -k 10 120 python -u scripts/gemm_c3_bench.py --no-torch --only dx > gpurun_out/diagdx_$d.log 2>&1 || exit 1
done
