# Where the 256 x 256 forward / dX products spend their time on the round-6 kernel: the VS_DEBUG_KNOBS
# build (scripts/variant_build.py dbg VS_DEBUG_KNOBS gemm.hip) timed with VSPIKE_G256_DBG 0 (normal),
# 1 (no operand DMA), 2 (no epilogue stores), 3 (neither) -- timing only, outputs WRONG for 1..3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export VSPIKE_LIB=$PWD/video-spike_amd/vspike/_build/libvspike_dbg.so
timeout -k 10 300 python -u scripts/gemm_c3_ab.py --knob g256_dbg --values 0,1,2,3 --rounds 5 --reps 5 --only fwd \
  --json gpurun_out/r06_g256_diag_fwd.json > gpurun_out/r06_g256_diag_fwd.log 2>&1 || { tail -20 gpurun_out/r06_g256_diag_fwd.log; exit 1; }
cat gpurun_out/r06_g256_diag_fwd.log
timeout -k 10 300 python -u scripts/gemm_c3_ab.py --knob g256_dbg --values 0,1,2,3 --rounds 5 --reps 5 --only dx \
  --json gpurun_out/r06_g256_diag_dx.json > gpurun_out/r06_g256_diag_dx.log 2>&1 || { tail -20 gpurun_out/r06_g256_diag_dx.log; exit 1; }
cat gpurun_out/r06_g256_diag_dx.log
