# The 256 x 256 GEMM's odd-slot start offset (VS_KNOB_G256_STAGGER, s_sleep(127) units of ~4 us) on the
# round-6 kernel: forward / dX products A/B'd in one process (outputs bitwise equal across values)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/gemm_c3_ab.py --knob g256_stagger --values 0,2,4,8 --rounds 5 --reps 5 \
  --json gpurun_out/r06_g256_stagger_ab.json > gpurun_out/r06_g256_stagger_ab.log 2>&1 || { tail -20 gpurun_out/r06_g256_stagger_ab.log; exit 1; }
cat gpurun_out/r06_g256_stagger_ab.log
