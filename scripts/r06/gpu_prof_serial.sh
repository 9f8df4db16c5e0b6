# rocprof kernel stats of the C2 bench step with every dW product in order on the main stream
# (VSPIKE_SIDE=0): per-kernel durations without the side stream's overlap, beside the overlapped
# profile of the final bench (r06_final_bench_kernel_stats.csv)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export VSPIKE_SIDE=0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_prof_serial -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-c4 --profile-steps 0 > gpurun_out/r06_prof_serial.log 2>&1
tail -c 400 gpurun_out/r06_prof_serial.log
