set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u bench.py > gpurun_out/r06_final_bench.json 2> gpurun_out/r06_final_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_prof_final -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-c4 --profile-steps 0 > gpurun_out/r06_prof_final.log 2>&1
tail -c 300 gpurun_out/r06_final_bench.json
