set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-x}
timeout -k 10 1000 python -u bench.py > gpurun_out/r06_${tag}_bench.json 2> gpurun_out/r06_${tag}_bench.log
tail -c 600 gpurun_out/r06_${tag}_bench.json
