# round-6 profile set: smoke, rocprof kernel stats of the C2 bench step, HBM traffic PMC passes,
# attention PMC passes and the attention clock (C2 and C3 head counts)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_smoke.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_prof -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-c4 --profile-steps 0 > gpurun_out/r06_prof_bench.log 2>&1
bash scripts/pmc_traffic.sh r06
MB_ARGS="--batch 128" bash scripts/pmc_attn.sh gpurun_out/r06_pmc_attn
python3 scripts/pmc_json.py gpurun_out/r06_pmc_attn gpurun_out/r06_pmc_attn.json attn
timeout -k 10 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/r06_clk2 -o c2 --output-format csv -- python3 scripts/microbench.py --only attn --reps 5 --batch 128 > gpurun_out/r06_clk2.log 2>&1
timeout -k 10 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/r06_clk3 -o c3 --output-format csv -- python3 scripts/microbench.py --only attn --reps 5 --batch 128 --heads 12 > gpurun_out/r06_clk3.log 2>&1
python3 scripts/attn_clock.py gpurun_out/r06_clk2 attn --json gpurun_out/r06_attn_clock_c2.json > gpurun_out/r06_attn_clock_c2.txt
python3 scripts/attn_clock.py gpurun_out/r06_clk3 attn --json gpurun_out/r06_attn_clock_c3.json > gpurun_out/r06_attn_clock_c3.txt
cat gpurun_out/r06_smoke.log | tail -2; cat gpurun_out/r06_attn_clock_c2.txt gpurun_out/r06_attn_clock_c3.txt
