set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench_r01a.json 2> gpurun_out/bench_r01a.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r01a -o run -- python3 bench.py --steps 20 --cpu-baseline off > gpurun_out/prof_r01a.log 2>&1
echo rc=$?
cat gpurun_out/smoke.log | tail -2; cat gpurun_out/bench_r01a.json; tail -3 gpurun_out/bench_r01a.err
