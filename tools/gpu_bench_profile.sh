# Round-end style measurement on one MI355X: smoke, the default bench line, the rocprofv3
# kernel-trace stats of the same command, and the PMC traffic passes (separate runs; no
# sys/runtime trace next to --pmc). Outputs under gpurun_out/, summaries copied to profiles/.
#   bash tools/gpu_bench_profile.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 bench.py --cpu-baseline off > gpurun_out/prof_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/pmc_fetch_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/pmc_write_$TAG.log 2>&1
rc=$?
echo rc=$rc
tail -2 gpurun_out/smoke_$TAG.log; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
exit $rc
