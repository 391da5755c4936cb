# Round measurement on one MI355X; every GPU step under its own time limit, chained with &&:
# GPU parity tests, smoke, the two PMC traffic passes of the default bench (FETCH_SIZE and
# WRITE_SIZE in separate runs, --kernel-trace only) summarised into profiles/ (so the bench line
# below carries the traffic), the default bench line (with the CPU baseline), and the rocprofv3
# kernel-trace stats of the same bench command. Outputs under gpurun_out/ (copy the summaries into
# profiles/ afterwards).
#   bash tools/gpu_round.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
KEY=512x512_M256_S32_V10
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/pmc_fetch_$TAG.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/pmc_write_$TAG.log 2>&1 && \
rm -f profiles/${TAG}_pmc_traffic.json && \
python3 tools/pmc_summary.py gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG profiles/${TAG}_pmc_traffic.json $KEY && \
cp profiles/${TAG}_pmc_traffic.json gpurun_out/${TAG}_pmc_traffic.json && \
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 bench.py --cpu-baseline off > gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo rc=$rc
tail -2 gpurun_out/tests_$TAG.log
tail -1 gpurun_out/smoke_$TAG.log
cat gpurun_out/bench_$TAG.json
exit $rc
