# Round measurement on one MI355X; every GPU step under its own time limit, chained with &&:
# GPU tests, smoke, PMC passes over bench.py (FETCH_SIZE, WRITE_SIZE; two SQ groups; the SQ
# instruction group again with the early exit off), their summaries into profiles/, then the
# default bench line (which quotes those summaries) and the rocprofv3 kernel-trace stats of the
# same bench command. Outputs under gpurun_out/.
#   bash tools/gpu_round2.sh <tag> [extra bench args...]
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r02}
shift
EXTRA="$*"
KEY=${KEY:-512x512_M256_S32_V10}
mkdir -p gpurun_out
PB="python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --aux-steps 0 $EXTRA"
pmc() {  # name, counters...
  local name=$1; shift
  timeout -k 10 200 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${name}_$TAG -o run -- $PB > gpurun_out/pmc_${name}_$TAG.log 2>&1
}
pmc_noexit() {
  local name=$1; shift
  RM_NO_EARLY_EXIT=1 timeout -k 10 200 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${name}_$TAG -o run -- $PB > gpurun_out/pmc_${name}_$TAG.log 2>&1
}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/tests_$TAG.log; exit 1; }
fi
pmc fetch FETCH_SIZE && pmc write WRITE_SIZE && \
pmc sq1 SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_WAVES && \
pmc sq2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE && \
pmc_noexit sq1x SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_WAVES && \
timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --cpu-baseline off $EXTRA > gpurun_out/bench_pmcargs_$TAG.json && \
python3 tools/pmc_summary.py gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG profiles/${TAG}_pmc_traffic.json $KEY && \
python3 tools/pmc_sq_summary.py profiles/${TAG}_pmc_sq.json $KEY gpurun_out/pmc_sq1_$TAG gpurun_out/pmc_sq2_$TAG gpurun_out/pmc_sq1x_$TAG gpurun_out/bench_pmcargs_$TAG.json && \
cp profiles/${TAG}_pmc_traffic.json profiles/${TAG}_pmc_sq.json gpurun_out/ && \
timeout -k 10 300 python bench.py $EXTRA > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 bench.py --cpu-baseline off --aux-steps 0 $EXTRA > gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo rc=$rc
[ -z "$SKIP_TESTS" ] && tail -3 gpurun_out/tests_$TAG.log
cat gpurun_out/bench_$TAG.json
exit $rc
