# Round measurement on one MI355X (every GPU step under its own time limit, chained with &&):
# the -m gpu suite and smoke, PMC passes over the default bench command (FETCH_SIZE, WRITE_SIZE;
# two SQ groups; the SQ instruction group again with the early exit off), their summaries into
# profiles/<tag>_pmc_*.json, then the default bench line (which quotes those summaries) and the
# rocprofv3 kernel-trace stats of the same command. Outputs under gpurun_out/<tag>/.
#   bash tools/gpu_round.sh <tag> [extra bench args...]   (SKIP_TESTS=1: measurement only; CALIB=<json>)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
shift
EXTRA="$*"
O=gpurun_out/$TAG
mkdir -p $O
# the key bench.py looks the summaries up by (its W x H, M, S, views per GPU)
KEY=${KEY:-512x512_M256_S32_V80}
PB="python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --aux-steps 0 $EXTRA"
pmc() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $R/$O/pmc_$name -o run -- $PB > $O/pmc_$name.log 2>&1
}
pmc_noexit() {
  local name=$1; shift
  RM_NO_EARLY_EXIT=1 timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $R/$O/pmc_$name -o run -- $PB > $O/pmc_$name.log 2>&1
}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
  cp gpurun_out/parity_margins.json $O/
fi
pmc fetch FETCH_SIZE && pmc write WRITE_SIZE && \
pmc sq1 SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_WAVES && \
pmc sq2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE && \
pmc_noexit sq1x SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_WAVES && \
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-baseline off $EXTRA > $O/bench_pmcargs.json && \
python3 tools/pmc_summary.py $O/pmc_fetch $O/pmc_write profiles/${TAG}_pmc_traffic.json $KEY auto $CALIB && \
python3 tools/pmc_sq_summary.py profiles/${TAG}_pmc_sq.json $KEY $O/pmc_sq1 $O/pmc_sq2 $O/pmc_sq1x $O/bench_pmcargs.json && \
cp profiles/${TAG}_pmc_traffic.json profiles/${TAG}_pmc_sq.json $O/ && \
timeout -k 10 300 python bench.py $EXTRA > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 bench.py --cpu-baseline off --aux-steps 0 $EXTRA > $O/prof.log 2>&1
rc=$?
echo rc=$rc
[ -z "$SKIP_TESTS" ] && tail -3 $O/tests.log
cat $O/bench.json
exit $rc
