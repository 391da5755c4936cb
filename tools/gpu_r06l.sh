# Round 5: contiguous record stores, and blocks without backward seeds write no record columns: the -m gpu suite,
# then WRITE_SIZE / FETCH_SIZE of the metric and C5g, and a same-box A/B against the previous build.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PB="python3 bench.py --steps 5 --warmup 2 --cpu-baseline off --aux-steps 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/$O/pmc_fetch -o run -- $PB > $O/pmc.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/$O/pmc_write -o run -- $PB >> $O/pmc.log 2>&1 && \
python3 tools/pmc_summary.py $O/pmc_fetch $O/pmc_write $O/traffic.json 512x512_M256_S32_V80 auto && \
CONFIGS="m c2cj c5g" ROUNDS=2 bash tools/gpu_ab.sh lib:r06k default 2>&1 | tee $O/ab.txt
