# rocprofv3 --kernel-trace --stats of one bench configuration (quick per-kernel durations).
#   bash tools/gpu_prof_quick.sh <tag> <bench args...>
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --cpu-baseline off --aux-steps 0 "$@" > gpurun_out/prof_$TAG/bench.json 2> gpurun_out/prof_$TAG/err.log || { tail -20 gpurun_out/prof_$TAG/err.log; exit 1; }
f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:9.2f} us')
PY
