# Quick GPU check: default bench line (no CPU baseline) + per-step kernel timeline.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --cpu-baseline off > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); r=d['roofline']; print('BENCH', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'])" && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/trace_$TAG.log 2>&1 && \
python3 tools/step_timeline.py gpurun_out/trace_$TAG 2
