# Kernel-trace timeline of the default bench (no PMC): per-step kernel sequence and gaps.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-tl}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/trace_$TAG.log 2>&1 && \
python3 tools/step_timeline.py gpurun_out/trace_$TAG 3
