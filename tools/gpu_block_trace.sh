# Per-wave timelines of one train launch (measurement build lib/var/trace.so, -DRM_BLOCK_TRACE) at
# the metric, C5 and C2, plus the default bench line as a regression check.
#   bash tools/gpu_block_trace.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-bt}
mkdir -p gpurun_out/bt_$TAG
export RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so
timeout -k 10 200 python tools/block_trace.py --out gpurun_out/bt_$TAG/metric.npz > gpurun_out/bt_$TAG/metric.txt 2>&1 && \
timeout -k 10 300 python tools/block_trace.py --spheres 4096 --march-steps 128 --views 1 --warm 2 --out gpurun_out/bt_$TAG/c5.npz > gpurun_out/bt_$TAG/c5.txt 2>&1 && \
timeout -k 10 200 python tools/block_trace.py --width 256 --height 256 --spheres 64 --out gpurun_out/bt_$TAG/c2.npz > gpurun_out/bt_$TAG/c2.txt 2>&1 && \
unset RM_LIB_PATH && \
timeout -k 10 300 python bench.py --cpu-baseline off > gpurun_out/bt_$TAG/bench.json 2> gpurun_out/bt_$TAG/bench.err
rc=$?
head -60 gpurun_out/bt_$TAG/c5.txt
exit $rc
