# Per-wave timelines of one train launch (measurement build lib/var/trace.so, -DRM_BLOCK_TRACE:
# bash tools/build_variant.sh WT trace -DRM_BLOCK_TRACE) at the metric, C5, C5 on a 64x64 view (lone
# waves) and C2.
#   bash tools/gpu_block_trace.sh <tag> [names...]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-bt}
shift
ONLY="$*"
mkdir -p gpurun_out/bt_$TAG
export RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so
run() {
  name=$1; shift
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $name "* ]]; then return 0; fi
  timeout -k 10 200 python tools/block_trace.py --out gpurun_out/bt_$TAG/$name.npz "$@" > gpurun_out/bt_$TAG/$name.txt 2>&1
}
run metric --bins 20 && \
run c5 --spheres 4096 --march-steps 128 --views 1 --warm 2 --bins 20 && \
run c5s --width 64 --height 64 --spheres 4096 --march-steps 128 --views 1 --warm 2 --bins 8 && \
run c2 --width 256 --height 256 --spheres 64 --bins 20 && \
run c3 --march-steps 64 --bins 20
