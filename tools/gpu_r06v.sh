# Round 5: the metric's per-wave timeline saved for offline analysis (dead waves' wait at the
# hand-off barrier), and C2's.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
export RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so
timeout -k 10 200 python tools/block_trace.py --views 16 --warm 3 --bins 20 --out $O/metric16.npz > $O/bt_metric16.txt 2>&1 && \
timeout -k 10 200 python tools/block_trace.py --width 256 --height 256 --spheres 64 --views 10 --warm 3 --bins 20 --out $O/c2.npz > $O/bt_c2.txt 2>&1
