# Per-phase wave time (march / post-march forward / backward) of the metric's train launch and of
# C2 on the cameras.json poses, from the measurement build (tools/block_trace.py).
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
export RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so
timeout -k 10 300 python tools/block_trace.py --views 20 --warm 3 > $O/bt_metric.txt 2>&1 && \
timeout -k 10 300 python tools/block_trace.py --width 256 --height 256 --spheres 64 --views 10 \
  --cameras tests/golden/cameras.json --warm 5 > $O/bt_c2cj.txt 2>&1
rc=$?
grep -h 'summed wave time\|launch span\|live waves' $O/bt_*.txt
exit $rc
