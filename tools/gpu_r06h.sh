# Round 5: C5g's continuation launch per-wave trace saved for offline analysis.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
export RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so
A="--march-steps 128 --views 1 --warm 2 --bins 20 --color-f16 --scene-json profiles/r05a_grown_scene_4096.json --cameras tests/golden/cameras.json"
timeout -k 10 200 python tools/block_trace.py $A --out $O/c5g_cont.npz > $O/bt_c5g_cont.txt 2>&1 && \
RM_CONT_ORDER=0 timeout -k 10 200 python tools/block_trace.py $A --out $O/c5g_cont_arrival.npz > $O/bt_c5g_cont_arrival.txt 2>&1
