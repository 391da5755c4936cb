# Round 5: per-wave timelines of C5g with 32-ray split groups -- the continuation launch (default)
# and the whole march as one launch -- and of C5's continuation (measurement build).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
export RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so
A="--march-steps 128 --views 1 --warm 2 --bins 20 --color-f16 --scene-json profiles/r05a_grown_scene_4096.json --cameras tests/golden/cameras.json"
timeout -k 10 200 python tools/block_trace.py $A > $O/bt_c5g_cont.txt 2>&1 && \
RM_SPLIT_CONT_STEPS=0 timeout -k 10 200 python tools/block_trace.py $A > $O/bt_c5g_one.txt 2>&1 && \
timeout -k 10 200 python tools/block_trace.py --spheres 4096 --march-steps 128 --views 1 --warm 2 --bins 20 > $O/bt_c5_cont.txt 2>&1
rc=$?
grep -h 'launch span\|mean live\|summed wave time\|CU last-wave\|live waves' $O/bt_*.txt
exit $rc
