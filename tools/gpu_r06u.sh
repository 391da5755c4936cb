# Round 5: per-wave timelines (measurement build) of C2 and C3cj (non-split, exact exits): how
# long the launch's tail is and how many waves are live in it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
export RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so
timeout -k 10 200 python tools/block_trace.py --width 256 --height 256 --spheres 64 --views 10 --warm 3 --bins 20 > $O/bt_c2.txt 2>&1 && \
timeout -k 10 200 python tools/block_trace.py --march-steps 64 --views 10 --warm 3 --bins 20 --cameras tests/golden/cameras.json > $O/bt_c3cj.txt 2>&1
rc=$?
grep -h 'launch span\|mean live\|summed wave time\|CU last-wave\|live waves' $O/bt_*.txt
exit $rc
