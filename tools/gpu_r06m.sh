# Round 5: per-wave timelines (lib/var/trace.so) of one N = 8 rank's slice (10 views in one
# launch, the ring's spread order) against the 80-view launch, and the step's kernels by rocprofv3.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06m
mkdir -p $O
export RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so
timeout -k 10 200 python tools/block_trace.py --views 10 --warm 3 --bins 20 > $O/bt_10.txt 2>&1 && \
timeout -k 10 200 python tools/block_trace.py --views 80 --warm 3 --bins 20 > $O/bt_80.txt 2>&1 || exit 1
unset RM_LIB_PATH
grep -h 'launch span\|mean live\|summed wave time\|CU last-wave\|live waves' $O/bt_*.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof10 -o run -- python3 bench.py --cpu-baseline off --aux-steps 0 --global-views 10 --ring 80 --steps 20 > $O/prof10.log 2>&1
