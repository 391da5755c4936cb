set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
A="--width 256 --height 256 --spheres 64 --march-steps 32 --views-per-gpu 10 --steps 20 --cpu-baseline off --aux-steps 0"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/c2 -o run -- python3 bench.py $A > $O/c2.log 2>&1 && \
RM_REDUCE_FUSED=0 RM_PREP_ORIGIN=0 RM_OPT_SMALL=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/c2old -o run -- python3 bench.py $A > $O/c2old.log 2>&1 && \
python3 tools/step_timeline.py $O/c2 2 && python3 tools/step_timeline.py $O/c2old 2 && \
CONFIGS="c2" ROUNDS=2 bash tools/gpu_ab.sh default "RM_REDUCE_FUSED=0 RM_PREP_ORIGIN=0 RM_OPT_SMALL=0"
