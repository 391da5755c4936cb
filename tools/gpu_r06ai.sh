#!/bin/bash
# Round 5: VALU / transcendental / MFMA wave-instructions of the metric's train kernel with the
# early exit off at M = 128, 256, 512 (same views and steps): the per-sphere slope and the
# per-step / per-ray intercept of the instruction count.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06ai
mkdir -p $O
for m in 128 256 512; do
  RM_NO_EARLY_EXIT=1 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_WAVES \
    --kernel-trace --output-format csv -d $R/$O/m$m -o run -- python3 bench.py --cpu-baseline off --aux-steps 0 \
    --steps 2 --warmup 1 --spheres $m --global-views 20 > $O/m$m.json 2> $O/m$m.err || { tail $O/m$m.err; exit 1; }
done
echo done
