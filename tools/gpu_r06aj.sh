#!/bin/bash
# Round 5: rm_train's timed stage loops hold ~2-3 ms per stage beyond the kernels' GPU span
# (r06ad trace). Per stage: how long the host takes to issue the 700 steps and how long the
# stream then takes to drain (RMH_STAGE_TIMES=1), one process and --ranks 1.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06aj
mkdir -p $O/train_out
export RMH_STAGE_TIMES=1
for mode in single ranks1; do
  extra=""; [ $mode = ranks1 ] && extra="--ranks 1"
  timeout -k 10 120 burn_raymarching_amd/lib/rm_train train $extra --cameras tests/golden/cameras.json --out $O/train_out \
    --no-previews --log-every 700 > $O/train_$mode.log 2>&1 || { tail $O/train_$mode.log; exit 1; }
  echo "== $mode"; grep -E "^stage|num_spheres" $O/train_$mode.log
done | tee $O/stage_times.txt
