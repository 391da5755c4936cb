#!/bin/bash
# Round 5: rocprofv3 kernel stats of rm_train --ranks 1 (the multi-rank step: sampled launch,
# RCCL all-reduce, optimizer) next to the one-process schedule, after the first-stage fix.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06al
mkdir -p $O/train_out
for mode in single; do  # (--ranks forks its rank processes: the profiler sees none of their kernels)
  extra=""; [ $mode = ranks1 ] && extra="--ranks 1"
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$mode -o run \
    -- burn_raymarching_amd/lib/rm_train train $extra --cameras tests/golden/cameras.json --out $O/train_out \
    --no-previews --log-every 700 > $O/train_$mode.log 2>&1 || { tail $O/train_$mode.log; exit 1; }
  echo "== $mode: $(tail -1 $O/train_$mode.log)"
  find $O/prof_$mode -name "*kernel_stats.csv" -exec head -6 {} \;
done
