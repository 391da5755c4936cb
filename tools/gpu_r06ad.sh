#!/bin/bash
# Round 5: rm_train's kernel time per step against its step time (one process; rocprofv3 kernel
# trace), to split the 19-20 us step into the kernel and the gap between launches.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ad
mkdir -p $O/train_out
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run \
  -- burn_raymarching_amd/lib/rm_train train --cameras tests/golden/cameras.json --out $O/train_out --no-previews \
  --log-every 700 > $O/train.log 2>&1 || { tail $O/train.log; exit 1; }
tail -1 $O/train.log
find $O/prof -name "*kernel_stats.csv" -exec cat {} \;
