#!/bin/bash
# Round 5: the small kernel's phase timeline (measurement build) at M = 7 and 9 after the
# final-block load addressing change.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ab
mkdir -p $O
for m in 7 9; do
  RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so timeout -k 10 200 python tools/small_trace.py --spheres $m \
    > $O/small_trace_m$m.json 2> $O/small_trace_m$m.err || { tail $O/small_trace_m$m.err; exit 1; }
done
cat $O/small_trace_m7.json
