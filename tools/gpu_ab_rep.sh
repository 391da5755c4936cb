#!/bin/bash
# Alternating repeated A/B of bench.py (no tests): default vs each RM_LIB_PATH/env given, R rounds.
#   bash tools/gpu_ab_rep.sh R "ENV=..." ...
mkdir -p gpurun_out
R=$1; shift
for r in $(seq 1 $R); do
  i=0
  for e in "NONE=1" "$@"; do
    i=$((i+1))
    env $e timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 > gpurun_out/abr_$i.json 2>gpurun_out/abr_$i.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/abr_$i.json')); print(sys.argv[1], d['value'], d['roofline']['kernel_ms'])" "$e"
  done
done
