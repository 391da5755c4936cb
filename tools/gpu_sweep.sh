#!/bin/bash
# Run bench.py once per argument set given as separate quoted arguments; print value, kernel ms,
# roofline frac and the early-exit stats of each.   gpurun -- 'bash tools/gpu_sweep.sh "--views-per-gpu 4" ...'
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  env $RM_ENV timeout -k 10 200 python bench.py --cpu-baseline off $a > gpurun_out/sweep_$i.json 2>gpurun_out/sweep_$i.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/sweep_$i.json')); r=d['roofline']; print(sys.argv[1], d['value'], r['kernel_ms'], r['frac'], d.get('early_exit'))" "$a"
done
