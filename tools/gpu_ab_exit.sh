#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --cpu-baseline off > gpurun_out/ab_exit.json 2>/dev/null
RM_NO_EARLY_EXIT=1 timeout -k 10 200 python bench.py --cpu-baseline off > gpurun_out/ab_noexit.json 2>/dev/null
for f in ab_exit ab_noexit; do python -c "import json; d=json.load(open('gpurun_out/$f.json')); r=d['roofline']; print('$f', d['value'], r['kernel_ms'], r['frac'], r['executed_frac'], d['early_exit'])"; done
exit $rc
