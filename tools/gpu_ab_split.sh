#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --cpu-baseline off > gpurun_out/ab_split.json 2>/dev/null
RM_MARCH_FUSED=1 timeout -k 10 200 python bench.py --cpu-baseline off > gpurun_out/ab_fused.json 2>/dev/null
for f in ab_split ab_fused; do python -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['roofline']['kernel_ms'])"; done
timeout -k 10 200 python tools/bench_parts.py
exit $rc
