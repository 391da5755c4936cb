#!/bin/bash
# GPU tests, then (unless the tests crashed or timed out) one default bench line.
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --cpu-baseline off > gpurun_out/bench_now.json 2> gpurun_out/bench_now.err
  rb=$?
  python -c "import json; d=json.load(open('gpurun_out/bench_now.json')); r=d['roofline']; print('BENCH', d['value'], r['kernel_ms'], r['frac'])" || tail -5 gpurun_out/bench_now.err
  exit $(( rc > rb ? rc : rb ))
fi
exit $rc
