#!/bin/bash
# GPU tests, then bench.py with the defaults and with each extra environment given as an
# argument (e.g. RM_VALU_ONLY=1, RM_LIB_PATH=burn_raymarching_amd/lib/var/<name>.so); prints
# value, kernel ms, roofline frac, executed frac, exited-wave share. Every GPU step has its own
# time limit; a failing step ends the script.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -le 1 ] || exit $rc
i=0
for e in "" "$@"; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --cpu-baseline off > gpurun_out/ab_$i.json 2>gpurun_out/ab_$i.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$i.json')); r=d['roofline']; print(sys.argv[1] or 'default', d['value'], r['kernel_ms'], r['frac'], r['executed_frac'], d['early_exit']['exited_frac'])" "$e"
done
exit $rc
