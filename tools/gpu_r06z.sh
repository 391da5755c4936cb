#!/bin/bash
# Round 5: the data-parallel rank's sampled step in one launch (rm_train_step_sampled): parity
# tests, then `rm_train train --ranks 1` (the RCCL path: sampled step, all-reduce, optimizer)
# timed against the two-call form (RM_FUSED_ITER=0) A B A B A B on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O/train_out
L=burn_raymarching_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_small.py \
  tests/test_gpu_host_ranks.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for v in one two; do
    if [ $v = one ]; then unset RM_FUSED_ITER; else export RM_FUSED_ITER=0; fi
    timeout -k 10 120 $L/rm_train train --ranks 1 --cameras tests/golden/cameras.json --out $O/train_out \
      --no-previews --log-every 700 > $O/train_${v}_$r.log 2>&1 || { tail $O/train_${v}_$r.log; exit 1; }
    echo "ranks1 $v $r: $(tail -1 $O/train_${v}_$r.log)"
  done
done | tee $O/ab.txt
unset RM_FUSED_ITER
timeout -k 10 120 $L/rm_train train --cameras tests/golden/cameras.json --out $O/train_out --no-previews \
  --log-every 700 > $O/train_single.log 2>&1 || { tail $O/train_single.log; exit 1; }
echo "single: $(tail -1 $O/train_single.log)" | tee -a $O/ab.txt
