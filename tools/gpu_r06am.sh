#!/bin/bash
# Round 5: the multi-rank step with the optimizer's gradient-independent part in the sampled
# launch (rm_train_step_sampled_prepared; RM_OPT_PREPARE=0: the full optimizer after the
# all-reduce): parity tests, then rm_train --ranks 1 A B A B A B (per-stage times).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06am
mkdir -p $O/train_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_small.py \
  tests/test_gpu_host_ranks.py tests/test_gpu_host.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  for v in prepared full; do
    if [ $v = full ]; then export RM_OPT_PREPARE=0; else unset RM_OPT_PREPARE; fi
    timeout -k 10 120 burn_raymarching_amd/lib/rm_train train --ranks 1 --cameras tests/golden/cameras.json \
      --out $O/train_out --no-previews --log-every 700 > $O/train_${v}_$r.log 2>&1 || { tail $O/train_${v}_$r.log; exit 1; }
    echo "ranks1 $v $r: $(tail -1 $O/train_${v}_$r.log)"
  done
done | tee $O/ab.txt
