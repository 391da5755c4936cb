#!/bin/bash
# Round 5: rm_train's final-block record sums two columns at a time (RM_SMALL_FIN_PAIRS=1) against
# one at a time (lib/var/finold.so, RM_SMALL_FIN_PAIRS=0): small-kernel parity tests, then the
# training loop timed A B A B A B on one box (the variant swapped in for libraymarch_hip.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06y
mkdir -p $O/train_out
L=burn_raymarching_amd/lib
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_small.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cp $L/libraymarch_hip.so $O/new.so
for r in 1 2 3; do
  for v in new finold; do
    if [ $v = new ]; then cp $O/new.so $L/libraymarch_hip.so; else cp $L/var/finold.so $L/libraymarch_hip.so; fi
    timeout -k 10 120 $L/rm_train train --cameras tests/golden/cameras.json --out $O/train_out --no-previews \
      --log-every 700 > $O/train_${v}_$r.log 2>&1 || { tail $O/train_${v}_$r.log; exit 1; }
    echo "$v $r: $(tail -1 $O/train_${v}_$r.log)"
  done
done | tee $O/ab.txt
cp $O/new.so $L/libraymarch_hip.so
