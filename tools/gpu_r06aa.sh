#!/bin/bash
# Round 5: small-kernel final-block A/B: the working tree against lib/var/finhead.so (built from the
# previous revision by tools/build_variant.sh; r06aa: 32-bit clamped load offsets, r06ac: one load round
# at M = 9): the small-kernel tests, then rm_train (one process and --ranks 1) A B A B A B on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06aa}
mkdir -p $O/train_out
L=burn_raymarching_amd/lib
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_small.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cp $L/libraymarch_hip.so $O/new.so
for r in 1 2 3; do
  for v in new ${VAR:-finhead}; do
    if [ $v = new ]; then cp $O/new.so $L/libraymarch_hip.so; else cp $L/var/${VAR:-finhead}.so $L/libraymarch_hip.so; fi
    for mode in single ranks1; do
      extra=""; [ $mode = ranks1 ] && extra="--ranks 1"
      timeout -k 10 120 $L/rm_train train $extra --cameras tests/golden/cameras.json --out $O/train_out --no-previews \
        --log-every 700 > $O/train_${v}_${mode}_$r.log 2>&1 || { tail $O/train_${v}_${mode}_$r.log; exit 1; }
      echo "$mode $v $r: $(tail -1 $O/train_${v}_${mode}_$r.log)"
    done
  done
done | tee $O/ab.txt
cp $O/new.so $L/libraymarch_hip.so
