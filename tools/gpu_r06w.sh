# Round 5: dead waves end at the hand-off (RM_DEAD_EARLY) -- the -m gpu suite, then a same-box A/B
# against the waiting form (lib:pre_dead) on the metric, C2cj, C3cj and k = 5.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
CONFIGS="m c2cj c3 k5" ROUNDS=2 bash tools/gpu_ab.sh lib:pre_dead default 2>&1 | tee $O/ab.txt
