# Round 5: the cost order per view set (12 slots): the order / graph / split / camera tests, then a
# same-box A/B against the single-slot order (lib:preslot) on C5, C5g (one rotating view per step),
# the metric and C2cj (fixed views).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_block_order.py tests/test_gpu_graph.py tests/test_gpu_parity_configs.py tests/test_gpu_split.py tests/test_gpu_cameras.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
CONFIGS="c5 c5g m c2cj" ROUNDS=2 bash tools/gpu_ab.sh lib:preslot default 2>&1 | tee $O/ab.txt
