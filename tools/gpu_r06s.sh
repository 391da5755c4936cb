# Round 5: the second continuation by default -- the split / growth / fp16 tests, then C5, C5f16
# and C5g (grown) with PMC into profiles/r06_*.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_growth.py tests/test_gpu_parity_configs.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PMC=1 bash tools/gpu_configs.sh r06 C5 C5f16 C5g
