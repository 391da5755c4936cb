# Round 5: continuation lists -- the split tests (four continuations bit-identical), then C5 / C5g
# with the default (48, 96) against three and four continuations, three rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
CONFIGS="c5 c5g" ROUNDS=3 bash tools/gpu_ab.sh default "RM_SPLIT_CONT_LIST=48,80,112" "RM_SPLIT_CONT_LIST=48,88,112" "RM_SPLIT_CONT_LIST=40,64,88,112" 2>&1 | tee $O/ab.txt
