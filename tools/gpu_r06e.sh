# Round 5: the -m gpu suite with 32-ray split groups as the default.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
