#!/bin/bash
# Round 5: the reduction's pass 1 with the visited rows' record offsets precomputed in its
# compaction (no 64-bit multiplies per load) against HEAD (lib/var/redhead.so): the fusion and
# reduction tests, then C2 / C2cj A B over three rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ae
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fusion.py \
  tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
CONFIGS="c2 c2cj" ROUNDS=3 timeout -k 10 900 bash tools/gpu_ab.sh default lib:redhead 2>&1 | tee $O/ab.txt
