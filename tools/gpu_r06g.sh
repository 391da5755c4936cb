# Round 5: the split continuation's class-ordered block lists (the blocks with the most rays still
# moving first) -- split / growth / early-exit tests, same-box A/B against arrival order
# (RM_CONT_ORDER=0) on C5 and C5g, and the continuation's per-wave timeline.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_growth.py tests/test_gpu_early_exit.py \
  tests/test_gpu_parity_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
CONFIGS="c5 c5g" ROUNDS=2 bash tools/gpu_ab.sh default "RM_CONT_ORDER=0" 2>&1 | tee $O/ab.txt || exit 1
export RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so
A="--march-steps 128 --views 1 --warm 2 --bins 20 --color-f16 --scene-json profiles/r05a_grown_scene_4096.json --cameras tests/golden/cameras.json"
timeout -k 10 200 python tools/block_trace.py $A > $O/bt_c5g_cont.txt 2>&1
rc=$?
grep -h 'launch span\|mean live\|CU last-wave' $O/bt_*.txt
exit $rc
