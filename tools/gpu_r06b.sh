# Round 5: the full -m gpu suite on the default build, then per-wave timelines of C5g and C5 as ONE
# launch (RM_SPLIT_CONT_STEPS=0: the whole march, post-march forward and backward of every block)
# -- where the split launches' wave time goes (tools/block_trace.py, measurement build).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
export RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so
RM_SPLIT_CONT_STEPS=0 timeout -k 10 200 python tools/block_trace.py --march-steps 128 --views 1 --warm 2 --bins 20 --color-f16 \
  --scene-json profiles/r05a_grown_scene_4096.json --cameras tests/golden/cameras.json > $O/bt_c5g_one.txt 2>&1 && \
RM_SPLIT_CONT_STEPS=0 timeout -k 10 200 python tools/block_trace.py --spheres 4096 --march-steps 128 --views 1 --warm 2 --bins 20 \
  > $O/bt_c5_one.txt 2>&1 && \
timeout -k 10 200 python tools/block_trace.py --views 80 --warm 2 --bins 20 > $O/bt_metric.txt 2>&1
rc=$?
grep -h 'launch span\|mean live\|summed wave time\|CU last-wave\|live waves' $O/bt_*.txt
exit $rc
