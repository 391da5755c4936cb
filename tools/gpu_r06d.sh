# Round 5: the -m gpu suite with the centre-distance clamp proof (rho_lb), then same-box A/B:
# HEAD before it (lib/var/r06c.so) vs the working tree on the metric, k = 5, C2cj and C5g, and
# 32-ray split groups (lib/var/sr32.so) on C5 / C5g; a per-wave trace of the metric at k = 5.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
CONFIGS="m k5 c2cj c5g" ROUNDS=2 bash tools/gpu_ab.sh lib:r06c default 2>&1 | tee $O/ab.txt || exit 1
CONFIGS="c5 c5g" ROUNDS=2 bash tools/gpu_ab.sh default lib:sr32 2>&1 | tee $O/ab_sr32.txt || exit 1
RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so timeout -k 10 200 python tools/block_trace.py --views 80 --warm 2 \
  --bins 20 --smooth-k 5 > $O/bt_k5.txt 2>&1
rc=$?
grep -h 'launch span\|mean live\|summed wave time\|by path' $O/bt_*.txt
exit $rc
