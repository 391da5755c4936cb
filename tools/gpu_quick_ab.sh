# GPU tests (fast subset or all), then an A/B of the in-tree library against lib/var variants.
#   K="origin" CONFIGS="m c2" bash tools/gpu_quick_ab.sh <variant>...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/tests_qab.log 2>&1 || { tail -40 gpurun_out/tests_qab.log; exit 1; }
tail -2 gpurun_out/tests_qab.log
ROUNDS=${ROUNDS:-1} CONFIGS="${CONFIGS:-m c2 c5}" timeout -k 10 900 bash tools/gpu_ab_libs.sh "$@" > gpurun_out/ab_q.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ab_q.log
exit $rc
