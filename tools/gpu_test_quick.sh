# GPU tests (stop at the first failure), then the quick bench + timeline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_quick.sh "${1:-q}"
