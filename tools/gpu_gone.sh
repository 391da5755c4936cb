set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_gone.log 2>&1 || { tail -40 gpurun_out/tests_gone.log; exit 1; }
tail -2 gpurun_out/tests_gone.log
ROUNDS=1 CONFIGS="m c2 c3 c4 c5" timeout -k 10 900 bash tools/gpu_ab_libs.sh head0 default > gpurun_out/ab_gone.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ab_gone.log
exit $rc
