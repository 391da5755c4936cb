# Round 5: the -m gpu suite with 32-ray split groups and rm_train_step_camera_adam, then a same-box
# A/B of the fused optimizer (bench --fused-adam on / off) on C2cj, C2 and the metric.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
CONFIGS="c2cj c2 m" ROUNDS=2 bash tools/gpu_ab.sh default "args:--fused-adam off" 2>&1 | tee $O/ab.txt
