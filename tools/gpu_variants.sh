# Parity tests of a kernel-library variant (lib/var/<V>.so), then a same-box A/B against the
# default library and further variants. Stops after a test run that did not end normally.
#   V=pk OTHERS="lib:m32v3" CONFIGS="m c5 c2" bash tools/gpu_variants.sh
mkdir -p gpurun_out/var gpurun_out/ab
RM_LIB_PATH=burn_raymarching_amd/lib/var/$V.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_early_exit.py \
  tests/test_gpu_parity_configs.py tests/test_gpu_cameras.py tests/test_gpu_graph.py tests/test_golden_vectors.py \
  tests/test_gpu_growth.py > gpurun_out/var/tests_$V.log 2>&1
rc=$?
tail -3 gpurun_out/var/tests_$V.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stop"; exit $rc; fi
CONFIGS=${CONFIGS:-"m c5 c2"} ROUNDS=${ROUNDS:-2} bash tools/gpu_ab.sh default lib:$V $OTHERS
