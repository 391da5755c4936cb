# The 32x32x16 march variant (-DRM_MFMA32=1, lib/var/m32.so): its parity tests, then a same-box
# A/B against the default library. Stops after a test run that did not end normally.
mkdir -p gpurun_out/m32 gpurun_out/ab
RM_LIB_PATH=burn_raymarching_amd/lib/var/m32.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_early_exit.py \
  tests/test_gpu_parity_configs.py tests/test_gpu_cameras.py tests/test_gpu_graph.py tests/test_golden_vectors.py \
  > gpurun_out/m32/tests.log 2>&1
rc=$?
tail -3 gpurun_out/m32/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stop"; exit $rc; fi
CONFIGS="m c2 c5" ROUNDS=2 bash tools/gpu_ab.sh default lib:m32
