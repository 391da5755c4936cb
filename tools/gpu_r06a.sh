# Round 5, first iteration: split blocks of 32 / 16 rays (RM_SPLIT_RAYS, lib/var/sr32.so, sr16.so)
# -- their parity tests, then a same-box A/B against the 64-ray default on C5 and C5g.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
T="tests/test_gpu_split.py tests/test_gpu_growth.py tests/test_gpu_parity_configs.py::test_color_f16_config4"
for v in sr32 sr16; do
  RM_LIB_PATH=burn_raymarching_amd/lib/var/$v.so timeout -k 10 400 python -u -m pytest $T -m gpu -x -q \
    --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/tests_$v.log; exit 1; }
  tail -1 $O/tests_$v.log
done
CONFIGS="c5 c5g" ROUNDS=2 bash tools/gpu_ab.sh default lib:sr32 lib:sr16 2>&1 | tee $O/ab.txt
