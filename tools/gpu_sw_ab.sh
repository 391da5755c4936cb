# Split-march waves per block: 4 (default build) vs 2 (lib/var/sw2.so): split tests on the sw2 build,
# then C5 (automatic split) and C4 (split forced) bench lines with each build.
set -o pipefail
mkdir -p gpurun_out/sw
RM_LIB_PATH=burn_raymarching_amd/lib/var/sw2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_origin.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sw/tests_sw2.log 2>&1 || { tail -30 gpurun_out/sw/tests_sw2.log; exit 1; }
tail -1 gpurun_out/sw/tests_sw2.log
b() {  # name lib env args...
  name=$1; lib=$2; e=$3; shift 3
  if [ $lib = default ]; then L=burn_raymarching_amd/lib/libraymarch_hip.so; else L=burn_raymarching_amd/lib/var/$lib.so; fi
  env RM_LIB_PATH=$L $e timeout -k 10 300 python bench.py --cpu-baseline off "$@" > gpurun_out/sw/$name.json 2>gpurun_out/sw/$name.err || return 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], (r['canonical'] or {}).get('frac'))" gpurun_out/sw/$name.json $name
}
C5="--spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 6 --warmup 2"
C4="--width 1024 --height 1024 --spheres 1024 --march-steps 64 --views-per-gpu 4 --steps 4 --warmup 2"
b c5_sw4 default RM_X=0 $C5 && b c5_sw2 sw2 RM_X=0 $C5 && b c5_sw4b default RM_X=0 $C5 && b c5_sw2b sw2 RM_X=0 $C5 && \
b c4_sw2 sw2 RM_SPLIT=1 $C4 && b c4_off default RM_X=0 $C4 && \
b c3_sw2 sw2 RM_SPLIT=1 --march-steps 64 --steps 10 && b m_sw2 sw2 RM_SPLIT=1 --steps 20
