# Split-march check: its GPU tests, the full GPU suite, then C5 / C4 / C3 / metric bench lines with
# the split march automatic (default), forced (RM_SPLIT=1) and off (RM_SPLIT=0).
set -o pipefail
mkdir -p gpurun_out/split
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 120 --timeout-method thread > gpurun_out/split/tests_split.log 2>&1 || { tail -40 gpurun_out/split/tests_split.log; exit 1; }
tail -2 gpurun_out/split/tests_split.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/split/tests_all.log 2>&1 || { tail -40 gpurun_out/split/tests_all.log; exit 1; }
tail -2 gpurun_out/split/tests_all.log
b() {  # name env args...
  name=$1; e=$2; shift 2
  env $e timeout -k 10 300 python bench.py --cpu-baseline off "$@" > gpurun_out/split/$name.json 2>gpurun_out/split/$name.err || return 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], (r['canonical'] or {}).get('frac'))" gpurun_out/split/$name.json $name
}
C5="--spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 6 --warmup 2"
C4="--width 1024 --height 1024 --spheres 1024 --march-steps 64 --views-per-gpu 4 --steps 4 --warmup 2"
b c5_auto RM_X=0 $C5 && b c5_off RM_SPLIT=0 $C5 && b c4_off RM_X=0 $C4 && b c4_on RM_SPLIT=1 $C4 && \
b c3_on RM_SPLIT=1 --march-steps 64 --steps 10 && b c3_off RM_X=0 --march-steps 64 --steps 10 && \
b m_on RM_SPLIT=1 --steps 20 && b m_off RM_X=0 --steps 20
