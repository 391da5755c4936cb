# bench.py at the other BASELINE.json configs on one MI355X (per-GPU shares; no CPU baseline):
#   C2 256x256 / 64 spheres / 32 steps / 10 views      C3 512x512 / 256 / 64 steps / 10 views
#   C4 1024x1024 / 1024 / 64 steps, 4 views (the per-GPU share of 32 views on 8 GPUs)
#   C5 512x512 / 4096 / 128 steps, 1 view              k = 5 at the metric config
set -o pipefail
mkdir -p gpurun_out
run() {
  name=$1; shift
  timeout -k 10 300 python bench.py --cpu-baseline off "$@" > gpurun_out/cfg_$name.json 2> gpurun_out/cfg_$name.err || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/cfg_$name.json')); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], r['executed_frac'], d['finite'])" "$name" || exit 1
}
run C2 --width 256 --height 256 --spheres 64 --march-steps 32 --steps 20 && \
run C3 --march-steps 64 --steps 10 && \
run C4 --width 1024 --height 1024 --spheres 1024 --march-steps 64 --views-per-gpu 4 --steps 5 --warmup 2 && \
run C5 --spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 5 --warmup 2 && \
run k5 --smooth-k 5 --steps 10
