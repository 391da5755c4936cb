# bench.py at the BASELINE.json configs on one MI355X (per-GPU shares; no CPU baseline), each
# as a bench line (replays on: executed and canonical fractions) plus a rocprofv3 kernel-trace
# --stats run of the same arguments (replays off, so the stats cover the bench's own steps):
#   C2 256x256 / 64 spheres / 32 steps / 10 views      C3 512x512 / 256 / 64 steps / 10 views
#   C4 1024x1024 / 1024 / 64 steps, 4 views (the per-GPU share of 32 views on 8 GPUs)
#   C5 512x512 / 4096 / 128 steps, 1 view (fp32 and fp16 colour)   k = 5 at the metric config
#   bash tools/gpu_configs2.sh <tag> [names...]
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r02}
shift
ONLY="$*"
mkdir -p gpurun_out/configs_$TAG
run() {
  name=$1; shift
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $name "* ]]; then return 0; fi
  timeout -k 10 300 python bench.py --cpu-baseline off "$@" > gpurun_out/configs_$TAG/$name.json 2> gpurun_out/configs_$TAG/$name.err || return $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/configs_$TAG/prof_$name -o run -- python3 bench.py --cpu-baseline off --aux-steps 0 "$@" > gpurun_out/configs_$TAG/prof_$name.log 2>&1 || return $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/configs_$TAG/$name.json')); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], r['executed_frac'], (r['canonical'] or {}).get('frac'), d['finite'])" "$name" || return 1
}
run C2 --width 256 --height 256 --spheres 64 --march-steps 32 --steps 20 && \
run C3 --march-steps 64 --steps 20 && \
run C4 --width 1024 --height 1024 --spheres 1024 --march-steps 64 --views-per-gpu 4 --steps 6 --warmup 2 && \
run C5 --spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 6 --warmup 2 && \
run C5f16 --spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 6 --warmup 2 --color-dtype f16 && \
run k5 --smooth-k 5 --steps 20 && \
python3 tools/configs_summary.py gpurun_out/configs_$TAG profiles/${TAG}_configs.json && cp profiles/${TAG}_configs.json gpurun_out/
