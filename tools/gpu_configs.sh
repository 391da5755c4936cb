# bench.py at the BASELINE.json configs on one MI355X (no CPU baseline), each as a bench line
# (replays on: executed and canonical fractions), a rocprofv3 --kernel-trace --stats run of the
# same arguments (replays off), and -- with PMC=1 -- the FETCH_SIZE / WRITE_SIZE / SQ passes of
# the same arguments, summarised into profiles/<tag>_pmc_{traffic,sq}.json under the config's
# bench key (what bench.py quotes as roofline.traffic / roofline.pmc for that workload).
#   C2 256x256 / 64 spheres / 32 steps / 10 views     C3 512x512 / 256 / 64 steps / 10 views
#   C4 1024x1024 / 1024 / 64 steps, 4 views (the per-GPU share of 32 views on 8 GPUs)
#   C4s the same 32 views on one GPU (strong-scaling N = 1 leg)
#   C5 512x512 / 4096 / 128 steps, 1 view (fp32 and fp16 colour)     k5: the metric at k = 5
#   ka: the metric with k annealed 5 -> 32 over the timed steps (train.rs:174)
#   C2cj / C3cj: C2 / C3 on the data/cameras.json poses (C2 on the reference's own target PNGs)
#   C5g: configs[4] on a model GROWN to 4096 spheres by prune_and_split (see grow below)
#   bash tools/gpu_configs.sh <tag> [names...]   (CALIB=<fetch_calibration.json>: calibrated traffic)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
shift
ONLY="$*"
O=gpurun_out/configs_$TAG
mkdir -p $O
run() {
  name=$1; key=$2; shift 2
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $name "* ]]; then return 0; fi
  timeout -k 10 300 python bench.py --cpu-baseline off "$@" > $O/$name.json 2> $O/$name.err || return $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$name -o run -- python3 bench.py --cpu-baseline off --aux-steps 0 "$@" > $O/prof_$name.log 2>&1 || return $?
  if [ -n "$PMC" ]; then
    local PB="python3 bench.py --cpu-baseline off --aux-steps 0 --steps 3 --warmup 1 $*"
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/$O/pmc_${name}_fetch -o run -- $PB > $O/pmc_$name.log 2>&1 && \
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/$O/pmc_${name}_write -o run -- $PB >> $O/pmc_$name.log 2>&1 && \
    timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_WAVES --kernel-trace --output-format csv -d $R/$O/pmc_${name}_sq1 -o run -- $PB >> $O/pmc_$name.log 2>&1 && \
    timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/$O/pmc_${name}_sq2 -o run -- $PB >> $O/pmc_$name.log 2>&1 && \
    RM_NO_EARLY_EXIT=1 timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_WAVES --kernel-trace --output-format csv -d $R/$O/pmc_${name}_sq1x -o run -- $PB >> $O/pmc_$name.log 2>&1 && \
    timeout -k 10 300 python3 bench.py --cpu-baseline off --steps 3 --warmup 1 "$@" > $O/${name}_pmcargs.json && \
    python3 tools/pmc_summary.py $O/pmc_${name}_fetch $O/pmc_${name}_write profiles/${TAG}_pmc_traffic.json $key auto $CALIB && \
    python3 tools/pmc_sq_summary.py profiles/${TAG}_pmc_sq.json $key $O/pmc_${name}_sq1 $O/pmc_${name}_sq2 $O/pmc_${name}_sq1x $O/${name}_pmcargs.json || return 1
  fi
  python3 -c "import json,sys; d=json.load(open('$O/$name.json')); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], r['executed_frac'], (r['canonical'] or {}).get('frac'), d['finite'])" "$name" || return 1
}
# configs[4] as stated: a model grown to 4096 spheres through prune_and_split (rm_train: every
# surviving sphere splits, capped at 4096; 11 stages x 100 steps at 512x512 / 128 steps / fp16
# colours on the generate.rs targets rendered at 512x512 from the data/cameras.json poses)
G=$O/grown
grow() {
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" C5g "* ]]; then return 0; fi
  mkdir -p $G/data
  timeout -k 10 120 burn_raymarching_amd/lib/rm_train generate --out $G/data --prefix "" --size 512x512 > $G/generate.log 2>&1 && \
  timeout -k 10 600 burn_raymarching_amd/lib/rm_train train --cameras $G/data/cameras.json --out $G --size 512x512 \
    --march-steps 128 --color-f16 --stages 11 --steps 100 --split-all --max-spheres 4096 \
    --log-every 100 --no-previews > $G/train.log 2>&1 || { tail $G/train.log; return 1; }
  GM=$(python3 -c "import json; print(len(json.load(open('$G/scene.json'))['radii']))")
  grep -E "Stage|Next N|num_spheres" $G/train.log
}
run C2 256x256_M64_S32_V10 --width 256 --height 256 --spheres 64 --march-steps 32 --views-per-gpu 10 --steps 20 && \
run C2cj 256x256_M64_S32_V10_cj --width 256 --height 256 --spheres 64 --march-steps 32 --views-per-gpu 10 --steps 20 \
  --cameras tests/golden/cameras.json --targets files && \
run C3cj 512x512_M256_S64_V10_cj --march-steps 64 --views-per-gpu 10 --steps 20 --cameras tests/golden/cameras.json \
  --targets dango && \
grow && \
run C5g 512x512_M${GM}_S128_V1_c16_cj_grown --march-steps 128 --views-per-gpu 1 --steps 6 --warmup 2 --color-dtype f16 \
  --cameras $G/data/cameras.json --targets files --scene-json $G/scene.json && \
run C3 512x512_M256_S64_V10 --march-steps 64 --views-per-gpu 10 --steps 20 && \
run C4 1024x1024_M1024_S64_V4 --width 1024 --height 1024 --spheres 1024 --march-steps 64 --views-per-gpu 4 --steps 6 --warmup 2 && \
run C4s 1024x1024_M1024_S64_V32 --width 1024 --height 1024 --spheres 1024 --march-steps 64 --global-views 32 --steps 3 --warmup 1 && \
run C5 512x512_M4096_S128_V1 --spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 6 --warmup 2 && \
run C5f16 512x512_M4096_S128_V1_c16 --spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 6 --warmup 2 --color-dtype f16 && \
run k5 512x512_M256_S32_V80_k5 --smooth-k 5 --steps 10 && \
run ka 512x512_M256_S32_V80_ka5 --anneal-k 5 --steps 10 && \
python3 tools/configs_summary.py $O profiles/${TAG}_configs.json && cp profiles/${TAG}_configs.json $O/ && \
{ [ -z "$PMC" ] || cp profiles/${TAG}_pmc_traffic.json profiles/${TAG}_pmc_sq.json $O/; }
