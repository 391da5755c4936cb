# Same-box A/B of variants on bench configurations, alternating A B A B over ROUNDS rounds.
# A variant is "default", an environment assignment list ("RM_SPLIT=0 RM_SMALL=1") or
# "lib:<name>" (the kernel library burn_raymarching_amd/lib/var/<name>.so, built with
# tools/build_variant.sh) or "args:<bench.py arguments>" (e.g. "args:--fused-adam off"). Configs: m (metric, strong default), m10 (10 views per GPU), m16 (the default's
# 80 views in calls of 16), ms / ms8 (the
# default's calls on 4 streams, 16 / 8 views per call), c2, c2cj (C2 on the cameras.json poses), c3,
# c4, c5, c5r1 (C5 on a fixed view), k5 (the metric at k = 5), c5s (C5 on a 64x64 view), c5g (configs[4] on the grown model).
#   CONFIGS="m c5" ROUNDS=2 bash tools/gpu_ab.sh default "RM_X=1" lib:trace
set -o pipefail
mkdir -p gpurun_out/ab
ROUNDS=${ROUNDS:-2}
CONFIGS=${CONFIGS:-"m c2 c5"}
for r in $(seq 1 $ROUNDS); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    unset RM_LIB_PATH
    envs=""
    extra=""
    case $v in
      default) ;;
      lib:*) export RM_LIB_PATH=burn_raymarching_amd/lib/var/${v#lib:}.so ;;
      args:*) extra=${v#args:} ;;
      *) envs=$v ;;
    esac
    for c in $CONFIGS; do
      case $c in
        m) args="--steps 10" ;;
        k5) args="--smooth-k 5 --steps 10" ;;
        m10) args="--views-per-gpu 10 --steps 20" ;;
        m16) args="--views-per-call 16 --steps 10" ;;
        ms) args="--streams 4 --steps 10" ;;
        ms8) args="--streams 4 --views-per-call 8 --steps 10" ;;
        c2) args="--width 256 --height 256 --spheres 64 --views-per-gpu 10 --steps 20" ;;
        c2cj) args="--width 256 --height 256 --spheres 64 --views-per-gpu 10 --steps 40 --cameras tests/golden/cameras.json --targets files" ;;
        c3) args="--march-steps 64 --views-per-gpu 10 --steps 10" ;;
        c4) args="--width 1024 --height 1024 --spheres 1024 --march-steps 64 --views-per-gpu 4 --steps 4 --warmup 2" ;;
        c5) args="--spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 4 --warmup 2" ;;
        c5r1) args="--spheres 4096 --march-steps 128 --views-per-gpu 1 --ring 1 --steps 4 --warmup 2" ;;
        c5s) args="--width 64 --height 64 --spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 4 --warmup 2" ;;
        c5g) args="--march-steps 128 --views-per-gpu 1 --steps 6 --warmup 2 --color-dtype f16 --cameras tests/golden/cameras.json --targets dango --scene-json profiles/r05a_grown_scene_4096.json" ;;
      esac
      env $envs timeout -k 10 200 python bench.py --cpu-baseline off $args $extra > gpurun_out/ab/${c}_v${i}_$r.json \
        2> gpurun_out/ab/${c}_v${i}_$r.err || { tail -5 gpurun_out/ab/${c}_v${i}_$r.err; exit 1; }
      # a variant whose executed work differs from the first variant's did other work (e.g. trained
      # differently): its time is not comparable, and the line says so
      python3 -c "
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
ref = json.load(open(sys.argv[4]))['roofline']['executed_frac']
flag = '' if abs(r['executed_frac'] - ref) <= 1e-4 else '  WORK DIFFERS FROM VARIANT 1'
print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], r['executed_frac'], flag)
" gpurun_out/ab/${c}_v${i}_$r.json $c "$v" gpurun_out/ab/${c}_v1_$r.json
    done
  done
done
