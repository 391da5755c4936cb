# Same-box A/B of kernel library variants (burn_raymarching_amd/lib/var/<name>.so, "default" =
# the in-tree build), alternating A B A B: the metric bench line, C2 and C5 (no CPU baseline).
#   bash tools/gpu_ab_libs.sh <name> <name> ...   (env ROUNDS=2, CONFIGS="m c2 c5")
set -o pipefail
mkdir -p gpurun_out/ab
ROUNDS=${ROUNDS:-2}
CONFIGS=${CONFIGS:-"m c2 c5"}
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    if [ $lib = default ]; then unset RM_LIB_PATH; else export RM_LIB_PATH=burn_raymarching_amd/lib/var/$lib.so; fi
    for c in $CONFIGS; do
      case $c in
        m) args="--steps 20" ;;
        c2) args="--width 256 --height 256 --spheres 64 --steps 20" ;;
        c5) args="--spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 4 --warmup 2" ;;
        c3) args="--march-steps 64 --steps 10" ;;
        c4) args="--width 1024 --height 1024 --spheres 1024 --march-steps 64 --views-per-gpu 4 --steps 4 --warmup 2" ;;
        c5r1) args="--spheres 4096 --march-steps 128 --views-per-gpu 1 --ring 1 --steps 4 --warmup 2" ;;
        c5w) args="--spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 4 --warmup 12" ;;
        c5s) args="--width 64 --height 64 --spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 4 --warmup 2" ;;
      esac
      timeout -k 10 200 python bench.py --cpu-baseline off $args > gpurun_out/ab/${c}_${lib}_$r.json || exit 1
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'])" gpurun_out/ab/${c}_${lib}_$r.json $c $lib
    done
  done
done
