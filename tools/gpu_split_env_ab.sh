# C5 / C5 fixed-view with the split march automatic vs forced off (RM_SPLIT=0), same box.
set -o pipefail
mkdir -p gpurun_out/sab
for r in 1 2; do
  for sp in auto 0; do
    for c in c5 c5r1; do
      case $c in
        c5) args="--spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 4 --warmup 2" ;;
        c5r1) args="--spheres 4096 --march-steps 128 --views-per-gpu 1 --ring 1 --steps 4 --warmup 2" ;;
      esac
      if [ $sp = auto ]; then unset RM_SPLIT; else export RM_SPLIT=$sp; fi
      timeout -k 10 200 python bench.py --cpu-baseline off $args > gpurun_out/sab/${c}_${sp}_$r.json || exit 1
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], r['executed_frac'])" gpurun_out/sab/${c}_${sp}_$r.json $c split=$sp
    done
  done
done
