# Same-box A/B of environment settings on one bench configuration, alternating, ROUNDS rounds:
#   ROUNDS=2 bash tools/gpu_env_ab.sh "<bench args>" "RM_X=0" "RM_VALU_ONLY=1" ...
set -o pipefail
mkdir -p gpurun_out/eab
ARGS=$1; shift
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    env $e timeout -k 10 200 python bench.py --cpu-baseline off $ARGS > gpurun_out/eab/v${i}_$r.json 2> gpurun_out/eab/v${i}_$r.err || { tail -5 gpurun_out/eab/v${i}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], d['ms_per_step_median'], r['kernel_ms_per_step'], r['frac'])" gpurun_out/eab/v${i}_$r.json "$e"
  done
done
