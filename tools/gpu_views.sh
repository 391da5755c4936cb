# bench.py at several --views-per-gpu values (same box).
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  timeout -k 10 200 python bench.py --cpu-baseline off --views-per-gpu $v > gpurun_out/views_$v.json 2>gpurun_out/views_$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/views_$v.json')); r=d['roofline']; print('views', $v, d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'])" || exit 1
done
