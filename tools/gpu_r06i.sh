# Round 5: the split continuation kernel at 5 / 6 waves per SIMD (lib/var/cont5.so, cont6.so: more
# of the ~1,600 continuing 32-ray groups of C5g resident in the first round) against the default
# 4 on C5 / C5g; then the metric's per-rank slices of the strong-scaling default on one GPU
# (bench --global-views 40 / 20 / 10 over the 80-camera ring = one rank's step at N = 2 / 4 / 8).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
CONFIGS="c5 c5g" ROUNDS=2 bash tools/gpu_ab.sh default lib:cont5 lib:cont6 2>&1 | tee $O/ab.txt || exit 1
for v in 40 20 10; do
  timeout -k 10 300 python bench.py --cpu-baseline off --global-views $v --ring 80 > $O/slice_$v.json 2> $O/slice_$v.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])" $O/slice_$v.json $v
done
