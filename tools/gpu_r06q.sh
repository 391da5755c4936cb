# Round 5: one N-rank step's launches on one GPU along the N = 1 trajectory: the default 80-view
# step as 80/N calls of N views... i.e. bench.py --views-per-call 80/N (each call its own launch,
# context and cost order, the full gradient into one Adam step): the per-launch train-kernel time
# is what one rank's launch takes at N ranks on the same scenes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
for v in 80 40 20 10; do
  timeout -k 10 300 python bench.py --cpu-baseline off --views-per-call $v > $O/vpc_$v.json 2> $O/vpc_$v.err || { tail -5 $O/vpc_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['kernel_ms'], r['launches_timed'], r['frac'], r['executed_frac'])" $O/vpc_$v.json $v
done
