# Round 5: every rank's share of the N = 2 / 4 / 8 strong-scaling step run alone on one GPU
# (bench.py --as-rank R/N: the rank's fixed views of the 80, the global ray count, no all-reduce).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
for n in 8 4 2; do
  for r in $(seq 0 $((n - 1))); do
    timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 --warmup 3 --ring 80 --as-rank $r/$n > $O/rank_${r}_of_$n.json 2> $O/rank_${r}_of_$n.err \
      || { tail -5 $O/rank_${r}_of_$n.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], r['executed_frac'])" $O/rank_${r}_of_$n.json "$r/$n"
  done
done
