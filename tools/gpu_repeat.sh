# Run-to-run spread of the default bench line on one box: the same `python bench.py` three times.
set -o pipefail
O=gpurun_out/repeat
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --cpu-baseline off > $O/bench_$i.json 2> $O/bench_$i.err || exit $?
  python3 -c "
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
print(sys.argv[2], d['value'], d['value_median'], d['value_exit_off'], d['ms_per_step'], r['kernel_ms'], r['frac'])
" $O/bench_$i.json $i
done
