# Round 5: the backward sweeps' ray counters (rm_stats seeded_rays / seeded_rays_a): the early-exit
# tests, then the metric, k = 5 and the k-annealed line with the executed work counted by them.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_early_exit.py tests/test_gpu_bench.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in m k5 ka; do
  case $c in
    m) a="--steps 10" ;;
    k5) a="--smooth-k 5 --steps 10" ;;
    ka) a="--anneal-k 5 --steps 10" ;;
  esac
  timeout -k 10 200 python bench.py --cpu-baseline off $a > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
  python3 -c "
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']; c = r['canonical']
print(sys.argv[2], d['value'], d['ms_per_step'], r['frac'], r['executed_frac'], r['backward_rays_frac'], c['frac'], c['frac_backward_all_rays'])
" $O/$c.json $c
done
