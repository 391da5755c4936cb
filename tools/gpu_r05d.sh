# Round-5 iteration d: the cost-order padding fix -- order probe, C2cj and the metric, the GPU tests
# that touch the dispatch order and the graph, then C3cj.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
C2="--width 256 --height 256 --spheres 64 --march-steps 32 --views-per-gpu 10 --steps 40 --cameras tests/golden/cameras.json --targets files --cpu-baseline off"
timeout -k 10 200 python tools/order_probe.py > $O/order_probe.json 2> $O/order_probe.err && \
timeout -k 10 200 python bench.py $C2 > $O/c2cj.json 2> $O/c2cj.err && \
timeout -k 10 300 python bench.py --cpu-baseline off > $O/metric.json 2> $O/metric.err && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_block_order.py tests/test_gpu_graph.py tests/test_gpu_parity_configs.py \
  tests/test_gpu_split.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 200 python bench.py --march-steps 64 --views-per-gpu 10 --steps 20 --cameras tests/golden/cameras.json --targets dango --cpu-baseline off > $O/c3cj.json 2> $O/c3cj.err
rc=$?
tail -2 $O/tests.log
python3 -c "
import json
d=json.load(open('$O/order_probe.json'))
print('cost', [(r['kernel_ms'], r['turn']) for r in d['cost']])
print('static', [r['kernel_ms'] for r in d['static']])"
for f in c2cj metric c3cj; do
  python3 -c "import json,sys; d=json.load(open('$O/$f.json')); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], d['ms_per_step_median'], r['kernel_ms_per_step'], r['frac'], d.get('value_exit_off'))" $f
done
exit $rc
