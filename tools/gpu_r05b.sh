# Round-5 iteration b: the -m gpu suite, then the C2 step (cameras.json poses, the reference's
# targets) eager vs hipGraph, the metric with the graph, and the one-rank RCCL all-reduce floor.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
C2="--width 256 --height 256 --spheres 64 --march-steps 32 --views-per-gpu 10 --steps 40 --cameras tests/golden/cameras.json --targets files --cpu-baseline off"
timeout -k 10 200 python bench.py $C2 --graph off > $O/c2_eager.json 2> $O/c2_eager.err && \
timeout -k 10 200 python bench.py $C2 --graph on > $O/c2_graph.json 2> $O/c2_graph.err && \
timeout -k 10 200 python bench.py $C2 --graph off > $O/c2_eager2.json 2>> $O/c2_eager.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c2_graph -o run -- python3 bench.py $C2 --graph on --aux-steps 0 > $O/prof_c2_graph.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_c2_eager -o run -- python3 bench.py $C2 --graph off --aux-steps 0 > $O/prof_c2_eager.log 2>&1 && \
timeout -k 10 120 python tools/allreduce_probe.py > $O/allreduce.json 2> $O/allreduce.err && \
RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so timeout -k 10 200 python tools/block_trace.py --march-steps 128 \
  --views 1 --warm 2 --bins 20 --color-f16 --scene-json profiles/r05a_grown_scene_4096.json \
  --cameras tests/golden/cameras.json --out $O/bt_c5g.npz > $O/bt_c5g.txt 2>&1 && \
RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so timeout -k 10 200 python tools/block_trace.py --spheres 4096 \
  --march-steps 128 --views 1 --warm 2 --bins 20 --out $O/bt_c5.npz > $O/bt_c5.txt 2>&1 && \
timeout -k 10 200 python bench.py --cpu-baseline off --graph on > $O/metric_graph.json 2> $O/metric_graph.err && \
bash tools/gpu_iter.sh r05b tests
rc=$?
for f in c2_eager c2_graph c2_eager2 metric_graph; do
  python3 -c "import json,sys; d=json.load(open('$O/$f.json')); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], d['ms_per_step_median'], r['kernel_ms_per_step'], r['frac'])" $f
done
cat $O/allreduce.json
exit $rc
