#!/bin/bash
# One parametrised launcher for the GPU-box steps (replaces the round-5 one-off gpu_r06*.sh
# scripts; every invocation is logged in tools/gpu_log.md). Every GPU step runs under its own
# time limit and the steps are chained with &&: the script stops at the first failure.
#
#   bash tools/gpu.sh tests  <tag>                 -m gpu suite + smoke             -> gpurun_out/<tag>/
#   bash tools/gpu.sh traj   <tag> [variants...]   the pinned rm_train trajectory (one process and
#                                                  --ranks 1) for the tree's library and for each
#                                                  lib/var/<variant>.so (tools/build_variant.sh)
#   bash tools/gpu.sh trainab <tag> <variant> [n]  rm_train timing A/B: tree vs lib/var/<variant>.so, n rounds
#   bash tools/gpu.sh benchab <tag> <variant> <n> <config> [bench args...]
#                                                  bench.py A/B (same box, alternating): tree vs variant
#   bash tools/gpu.sh round  <tag> [bench args]    tools/gpu_round.sh (tests, PMC, bench, rocprof)
#   bash tools/gpu.sh configs <tag> [names]        tools/gpu_configs.sh (PMC=1 for the counters)
set -o pipefail
export TMPDIR=/tmp
RECIPE=$1; TAG=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
L=burn_raymarching_amd/lib
cp $L/libraymarch_hip.so $O/tree.so
use() {  # use <variant|tree>: put that kernel library where rm_train / the tests load it
  if [ "$1" = tree ]; then cp $O/tree.so $L/libraymarch_hip.so; else cp $L/var/$1.so $L/libraymarch_hip.so; fi
}
trap 'cp $O/tree.so $L/libraymarch_hip.so' EXIT
case $RECIPE in
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && \
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; tail -3 $O/tests.log; tail -1 $O/smoke.log; exit $rc ;;
traj)
  for v in tree "$@"; do
    use $v && timeout -k 10 300 python -u tools/pin_trajectory.py --write $O/traj_$v.json > $O/traj_$v.log 2>&1 \
      || { echo "traj $v failed"; tail -20 $O/traj_$v.log; exit 1; }
    echo "$v: $(tail -3 $O/traj_$v.log | head -2 | tr '\n' ' ')"
  done ;;
trainab)
  V=$1; N=${2:-3}
  for r in $(seq $N); do
    for v in tree $V; do
      use $v || exit 1
      for mode in single ranks1; do
        extra=""; [ $mode = ranks1 ] && extra="--ranks 1"
        timeout -k 10 120 $L/rm_train train $extra --cameras tests/golden/cameras.json --out $O/train_out --no-previews \
          --log-every 700 > $O/train_${v}_${mode}_$r.log 2>&1 || { tail $O/train_${v}_${mode}_$r.log; exit 1; }
        echo "$mode $v $r: $(tail -1 $O/train_${v}_${mode}_$r.log)"
      done
    done
  done | tee $O/ab.txt ;;
benchab)
  V=$1; N=$2; C=$3; shift 3
  for r in $(seq $N); do
    for v in tree $V; do
      use $v || exit 1
      timeout -k 10 300 python bench.py --cpu-baseline off "$@" > $O/${C}_${v}_$r.json 2> $O/${C}_${v}_$r.err \
        || { tail $O/${C}_${v}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], r['executed_frac'])" \
        $O/${C}_${v}_$r.json $C $v
    done
  done | tee -a $O/ab.txt ;;
envab)
  # envab <tag> <n> <config> <ENV=V|-> ... -- <bench args>: bench.py per environment setting
  # (- = none), alternating, n rounds. {G} in the bench args = gpurun_out/<tag>/grown (see grow)
  N=$1; C=$2; shift 2; ENVS=()
  while [ "$1" != "--" ]; do ENVS+=("$1"); shift; done; shift
  ARGS=$(echo "$@" | sed "s#{G}#$O/grown#g")
  for r in $(seq $N); do
    for e in "${ENVS[@]}"; do
      tagv=$(echo "$e" | tr -c 'A-Za-z0-9_\n' '_')
      if [ "$e" = - ]; then e="RM_NOOP=1"; fi
      env $e timeout -k 10 300 python bench.py --cpu-baseline off $ARGS > $O/${C}_${tagv}_$r.json 2> $O/${C}_${tagv}_$r.err \
        || { tail $O/${C}_${tagv}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], r['executed_frac'])" \
        $O/${C}_${tagv}_$r.json $C "$e"
    done
  done | tee -a $O/ab.txt ;;
grow)
  # configs[4]'s grown model (tools/gpu_configs.sh grow): generate.rs targets at 512x512 on the
  # cameras.json poses, then 11 x 100 steps of prune_and_split growth to 4096 spheres, fp16 colours
  G=$O/grown; mkdir -p $G/data
  timeout -k 10 120 $L/rm_train generate --out $G/data --prefix "" --size 512x512 > $G/generate.log 2>&1 && \
  timeout -k 10 600 $L/rm_train train --cameras $G/data/cameras.json --out $G --size 512x512 \
    --march-steps 128 --color-f16 --stages 11 --steps 100 --split-all --max-spheres 4096 \
    --log-every 100 --no-previews > $G/train.log 2>&1 || { tail $G/train.log; exit 1; }
  grep -E "Next N|num_spheres" $G/train.log | tail -3 ;;
round) bash tools/gpu_round.sh $TAG "$@" ;;
configs) bash tools/gpu_configs.sh $TAG "$@" ;;
*) echo "unknown recipe $RECIPE"; exit 2 ;;
esac
