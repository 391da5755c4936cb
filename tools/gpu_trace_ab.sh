# Per-step kernel timeline for the default library and for each lib/var/<name>.so given.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in default "$@"; do
  if [ "$v" = default ]; then unset RM_LIB_PATH; else export RM_LIB_PATH=$R/burn_raymarching_amd/lib/var/$v.so; fi
  echo "=== $v"
  timeout -k 10 200 python bench.py --cpu-baseline off > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); r=d['roofline']; print('BENCH', d['value'], d['ms_per_step'], r['kernel_ms'])" || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace_ab_$v -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/trace_ab_$v.log 2>&1 || exit $?
  python3 tools/step_timeline.py gpurun_out/trace_ab_$v 1 || exit 1
done
