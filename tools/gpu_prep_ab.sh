# rocprofv3 kernel-trace stats of the prep kernel for the default library and each variant.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in default "$@"; do
  if [ "$v" = default ]; then unset RM_LIB_PATH; else export RM_LIB_PATH=$R/burn_raymarching_amd/lib/var/$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pab_$v -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/pab_$v.log 2>&1 || exit $?
  echo "=== $v"; grep -h "prep\|finalize\|reduce" $(find gpurun_out/pab_$v -name "*kernel_stats.csv") | cut -d, -f1-5
done
