# SQ counter passes (one rocprofv3 --pmc pass per group, kernel trace only) over a bench run whose
# waves run alone on their SIMDs (C5 scene on a 64x64 view: 16 blocks, 64 waves) and over the metric
# bench, for the train kernel: where a lone wave's cycles go.
#   bash tools/gpu_pmc_lone.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-lone}
mkdir -p gpurun_out
run() {  # name args...
  local name=$1; shift
  local i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_INSTS_SALU" \
             "SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG}_${name}_$i -o run -- python3 bench.py --cpu-baseline off --aux-steps 0 "$@" > gpurun_out/pmc_${TAG}_${name}_$i.log 2>&1 || return $?
  done
}
run c5s --width 64 --height 64 --spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 2 --warmup 1 && \
run m --steps 3 --warmup 2 && \
python3 - "$TAG" <<'PY'
import csv, glob, sys
tag = sys.argv[1]
for name in ("c5s", "m"):
    vals, dur = {}, []
    for f in glob.glob(f"gpurun_out/pmc_{tag}_{name}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rm_ray_kernel<2" not in r["Kernel_Name"]:
                continue
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(name)
    for k, v in sorted(vals.items()):
        print(f"  {k:32s} {sum(v)/len(v):18.1f}  (n={len(v)})")
PY
