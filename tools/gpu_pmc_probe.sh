#!/bin/bash
# PMC counter groups (one rocprofv3 --pmc pass each, kernel trace only) over tools/pmc_probe.py.
#   bash tools/gpu_pmc_probe.sh <tag> [S] [mode]   (env e.g. RM_NO_EARLY_EXIT=1 passes through)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-probe}
mkdir -p gpurun_out
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA" \
           "SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG}_$i -o run -- python3 tools/pmc_probe.py ${2:-32} ${3:-fwd} > gpurun_out/pmc_${TAG}_$i.log 2>&1 || exit $?
done
python3 - "$TAG" <<'PY'
import csv, glob, sys
tag = sys.argv[1]
vals = {}
for f in glob.glob(f"gpurun_out/pmc_{tag}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rm_ray_kernel" not in r["Kernel_Name"]:
            continue
        vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, v in sorted(vals.items()):
    print(f"{k:32s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
