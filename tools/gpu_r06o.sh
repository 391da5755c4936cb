# Round 5: (1) every rank's share of the N = 2 / 4 / 8 strong step alone on one GPU (gpu_r06n.sh);
# (2) the split continuation's step on the 32-ray groups: 48 (default) vs 64 / 80, and a second
# continuation at 96, and the static centre-out order (the rotating view reuses another view's cost order), on C5 and C5g.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_r06n.sh || exit 1
mkdir -p gpurun_out/r06o
CONFIGS="c5 c5g" ROUNDS=2 bash tools/gpu_ab.sh default "RM_SPLIT_CONT_STEPS=64" "RM_SPLIT_CONT_STEPS=80" "RM_SPLIT_CONT2_STEPS=96" "RM_STATIC_ORDER=1" 2>&1 | tee gpurun_out/r06o/ab.txt
# (3) the backward's finish_split inlined (no scratch memory: 80 -> 0 bytes per lane) vs before (lib:scr)
CONFIGS="m c2cj c5g" ROUNDS=2 bash tools/gpu_ab.sh lib:scr default 2>&1 | tee gpurun_out/r06o/ab_scr.txt
