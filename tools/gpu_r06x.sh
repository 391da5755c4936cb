# Round 5: the two continuation steps around the default (48, 96) on C5 and C5g, three rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06x
CONFIGS="c5 c5g" ROUNDS=3 bash tools/gpu_ab.sh default "RM_SPLIT_CONT_LIST=40,96" "RM_SPLIT_CONT_LIST=56,96" "RM_SPLIT_CONT_LIST=48,104" "RM_SPLIT_CONT_LIST=48,88" 2>&1 | tee gpurun_out/r06x/ab.txt
