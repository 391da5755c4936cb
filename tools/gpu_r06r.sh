# Round 5: a second split continuation (at 96 of 128 steps), alone and with the first at 64, on
# C5 and C5g, three rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06r
CONFIGS="c5 c5g" ROUNDS=3 bash tools/gpu_ab.sh default "RM_SPLIT_CONT2_STEPS=96" "RM_SPLIT_CONT_STEPS=64 RM_SPLIT_CONT2_STEPS=96" "RM_SPLIT_CONT2_STEPS=88" 2>&1 | tee gpurun_out/r06r/ab.txt
