#!/bin/bash
# A/B of the exact escape skip and of the camera-mode pixel tiling on the metric config (1 GPU).
set -e
mkdir -p gpurun_out
B="timeout -k 10 300 python bench.py --cpu-baseline off"
$B --skip-escaped off > gpurun_out/ab_off_t2.json
$B --skip-escaped on > gpurun_out/ab_on_t2.json
RM_TILING_EXPERIMENT=0 $B --skip-escaped off > gpurun_out/ab_off_t0.json
RM_TILING_EXPERIMENT=1 $B --skip-escaped off > gpurun_out/ab_off_t1.json
$B --skip-escaped on --lr 0.0 > gpurun_out/ab_on_t2_lr0.json
