# The split continuation at the round-4 end (packed accumulate: four waves per SIMD): per-wave
# timelines of C5g's and C5's continuation launches (tools/block_trace.py, measurement build).
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
export RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so
timeout -k 10 200 python tools/block_trace.py --march-steps 128 --views 1 --warm 2 --bins 20 --color-f16 \
  --scene-json profiles/r05a_grown_scene_4096.json --cameras tests/golden/cameras.json > $O/bt_c5g.txt 2>&1 && \
timeout -k 10 200 python tools/block_trace.py --spheres 4096 --march-steps 128 --views 1 --warm 2 --bins 20 \
  > $O/bt_c5.txt 2>&1
rc=$?
grep -h 'launch span\|mean live\|summed wave time\|CU last-wave' $O/bt_*.txt
exit $rc
