# Split march forced on / off (RM_SPLIT=1 / 0) over workload shapes, one box: where the automatic
# choice should switch. Prints: shape, split, Mrays/s, ms/step, kernel ms.
set -o pipefail
mkdir -p gpurun_out/ssw
run() {  # name args...
  name=$1; shift
  for sp in 0 1; do
    RM_SPLIT=$sp timeout -k 10 200 python bench.py --cpu-baseline off --aux-steps 0 "$@" > gpurun_out/ssw/${name}_$sp.json 2> gpurun_out/ssw/${name}_$sp.err || { tail -3 gpurun_out/ssw/${name}_$sp.err; return 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], 'split', sys.argv[3], d['value'], d['ms_per_step'], r['kernel_ms_per_step'])" gpurun_out/ssw/${name}_$sp.json $name $sp
  done
}
run m256_s32_v10 --steps 10 && \
run m256_s64_v10 --march-steps 64 --steps 10 && \
run m256_s32_v1 --views-per-gpu 1 --steps 10 && \
run m256_s32_v4 --views-per-gpu 4 --steps 10 && \
run m256_s64_v4 --march-steps 64 --views-per-gpu 4 --steps 10 && \
run m256_s128_v1 --march-steps 128 --views-per-gpu 1 --steps 10 && \
run m512_s32_v1 --spheres 512 --views-per-gpu 1 --steps 10 && \
run m512_s64_v4 --spheres 512 --march-steps 64 --views-per-gpu 4 --steps 6 && \
run m1024_s32_v1 --spheres 1024 --views-per-gpu 1 --steps 10 && \
run m1024_s64_v4 --spheres 1024 --march-steps 64 --views-per-gpu 4 --steps 6 && \
run c4 --width 1024 --height 1024 --spheres 1024 --march-steps 64 --views-per-gpu 4 --steps 4 --warmup 2 && \
run m2048_s128_v4 --spheres 2048 --march-steps 128 --views-per-gpu 4 --steps 4 --warmup 2 && \
run m4096_s128_v4 --spheres 4096 --march-steps 128 --views-per-gpu 4 --steps 4 --warmup 2 && \
run m4096_s32_v1 --spheres 4096 --march-steps 32 --views-per-gpu 1 --steps 6
