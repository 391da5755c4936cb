set -o pipefail
mkdir -p gpurun_out/ab
for lib in default b64; do
  if [ $lib = default ]; then unset RM_LIB_PATH; else export RM_LIB_PATH=burn_raymarching_amd/lib/var/$lib.so; fi
  timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 > gpurun_out/ab/m_$lib.json || exit 1
  timeout -k 10 200 python bench.py --cpu-baseline off --width 256 --height 256 --spheres 64 --steps 20 > gpurun_out/ab/c2_$lib.json || exit 1
  timeout -k 10 200 python bench.py --cpu-baseline off --spheres 4096 --march-steps 128 --views-per-gpu 1 --steps 4 --warmup 2 > gpurun_out/ab/c5_$lib.json || exit 1
done
for f in gpurun_out/ab/*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['kernel_ms_per_step'], r['frac'], (r['canonical'] or {}).get('frac'))" $f; done
