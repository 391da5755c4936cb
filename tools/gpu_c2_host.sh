set -o pipefail
mkdir -p gpurun_out
for st in 20 200; do
timeout -k 10 200 python bench.py --cpu-baseline off --width 256 --height 256 --spheres 64 --steps $st > gpurun_out/c2h_$st.json || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['ms_per_step_median'], d['host_submit_ms_per_step'], d['roofline']['kernel_ms_per_step'])" gpurun_out/c2h_$st.json
done
timeout -k 10 200 python bench.py --cpu-baseline off --steps 20 > gpurun_out/mh.json || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['ms_per_step_median'], d['host_submit_ms_per_step'], d['roofline']['kernel_ms_per_step'])" gpurun_out/mh.json
