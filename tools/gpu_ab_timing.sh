# Cost of the kernel-timing events in the bench loop: bench.py alternately with and without them
# (same box, ms per step). Every GPU step under its own time limit.
mkdir -p gpurun_out
for i in 1 2 3; do
  for kt in on off; do
    timeout -k 10 200 python bench.py --cpu-baseline off --kernel-timing $kt > gpurun_out/abt_${kt}_$i.json 2>gpurun_out/abt_${kt}_$i.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/abt_${kt}_$i.json $kt
  done
done
