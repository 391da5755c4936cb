export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pa_d0 -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/pa_d0.log 2>&1 && \
RM_PER_RAY_ORIGIN=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pa_pr -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/pa_pr.log 2>&1
