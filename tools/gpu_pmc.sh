# rocprofv3 PMC passes for the train kernel (FETCH_SIZE and WRITE_SIZE in separate runs,
# --kernel-trace only; no sys/runtime trace alongside --pmc).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/pmc_fetch_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/pmc_write_$TAG.log 2>&1 && \
python3 tools/pmc_summary.py gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG gpurun_out/${TAG}_pmc_traffic.json 512x512_M256_S32_V2 && cp gpurun_out/${TAG}_pmc_traffic.json profiles/
