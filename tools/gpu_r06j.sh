# Round 5: the k = 5 gap and the backward's LDS share.
#  1. same-box A/B of |p|^2 formed in registers in the backward sweeps (lib/var/psq.so) on the
#     metric and k = 5, and the k-annealed bench line (5 -> 32 over the timed steps);
#  2. per-wave timelines (lib/var/trace.so) of the metric with the exit off at k = 32 and k = 5:
#     the march / post-march / backward shares of the wave time;
#  3. one PMC pass of LDS counters over the metric.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06j
mkdir -p $O
CONFIGS="m k5" ROUNDS=2 bash tools/gpu_ab.sh default lib:psq 2>&1 | tee $O/ab.txt || exit 1
timeout -k 10 200 python bench.py --cpu-baseline off --anneal-k 5 --steps 10 > $O/kanneal.json 2> $O/kanneal.err || exit 1
python3 -c "import json; d=json.load(open('$O/kanneal.json')); r=d['roofline']; print('kanneal', d['value'], d['ms_per_step'], r['frac'], r['executed_frac'], (r.get('canonical') or {}).get('frac'))"
export RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so
RM_NO_EARLY_EXIT=1 timeout -k 10 200 python tools/block_trace.py --views 80 --warm 2 --bins 20 > $O/bt_m_exitoff.txt 2>&1 && \
RM_NO_EARLY_EXIT=1 timeout -k 10 200 python tools/block_trace.py --views 80 --warm 2 --bins 20 --smooth-k 5 > $O/bt_k5_exitoff.txt 2>&1 || exit 1
unset RM_LIB_PATH
grep -h 'launch span\|summed wave time\|live waves' $O/bt_*.txt
PB="python3 bench.py --cpu-baseline off --aux-steps 0 --steps 3 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/$O/pmc_lds -o run -- $PB > $O/pmc_lds.log 2>&1
rc=$?
echo "pmc rc $rc"
exit 0
