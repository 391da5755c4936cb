# One GPU iteration: the -m gpu suite (stop at the first failure), then optional steps by name.
#   bash tools/gpu_iter.sh <tag> [tests] [small] [smallm] [bench] [train] [trace] [calib]
# tests: pytest -m gpu; small: tools/small_batch_sweep.py + its rocprofv3 stats; smallm: the
# sweep's small-kernel leg at 4 / 7 / 20 / 32 spheres; bench: bench.py; train: the C++ driver's
# whole schedule (rm_train) timed + its rocprofv3 stats; trace: per-wave timelines of one train
# launch (measurement build lib/var/trace.so: bash tools/build_variant.sh WT trace -DRM_BLOCK_TRACE)
# at the metric, C5, C5 on a 64x64 view and C2; calib: FETCH_SIZE / WRITE_SIZE of tools/fetch_calib
# (known byte counts; build it first) into profiles/<tag>_fetch_calibration.json. Outputs under gpurun_out/<tag>/. Every GPU step
# runs under its own time limit; the first failure ends the run.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-it}
shift
O=gpurun_out/$TAG
mkdir -p $O
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
        || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
      tail -2 $O/tests.log; cp gpurun_out/parity_margins.json $O/ ;;
    small)
      timeout -k 10 300 python tools/small_batch_sweep.py > $O/small.json 2> $O/small.err || { tail $O/small.err; exit 1; }
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_small -o run \
        -- python3 tools/small_batch_sweep.py > $O/prof_small.log 2>&1 || { tail $O/prof_small.log; exit 1; } ;;
    smallm)
      for m in 4 7 20 32; do
        timeout -k 10 300 python tools/small_batch_sweep.py --spheres $m --kernels small > $O/small_m$m.json 2>> $O/small.err \
          || { tail $O/small.err; exit 1; }
      done ;;
    bench)
      timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
      cat $O/bench.json ;;
    train)
      mkdir -p $O/train_out
      timeout -k 10 300 burn_raymarching_amd/lib/rm_train train --cameras tests/golden/cameras.json --out $O/train_out \
        --no-previews --log-every 700 > $O/train.log 2>&1 || { tail $O/train.log; exit 1; }
      tail -4 $O/train.log
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_train -o run \
        -- burn_raymarching_amd/lib/rm_train train --cameras tests/golden/cameras.json --out $O/train_out --no-previews \
        --log-every 0 > $O/prof_train.log 2>&1 || { tail $O/prof_train.log; exit 1; } ;;
    calib)
      timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/calib_fetch \
        -o run -- ./tools/fetch_calib > $O/calib_bytes.json 2> $O/calib.log && \
      timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/calib_write \
        -o run -- ./tools/fetch_calib > /dev/null 2>> $O/calib.log && \
      python3 tools/fetch_calib.py $O/calib_fetch $O/calib_write $O/calib_bytes.json profiles/${TAG}_fetch_calibration.json \
        || { tail $O/calib.log; exit 1; }
      cp profiles/${TAG}_fetch_calibration.json $O/ ;;
    trace)
      for c in "metric --bins 20" "c5 --spheres 4096 --march-steps 128 --views 1 --warm 2 --bins 20" \
               "c5s --width 64 --height 64 --spheres 4096 --march-steps 128 --views 1 --warm 2 --bins 8" \
               "c2 --width 256 --height 256 --spheres 64 --bins 20"; do
        set -- $c
        name=$1; shift
        RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so timeout -k 10 200 python tools/block_trace.py \
          --out $O/bt_$name.npz "$@" > $O/bt_$name.txt 2>&1 || { tail $O/bt_$name.txt; exit 1; }
      done ;;
  esac
done
echo done
