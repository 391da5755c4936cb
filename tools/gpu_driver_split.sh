# The C++ driver's whole schedule (5 x 700 steps, batch 16384) with the automatic split choice and
# with the split march off (RM_SPLIT=0), same box.
set -o pipefail
mkdir -p gpurun_out/drv
E=burn_raymarching_amd/lib/rm_train
timeout -k 10 120 $E generate --out gpurun_out/drv/data --prefix "" > /dev/null || exit 1
for r in 1 2; do
  for sp in auto 0; do
    if [ $sp = auto ]; then unset RM_SPLIT; else export RM_SPLIT=0; fi
    timeout -k 10 200 $E train --cameras gpurun_out/drv/data/cameras.json --out gpurun_out/drv/run_$sp > gpurun_out/drv/train_${sp}_$r.log 2>&1 || { tail -5 gpurun_out/drv/train_${sp}_$r.log; exit 1; }
    echo "split=$sp $(tail -1 gpurun_out/drv/train_${sp}_$r.log)"
  done
done
