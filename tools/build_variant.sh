#!/bin/bash
# Build libraymarch_hip.so from a git revision of the kernel source into lib/var/<name>.so, for
# same-box A/B timing (RM_LIB_PATH=burn_raymarching_amd/lib/var/<name>.so).
#   bash tools/build_variant.sh <rev|WT> <name> [extra hipcc flags]   (WT: the working tree)
set -e
REV=$1; NAME=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/burn_raymarching_amd/csrc
mkdir -p "$ROOT/burn_raymarching_amd/lib/var"
if [ "$REV" = WT ]; then  # the working tree
  cp "$CS/rm_kernels.hip" "$CS/_variant_$NAME.hip"
  cp "$CS/rm_device.h" "$CS/_variant_device_$NAME.h"
  cp "$CS/rm_small.h" "$CS/_variant_small_$NAME.h"
else
  git -C "$ROOT" show "$REV:burn_raymarching_amd/csrc/rm_kernels.hip" > "$CS/_variant_$NAME.hip"
  git -C "$ROOT" show "$REV:burn_raymarching_amd/csrc/rm_device.h" > "$CS/_variant_device_$NAME.h"
  git -C "$ROOT" show "$REV:burn_raymarching_amd/csrc/rm_small.h" > "$CS/_variant_small_$NAME.h"
fi
sed -i "s/#include \"rm_device.h\"/#include \"_variant_device_$NAME.h\"/" "$CS/_variant_$NAME.hip"
sed -i "s/#include \"rm_small.h\"/#include \"_variant_small_$NAME.h\"/" "$CS/_variant_$NAME.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result "$@" \
  -o "$ROOT/burn_raymarching_amd/lib/var/$NAME.so" "$CS/_variant_$NAME.hip"
rm -f "$CS/_variant_$NAME.hip" "$CS/_variant_device_$NAME.h" "$CS/_variant_small_$NAME.h"
echo "built lib/var/$NAME.so from $REV"
