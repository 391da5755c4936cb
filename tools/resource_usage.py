#!/usr/bin/env python3
"""Register / occupancy / spill figures of every kernel in rm_kernels.hip, from the compiler's
own report (hipcc -Rpass-analysis=kernel-resource-usage, device-only, gfx950), one line per kernel
in the format of profiles/r07_resource_usage.txt.

    python3 tools/resource_usage.py [rev-label] > profiles/<tag>_resource_usage.txt
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "burn_raymarching_amd", "csrc", "rm_kernels.hip")
FIELDS = [("VGPRs", "V"), ("AGPRs", "A"), ("Occupancy [waves/SIMD]", "occ"), ("SGPRs Spill", "sgprspill"),
          ("VGPRs Spill", "vgprspill"), ("ScratchSize [bytes/lane]", "scratch")]


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "working tree"
    with tempfile.TemporaryDirectory() as td:
        out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                              "-c", SRC, "-o", os.path.join(td, "k.o"), "-Rpass-analysis=kernel-resource-usage"],
                             capture_output=True, text=True, check=True).stderr
    kern, rows = None, {}
    for line in out.splitlines():
        m = re.search(r"remark: Function Name: _ZN2rm(\S+)", line)
        if m:
            kern = m.group(1)
            rows[kern] = {}
            continue
        m = re.search(r"remark:\s+([^:]+): (\d+)", line)
        if m and kern is not None:
            rows[kern][m.group(1).strip()] = m.group(2)
    print(f"# hipcc -O3 --offload-arch=gfx950 --cuda-device-only -Rpass-analysis=kernel-resource-usage on {label}")
    print("# kernel  VGPRs  AGPRs  occupancy(waves/SIMD)  SGPR-spill  VGPR-spill  scratch(B/lane); "
          "template <MODE 0 fwd 1 bwd 2 train 3 render, CAMERA, SPLIT>")
    for k in sorted(rows):
        r = rows[k]
        print(k + " " + " ".join(f"{short} {r.get(name, '?')}" for name, short in FIELDS))


if __name__ == "__main__":
    main()
