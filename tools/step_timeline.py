"""Per-step GPU timeline from a rocprofv3 --kernel-trace CSV: for the last few occurrences of the
train kernel, list every kernel of that step with its start offset, duration and the idle gap
before it -- where the non-kernel part of a bench step goes.

    python tools/step_timeline.py <dir with *_kernel_trace.csv> [steps]
"""
import csv
import glob
import os
import sys


def main():
    path = sys.argv[1]
    nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    f = path if path.endswith(".csv") else glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "rm_ray_kernel" in r["Kernel_Name"]]
    for si in range(max(0, len(starts) - nsteps - 1), len(starts) - 1):
        a, b = starts[si], starts[si + 1]
        t0 = int(rows[a]["Start_Timestamp"])
        tend = int(rows[b]["Start_Timestamp"])
        print(f"-- step: {(tend - t0) / 1e3:.1f} us from train-kernel start to the next")
        prev_end = None
        for r in rows[a:b + 1]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
            print(f"   +{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:6.1f}  {r['Kernel_Name'][:70]}")
            prev_end = e


if __name__ == "__main__":
    main()
