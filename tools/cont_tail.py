#!/usr/bin/env python3
"""Where a split continuation launch's tail comes from (tools/block_trace.py --out npz of a
measurement build): the waves that end in the launch's last fifth -- when they started, how many
march steps they ran, how long a step took them and how many other waves shared their SIMD.

    python tools/cont_tail.py gpurun_out/r06h/c5g_cont.npz --steps 128
"""
import argparse

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--frac", type=float, default=0.2, help="the tail: waves ending in the last FRAC of the span")
    args = ap.parse_args()
    tr = np.load(args.npz)["trace"]
    tr = tr[tr[:, 0] != 0]
    t0, t1 = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
    base = t0.min()
    s, e = (t0 - base) / 100.0, (t1 - base) / 100.0
    hw = tr[:, 2]
    xcc = (hw >> np.uint64(32)).astype(np.int64) & 0xF
    lo = (hw & np.uint64(0xFFFFFFFF)).astype(np.int64)
    simd_key = ((((xcc * 8 + ((lo >> 13) & 7)) * 2 + ((lo >> 12) & 1)) * 16 + ((lo >> 8) & 0xF)) * 4 + ((lo >> 4) & 3))
    steps = args.steps - tr[:, 6].astype(np.int64)
    real = (e - s) > 5.0  # waves that did work (empty continuation blocks end at once)
    span = e.max()
    tail = real & (e >= (1.0 - args.frac) * span)
    print(f"span {span:.0f} us, working waves {int(real.sum())}, waves ending in the last {args.frac:.0%}: {int(tail.sum())}")
    for name, m in (("all working", real), ("tail", tail)):
        st = s[m]
        print(f"{name:12s} start us  p10/50/90/max: " + " ".join(f"{np.percentile(st, p):.0f}" for p in (10, 50, 90, 100))
              + f"   steps p10/50/90: " + " ".join(f"{np.percentile(steps[m], p):.0f}" for p in (10, 50, 90))
              + f"   us/step median: {np.median((e[m] - s[m]) / np.maximum(steps[m] - 48, 1)):.1f}")
    # how many waves were live on the tail waves' SIMDs at their start
    live_at = []
    for i in np.flatnonzero(tail)[:400]:
        same = (simd_key == simd_key[i]) & real
        live_at.append(int(((s[same] <= s[i]) & (e[same] > s[i])).sum()))
    if live_at:
        print("tail waves: live waves on their SIMD when they started, p10/50/90: "
              + " ".join(f"{np.percentile(live_at, p):.0f}" for p in (10, 50, 90)))
    # start-time histogram of waves that ran all remaining steps vs the rest
    full = real & (steps >= args.steps - 1)
    print(f"waves that marched to the last step: {int(full.sum())}; their start us p10/50/90: "
          + (" ".join(f"{np.percentile(s[full], p):.0f}" for p in (10, 50, 90)) if full.any() else "-"))


if __name__ == "__main__":
    main()
