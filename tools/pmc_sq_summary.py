"""Summarise rocprofv3 --pmc SQ passes over bench.py for the train kernel into
profiles/<round>_pmc_sq.json (what bench.py quotes as roofline.pmc).

    python3 tools/pmc_sq_summary.py OUT.json KEY default_dir1 default_dir2 noexit_dir1 [bench.json]

default_dir1 / noexit_dir1: a pass with SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA
SQ_WAVES over `bench.py --aux-steps 0` with the early exit on (default) and off
(RM_NO_EARLY_EXIT=1); default_dir2: SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU on the default run. Each directory also holds the kernel trace of its run
(durations). SQ instruction counters count wave-instructions (one per wave64 instruction).

Derived, per train step (the dispatches of rm_ray_kernel<2, true> and of a split launch's
continuation kernel rm_cont_kernel<2, true> summed; steps = the first kernel's dispatches):
  * trans_issue_frac: transcendental wave-instructions x their measured issue cost (cycles per
    wave-instruction per SIMD, profiles/r01_valu_rates.txt: sqrt 8.35, exp 9.37, log 8.37,
    rcp 8.44, rsq 8.26 -> 8.6 on the kernel's mix) / (1024 SIMDs x clock x kernel time) -- the
    fraction of the transcendental-issue ceiling the kernel uses;
  * executed_ratio_pmc: transcendental instructions with the early exit on / off -- the share of
    the full per-ray work that ran, measured by the hardware, to compare with the bench's
    stats-based executed_frac / executed_frac(exit off) of the same steps (bench.json: a bench
    line with the PMC passes' arguments and the replays on; exit off runs S - 1 march steps (the
    shared origin step), 3 post-march sweeps and the seeded rays' 2 backward sweeps of the S + 10
    per wave).
"""
import csv
import glob
import json
import os
import sys

KERNEL = "rm_ray_kernel<2, true"  # <2, true, SPLIT>: the camera-mode train kernel
KERNELS = (KERNEL, "rm_cont_kernel<2, true")  # ... and a split launch's continuation kernel


def is_train(name):
    return any(k in name for k in KERNELS)
TRANS_CYCLES = 8.6    # cycles per transcendental wave-instruction per SIMD (r01_valu_rates.txt)
OTHER_CYCLES = 4.0    # other VALU: fma 2.96, add 3.56, max 4.45, packed fma 5.02 (r01_valu_rates.txt)
SIMDS = 1024          # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4       # nominal (MI355X_MICROARCH.md); the measured clock is used when available


def rows(path, suffix):
    out = []
    for f in glob.glob(os.path.join(path, "**", f"*{suffix}"), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def counters(path):
    """Per train step: the counters summed over the step's train dispatches (a split launch with a
    continuation dispatches twice per step), divided by the steps (the first kernel's dispatches)."""
    vals, firsts = {}, {}
    for r in rows(path, "counter_collection.csv"):
        if not is_train(r["Kernel_Name"]):
            continue
        vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if KERNEL in r["Kernel_Name"]:  # (one row per dispatch and counter without a dispatch id)
            ids = firsts.setdefault(r["Counter_Name"], set())
            ids.add(r.get("Dispatch_Id") or len(ids))
    steps = max((len(v) for v in firsts.values()), default=0)
    return {k: v / steps for k, v in vals.items()} if steps else {}, steps


def duration_ns(path):
    """Per train step: the summed durations of the step's train dispatches."""
    tr = [r for r in rows(path, "kernel_trace.csv") if is_train(r["Kernel_Name"])]
    steps = sum(1 for r in tr if KERNEL in r["Kernel_Name"])
    d = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr)
    return d / steps if steps else None


def main():
    out, key, d1, d2, n1 = sys.argv[1:6]
    bench = json.load(open(sys.argv[6])) if len(sys.argv) > 6 else None
    c1, launches = counters(d1)
    c2, _ = counters(d2)
    cn, _ = counters(n1)
    dur = duration_ns(d1)
    dur2 = duration_ns(d2)
    clock = None
    if "GRBM_GUI_ACTIVE" in c2 and dur2:
        clock = c2["GRBM_GUI_ACTIVE"] / dur2  # cycles per ns = GHz
        if clock > 4.0:  # summed over the 8 XCDs
            clock /= 8.0
    clk = clock or CLOCK_GHZ
    trans = c1.get("SQ_INSTS_VALU_TRANS_F32")
    res = {
        "kernel": KERNEL,
        "launches": launches,
        "kernel_ns": dur,
        "counters": {**c1, **c2},
        "counters_exit_off": cn,
        "clock_GHz": clock,
        "trans_issue_frac": (trans * TRANS_CYCLES / (SIMDS * clk * dur)) if trans and dur else None,
        "trans_cycles_per_inst": TRANS_CYCLES,
        "valu_insts": c1.get("SQ_INSTS_VALU"),
        "trans_insts": trans,
        "mfma_insts": c1.get("SQ_INSTS_MFMA"),
        "trans_share_of_valu": trans / c1["SQ_INSTS_VALU"] if trans and c1.get("SQ_INSTS_VALU") else None,
        "executed_ratio_pmc": (trans / cn["SQ_INSTS_VALU_TRANS_F32"]) if trans and cn.get("SQ_INSTS_VALU_TRANS_F32")
        else None,
        # wave-level: share of a wave's lifetime spent issuing VALU (both counters in quad-cycles)
        "valu_active_frac": (c2["SQ_ACTIVE_INST_VALU"] / c2["SQ_WAVE_CYCLES"])
        if c2.get("SQ_ACTIVE_INST_VALU") and c2.get("SQ_WAVE_CYCLES") else None,
        # SIMD-level estimate: all VALU wave-instructions at their measured issue costs (others at
        # a representative OTHER_CYCLES) over the SIMD-cycles of the launch
        "valu_issue_frac_est": ((trans * TRANS_CYCLES + (c1["SQ_INSTS_VALU"] - trans) * OTHER_CYCLES)
                                / (SIMDS * clk * dur)) if trans and dur and c1.get("SQ_INSTS_VALU") else None,
    }
    if bench and bench.get("roofline") and bench["roofline"].get("executed_frac"):
        S = bench["config"]["march_steps"]
        ef = bench["roofline"]["executed_frac"]
        res["executed_frac_stats"] = ef
        # exit off: S - 1 march steps (the shared origin step), 3 post-march sweeps, and the two
        # backward sweeps of the rays with non-zero seeds (the same rays with the exit on and off)
        bw = bench["roofline"].get("backward_rays_frac")
        post = 3 + sum(bw) if bw else 5
        res["executed_ratio_stats"] = ef / ((S - 1 + post) / (S + 10))
        res["stats_source"] = os.path.basename(sys.argv[6])
    data = json.load(open(out)) if os.path.exists(out) else {}
    data.setdefault("train_kernel", {})[key] = res
    data["note"] = __doc__
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("counters", "counters_exit_off")}))


if __name__ == "__main__":
    main()
