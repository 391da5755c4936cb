"""Summarise rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE, separate runs) for the train
kernel into profiles/<round>_pmc_traffic.json: HBM bytes per launch and, given the number of
bench steps the passes ran (warm-up + timed), per step -- a step may hold several launches (the
strong-scaling default issues 16 views per launch; C5 adds a continuation launch). bench.py
quotes the per-step figure next to its per-step achieved rate.

    python3 tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json KEY [STEPS [CALIB.json]]

STEPS 0 or 'auto': the number of optimizer dispatches (one per step) in FETCH_DIR's kernel trace.

MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB and come from the L2's fabric-side
request counters; on gfx950 FETCH_SIZE reads 1/2 of the bytes of wide (16 B/lane) coalesced
streams, and other widths are uncalibrated. This kernel's HBM reads are dword-wide (the AoS
float3 targets) and its stores dword-wide partial records, so CALIB.json (tools/fetch_calib.py:
the same widths and the record write pattern on known byte counts) supplies the factors:
traffic = FETCH x read_f3_factor + WRITE x write_rec_factor. Without it the raw sum is recorded.
"""
import csv
import glob
import json
import os
import sys


def rows(path):
    out = []
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def per_kernel(path, counter):
    vals = {}
    for r in rows(path):
        if r.get("Counter_Name") != counter:
            continue
        k = r["Kernel_Name"]
        vals.setdefault(k, []).append(float(r["Counter_Value"]))
    return vals


def optimizer_dispatches(path):
    n = 0
    for f in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
        n += sum(1 for r in csv.DictReader(open(f)) if "rm_optimizer" in r["Kernel_Name"])
    return n


def main():
    fetch_dir, write_dir, out, key = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
    steps = sys.argv[5] if len(sys.argv) > 5 else "auto"
    steps = optimizer_dispatches(fetch_dir) if steps in ("0", "auto") else int(steps)
    calib = json.load(open(sys.argv[6])) if len(sys.argv) > 6 else None
    rf = calib["read_f3_factor"] if calib else 1.0
    wf = calib["write_rec_factor"] if calib else 1.0
    f = per_kernel(fetch_dir, "FETCH_SIZE")
    w = per_kernel(write_dir, "WRITE_SIZE")
    # camera-mode train kernel (split or not) and a split launch's continuation kernel
    names = [k for k in f if "rm_ray_kernel<2, true" in k or "rm_cont_kernel<2, true" in k]
    if not names:
        raise SystemExit("train kernel not found in the counter CSVs")
    fv = [x for k in names for x in f[k]]
    wv = [x for k in names for x in w.get(k, [])]
    fk = sum(fv) / len(fv)
    wk = sum(wv) / max(len(wv), 1)
    data = json.load(open(out)) if os.path.exists(out) else {}
    data.setdefault("train_kernel_bytes_per_launch", {})[key] = (fk * rf + wk * wf) * 1024.0
    if steps > 0:
        data.setdefault("train_kernel_bytes_per_step", {})[key] = (sum(fv) * rf + sum(wv) * wf) * 1024.0 / steps
    data.setdefault("detail", {})[key] = {
        "kernels": names, "FETCH_SIZE_KiB_per_launch": fk, "WRITE_SIZE_KiB_per_launch": wk, "launches": len(fv),
        "steps": steps, "raw_bytes_per_launch": (fk + wk) * 1024.0,
        "calibration": {"read_f3_factor": rf, "write_rec_factor": wf, "file": sys.argv[6]} if calib else None,
        "note": "traffic = FETCH x read factor + WRITE x write factor (dword-wide accesses, calibrated on known "
                "byte counts by tools/fetch_calib)" if calib else "uncalibrated raw FETCH+WRITE"}
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps(data["detail"][key]))


if __name__ == "__main__":
    main()
