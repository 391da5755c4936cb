"""Summarise rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE, separate runs) for the train
kernel into profiles/<round>_pmc_traffic.json: HBM bytes per launch and, given the number of
bench steps the passes ran (warm-up + timed), per step -- a step may hold several launches (the
strong-scaling default issues 16 views per launch; C5 adds a continuation launch). bench.py
quotes the per-step figure next to its per-step achieved rate.

    python3 tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json KEY [STEPS]

MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB and come from the L2's fabric-side
request counters; on gfx950 FETCH_SIZE reads 1/2 of the bytes of wide (16 B/lane) coalesced
streams. This kernel's global reads are dword-wide (targets, sphere tables, all L2/MALL
resident) and its stores dword-wide partial slabs, for which the guide has no calibration, so
both the raw and the x2-corrected read figure are recorded and the raw sum is used.
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


def main():
    fetch_dir, write_dir, out, key = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    f = per_kernel(fetch_dir, "FETCH_SIZE")
    w = per_kernel(write_dir, "WRITE_SIZE")
    names = [k for k in f if "rm_ray_kernel<2, true" in k]  # camera-mode train kernel (split or not)
    if not names:
        raise SystemExit("train kernel not found in the counter CSVs")
    fv = [x for k in names for x in f[k]]
    wv = [x for k in names for x in w.get(k, [])]
    fk = sum(fv) / len(fv)
    wk = sum(wv) / max(len(wv), 1)
    data = json.load(open(out)) if os.path.exists(out) else {}
    data.setdefault("train_kernel_bytes_per_launch", {})[key] = (fk + wk) * 1024.0
    if steps > 0:
        data.setdefault("train_kernel_bytes_per_step", {})[key] = (sum(fv) + sum(wv)) * 1024.0 / steps
    data.setdefault("detail", {})[key] = {
        "kernels": names, "FETCH_SIZE_KiB_per_launch": fk, "WRITE_SIZE_KiB_per_launch": wk, "launches": len(fv),
        "steps": steps, "fetch_bytes_x2_corrected_per_launch": fk * 2048.0,
        "note": "dword-wide accesses: the gfx950 FETCH x2 correction applies to 16 B/lane streams only; raw "
                "FETCH+WRITE used as traffic"}
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps(data["detail"][key]))


if __name__ == "__main__":
    main()
