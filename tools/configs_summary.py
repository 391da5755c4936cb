"""Collect the per-config bench lines and rocprofv3 stats of tools/gpu_configs.sh into one
profiles/<tag>_configs.json: per config the bench numbers (value, ms per step, train-kernel time,
executed and canonical roofline fractions) and, from the rocprofv3 --stats run of the same
arguments, the average time per call of every kernel and the per-step time outside the train
kernel.

    python3 tools/configs_summary.py gpurun_out/configs_<tag> profiles/<tag>_configs.json
"""
import csv
import glob
import json
import os
import sys


def main():
    src, out = sys.argv[1], sys.argv[2]
    res = {}
    for path in sorted(glob.glob(os.path.join(src, "*.json"))):
        name = os.path.basename(path)[:-5]
        try:
            d = json.load(open(path))
        except ValueError:
            continue
        if "config" not in d:  # not a bench line (e.g. an earlier summary copied alongside)
            continue
        r = d.get("roofline") or {}
        entry = {"config": d["config"], "value": d["value"], "value_median": d.get("value_median"),
                 "ms_per_step": d["ms_per_step"], "ms_per_step_median": d.get("ms_per_step_median"),
                 "train_kernel_ms": r.get("kernel_ms_per_step"), "frac": r.get("frac"),
                 "executed_frac": r.get("executed_frac"), "canonical_frac": (r.get("canonical") or {}).get("frac"),
                 "backward_rays_frac": r.get("backward_rays_frac"), "value_exit_off": d.get("value_exit_off"),
                 "finite": d.get("finite")}
        if r.get("kernel_ms_per_step") is not None:  # the step's wall time outside the train kernel
            entry["outside_us_per_step"] = round((d["ms_per_step"] - r["kernel_ms_per_step"]) * 1e3, 2)
        stats = glob.glob(os.path.join(src, f"prof_{name}", "**", "*kernel_stats.csv"), recursive=True)
        if stats:
            rows = list(csv.DictReader(open(stats[0])))
            kern = {}
            for row in rows:
                kern[row["Name"][:90]] = {"calls": int(row["Calls"]), "avg_us": round(float(row["AverageNs"]) / 1e3, 2)}
            entry["rocprof_kernels"] = kern
            # the camera-mode train kernel: rm_ray_kernel<2, true, SPLIT> and a split launch's
            # continuation kernel rm_cont_kernel<2, true> (summed)
            tk = [v for k, v in kern.items() if "rm_ray_kernel<2, true" in k or "rm_cont_kernel<2, true" in k]
            train = None
            if tk:
                calls = sum(v["calls"] for v in tk)
                train = {"calls": calls, "avg_us": round(sum(v["avg_us"] * v["calls"] for v in tk) / calls, 2)}
            opt = next((v for k, v in kern.items() if "rm_optimizer" in k), None)
            if train:
                # steps = optimizer calls (one per step); a split launch with a continuation runs the
                # train kernel twice per step
                steps = opt["calls"] if opt else train["calls"]
                entry["rocprof_train_avg_us"] = train["avg_us"]
                entry["rocprof_train_launches_per_step"] = round(train["calls"] / steps, 2)
                entry["rocprof_train_us_per_step"] = round(train["avg_us"] * train["calls"] / steps, 2)
                # the per-step kernels besides the train kernel (one-off setup launches, e.g. the
                # target render, run fewer times than there are steps)
                other = sum(v["avg_us"] * v["calls"] for k, v in kern.items()
                            if ("rm::" in k or "rm_optimizer" in k) and "rm_ray_kernel" not in k and "rm_cont_kernel" not in k
                            and v["calls"] >= steps)
                entry["rocprof_other_us_per_step"] = round(other / steps, 2)
        res[name] = entry
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        print(k, v["value"], v["ms_per_step"], v.get("train_kernel_ms"), v.get("frac"), v.get("canonical_frac"),
              v.get("rocprof_train_us_per_step"), v.get("rocprof_other_us_per_step"))


if __name__ == "__main__":
    main()
