"""The profile summarisers that turn rocprofv3 output into the committed profiles/ numbers
(tools/configs_summary.py, tools/pmc_summary.py, tools/pmc_sq_summary.py): on synthetic CSVs of
the rocprofv3 layout, a split launch's continuation kernel (rm_cont_kernel) is counted as train
kernel time next to rm_ray_kernel, and the per-step figures divide by the optimizer dispatches."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RAY = "void rm::rm_ray_kernel<2, true, true>(rm::KArgs)"
CONT = "void rm::rm_cont_kernel<2, true>(rm::KArgs)"
OPT = "rm::rm_optimizer_kernel(float*, ...)"
RED = "rm::rm_reduce_partials(float const*, ...)"


def _write_csv(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def _tool(*args):
    return subprocess.run([sys.executable, os.path.join(ROOT, "tools", args[0]), *args[1:]], check=True,
                          capture_output=True, text=True).stdout


def test_configs_summary_counts_the_continuation(tmp_path):
    src = tmp_path / "configs"
    line = {"config": {"workload": "x"}, "value": 50.0, "ms_per_step": 5.0,
            "roofline": {"kernel_ms_per_step": 4.8, "frac": 0.4, "executed_frac": 0.13, "canonical": {"frac": 0.7}}}
    os.makedirs(src)
    json.dump(line, open(src / "C5.json", "w"))
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"]
    # 4 steps: the first launch 3000 us and the continuation 1500 us per step, 50 us of reduction
    _write_csv(str(src / "prof_C5" / "run_kernel_stats.csv"), hdr,
               [[RAY, 4, 12e6, 3e6, 60, 0, 0, 0], [CONT, 4, 6e6, 1.5e6, 30, 0, 0, 0],
                [RED, 4, 2e5, 5e4, 1, 0, 0, 0], [OPT, 4, 4e4, 1e4, 1, 0, 0, 0]])
    out = tmp_path / "configs.json"
    _tool("configs_summary.py", str(src), str(out))
    e = json.load(open(out))["C5"]
    assert e["rocprof_train_launches_per_step"] == 2.0
    assert e["rocprof_train_us_per_step"] == 4500.0
    assert e["rocprof_train_avg_us"] == 2250.0
    assert e["rocprof_other_us_per_step"] == 60.0  # reduction + optimizer, not the continuation
    assert abs(e["outside_us_per_step"] - 200.0) < 1e-6


def test_pmc_summary_counts_the_continuation(tmp_path):
    hdr = ["Kernel_Name", "Counter_Name", "Counter_Value"]
    # FETCH / WRITE in KiB per dispatch: two launches per step over 2 steps
    _write_csv(str(tmp_path / "fetch" / "run_counter_collection.csv"), hdr,
               [[RAY, "FETCH_SIZE", 100], [CONT, "FETCH_SIZE", 50]] * 2)
    _write_csv(str(tmp_path / "write" / "run_counter_collection.csv"), hdr,
               [[RAY, "WRITE_SIZE", 10], [CONT, "WRITE_SIZE", 30]] * 2)
    _write_csv(str(tmp_path / "fetch" / "run_kernel_trace.csv"), ["Kernel_Name"], [[OPT], [OPT]])
    out = tmp_path / "traffic.json"
    _tool("pmc_summary.py", str(tmp_path / "fetch"), str(tmp_path / "write"), str(out), "K")
    d = json.load(open(out))
    assert d["detail"]["K"]["launches"] == 4 and d["detail"]["K"]["steps"] == 2
    assert d["train_kernel_bytes_per_step"]["K"] == (300 + 80) * 1024.0 / 2  # uncalibrated raw sum
    assert sorted(d["detail"]["K"]["kernels"]) == sorted([RAY, CONT])


def test_pmc_sq_summary_counts_the_continuation(tmp_path):
    """Per train step: a split step's two dispatches (first launch + continuation) summed, against
    the exit-off run's one launch per step (the mean per dispatch would halve the split step)."""
    hdr = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]
    thdr = ["Kernel_Name", "Start_Timestamp", "End_Timestamp"]
    _write_csv(str(tmp_path / "d1" / "run_counter_collection.csv"), hdr,
               [[1, RAY, "SQ_INSTS_VALU_TRANS_F32", 1000], [2, CONT, "SQ_INSTS_VALU_TRANS_F32", 1000],
                [1, RAY, "SQ_INSTS_VALU", 2000], [2, CONT, "SQ_INSTS_VALU", 2000]])
    _write_csv(str(tmp_path / "d1" / "run_kernel_trace.csv"), thdr, [[RAY, 0, 1000], [CONT, 0, 3000], [OPT, 0, 5]])
    _write_csv(str(tmp_path / "n1" / "run_counter_collection.csv"), hdr,
               [[1, RAY, "SQ_INSTS_VALU_TRANS_F32", 8000], [1, RAY, "SQ_INSTS_VALU", 16000]])
    _write_csv(str(tmp_path / "n1" / "run_kernel_trace.csv"), thdr, [[RAY, 0, 9000]])
    _write_csv(str(tmp_path / "d2" / "run_counter_collection.csv"), hdr, [[1, RAY, "GRBM_GUI_ACTIVE", 4000]])
    _write_csv(str(tmp_path / "d2" / "run_kernel_trace.csv"), thdr, [[RAY, 0, 2000]])
    out = tmp_path / "sq.json"
    _tool("pmc_sq_summary.py", str(out), "K", str(tmp_path / "d1"), str(tmp_path / "d2"), str(tmp_path / "n1"))
    r = json.load(open(out))["train_kernel"]["K"]
    assert r["launches"] == 1 and r["kernel_ns"] == 4000.0  # both dispatches of the one step
    assert r["executed_ratio_pmc"] == 0.25  # (1000 + 1000) / 8000
    assert r["trans_share_of_valu"] == 0.5


def test_predict_scaling_per_call(tmp_path):
    """tools/predict_scaling.py --per-call: T(N) = one call's train kernel (the N = 1 step run as N
    calls) x the slowest-over-mean slice + one call's share of the step's other kernels + the
    all-reduce floor + 2 (N - 1) hops; efficiency against the N = 1 line."""
    def line(ms, kern_step, kern, launches):
        return {"ms_per_step": ms, "config": {"spheres": 256, "rays_per_step": 8_000_000},
                "roofline": {"kernel_ms_per_step": kern_step, "kernel_ms": kern, "launches_timed": launches,
                             "frac": 0.5}}
    json.dump(line(10.0, 9.8, 9.8, 6), open(tmp_path / "n1.json", "w"))
    json.dump(line(10.4, 10.0, 5.0, 12), open(tmp_path / "n2.json", "w"))
    json.dump({"spread": {"2": {"slice_ms": [1.0, 1.02]}}}, open(tmp_path / "bal.json", "w"))
    json.dump({"allreduce": {"256": {"median_us": 15.0}}}, open(tmp_path / "ar.json", "w"))
    out = _tool("predict_scaling.py", "--bench", str(tmp_path / "n1.json"), "--balance", str(tmp_path / "bal.json"),
                "--allreduce", str(tmp_path / "ar.json"), "--per-call", f"2={tmp_path / 'n2.json'}")
    c = json.loads(out)["curve"]["2"]
    imb = 1.02 / 1.01
    t = 5.0 * imb + 0.4 / 2 + (15.0 + 2 * 2.5) * 1e-3
    assert abs(c["step_ms"] - round(t, 4)) < 1e-9
    assert abs(c["efficiency"] - round(8.0 / t * 1e3 / (2 * 800.0), 3)) <= 1e-3
