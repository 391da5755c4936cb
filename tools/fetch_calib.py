"""FETCH_SIZE / WRITE_SIZE calibration factors from tools/fetch_calib (see that file):

    python3 tools/fetch_calib.py FETCH_DIR WRITE_DIR BYTES.json OUT.json

For each calibration kernel: counted bytes (counter KiB x 1024) and the factor true / counted.
tools/pmc_summary.py multiplies the train kernel's FETCH_SIZE by the dword-read factor (its reads
are dword-wide) and its WRITE_SIZE by the record-pattern factor (write_rec: the partial records are written, then
half of their columns read-modified-written).
"""
import json
import sys

from pmc_summary import per_kernel


def main():
    fetch_dir, write_dir, bytes_json, out = sys.argv[1:5]
    true = json.loads(open(bytes_json).read().strip().splitlines()[-1])
    f = per_kernel(fetch_dir, "FETCH_SIZE")
    w = per_kernel(write_dir, "WRITE_SIZE")
    res = {}
    for name, nbytes in true.items():
        src = f if name.startswith("read") else w
        vals = [v for k, v in src.items() if k.split("(")[0].strip() == name or k.startswith(name + "(")]
        if not vals:
            raise SystemExit(f"{name}: not in the counter CSVs")
        counted = vals[0][0] * 1024.0
        res[name] = {"bytes": nbytes, "counted_bytes": counted, "factor": nbytes / counted}
    data = {"kernels": res, "read_dword_factor": res["read_dword"]["factor"],
            "read_f3_factor": res["read_f3"]["factor"], "write_dword_factor": res["write_dword"]["factor"],
            "write_rec_factor": res["write_rec"]["factor"],
            "note": "factor = true bytes / (counter KiB x 1024); tools/fetch_calib.hip, one dispatch each"}
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps(data))


if __name__ == "__main__":
    main()
