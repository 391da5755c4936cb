"""Format a rocprofv3 --kernel-trace --stats kernel_stats.csv as the plain table kept under
profiles/ (one line per kernel: calls, average/min/max microseconds, share of kernel time).

    python tools/prof_summary.py <kernel_stats.csv> "<header line>" > profiles/<tag>_kernel_stats.txt
"""
import csv
import sys


def main():
    path, header = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(path)))
    print(header)
    print(f"{'kernel':<72}{'calls':>7}{'avg_us':>11}{'min_us':>11}{'max_us':>11}{'pct':>8}")
    for r in rows:
        name = r["Name"][:70]
        print(f"{name:<72}{int(r['Calls']):>7}{float(r['AverageNs']) / 1e3:>11.2f}{float(r['MinNs']) / 1e3:>11.2f}"
              f"{float(r['MaxNs']) / 1e3:>11.2f}{float(r['Percentage']):>8.2f}")


if __name__ == "__main__":
    main()
