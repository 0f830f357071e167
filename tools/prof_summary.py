"""Summarise a rocprofv3 --kernel-trace --stats run into profiles/.

usage: python tools/prof_summary.py <rocprof output dir> <out.csv> [name filter]
Reads either the SQLite database (default output) or *_kernel_stats.csv
(--output-format csv) and writes name, calls, total_us, avg_us, pct.
"""
import csv
import glob
import os
import sqlite3
import sys


def rows_from_dir(d):
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        with open(stats[0]) as f:
            for r in csv.DictReader(f):
                yield (r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                       float(r["AverageNs"]) / 1e3, float(r["Percentage"]))
        return
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    c = sqlite3.connect(dbs[0])
    for name, calls, tot, avg, pct in c.execute("select * from top_kernels"):
        # top_kernels reports durations in microseconds
        yield name, int(calls), float(tot), float(avg), float(pct)


def main():
    src, out = sys.argv[1], sys.argv[2]
    flt = sys.argv[3] if len(sys.argv) > 3 else None
    rows = [r for r in rows_from_dir(src) if not flt or flt in r[0]]
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "pct_of_profiled_gpu_time"])
        for name, calls, tot, avg, pct in rows:
            w.writerow([name[:160], calls, f"{tot:.1f}", f"{avg:.3f}", f"{pct:.2f}"])
    for r in rows[:12]:
        print(f"{r[3]:10.3f} us x {r[1]:6d}  {r[0][:90]}")


if __name__ == "__main__":
    main()
