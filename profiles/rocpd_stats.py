"""Kernel statistics from a rocprofv3 results database (the default rocpd SQLite output) or
from its CSV kernel trace (--output-format csv):

    python profiles/rocpd_stats.py RUN_results.db|RUN_kernel_trace.csv OUT_PREFIX

writes OUT_PREFIX_kernel_stats.csv (name, calls, total / average / median / min / max ns) and
OUT_PREFIX_by_grid.csv (the same per (kernel, grid size, workgroup size): one bench line's
launches apart from the other configurations that share the kernel instance).
"""
import csv
import sqlite3
import statistics
import sys
from collections import defaultdict


def main():
    db, prefix = sys.argv[1], sys.argv[2]
    by_name, by_grid = defaultdict(list), defaultdict(list)
    if db.endswith(".csv"):
        rows = ((r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]),
                 int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                for r in csv.DictReader(open(db)))
    else:
        rows = sqlite3.connect(db).execute(
            "select name, grid_x, workgroup_x, duration from kernels")
    for name, gx, wx, dur in rows:
        by_name[name].append(dur)
        by_grid[(name, gx, wx)].append(dur)

    def row(v):
        return [len(v), sum(v), round(statistics.mean(v), 1), round(statistics.median(v), 1),
                min(v), max(v)]
    with open(prefix + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["name", "calls", "total_ns", "avg_ns", "median_ns", "min_ns", "max_ns"])
        for name, v in sorted(by_name.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name] + row(v))
    with open(prefix + "_by_grid.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["name", "grid_x", "workgroup_x", "calls", "total_ns", "avg_ns", "median_ns",
                     "min_ns", "max_ns"])
        for (name, gx, wx), v in sorted(by_grid.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, gx, wx] + row(v))


if __name__ == "__main__":
    main()
