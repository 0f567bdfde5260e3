"""Kernel statistics from a rocprofv3 results database (the default rocpd SQLite output):

    python profiles/rocpd_stats.py RUN_results.db OUT_PREFIX

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
    con = sqlite3.connect(db)
    by_name, by_grid = defaultdict(list), defaultdict(list)
    for name, gx, wx, dur in con.execute(
            "select name, grid_x, workgroup_x, duration from kernels"):
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
