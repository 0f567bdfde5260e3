"""Summarise rocprofv3 CSV output of profiles/collect.sh into profiles/<round>/.

summary.json per kernel (name prefix):
  calls, avg_ns, min_ns, max_ns                      from the --kernel-trace --stats pass
  fetch_bytes_avg = FETCH_SIZE[KB] * 1024 * 2        gfx950 reports half the bytes of wide
                                                     coalesced reads (MI355X_MICROARCH.md HBM)
  write_bytes_avg = WRITE_SIZE[KB] * 1024
  hbm_bytes_avg   = fetch + write                    per launch
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys


def find(pattern):
    hits = glob.glob(pattern, recursive=True)
    return hits[0] if hits else None


def per_kernel_counter(path, counter):
    vals = {}
    if not path:
        return vals
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name", row.get("Counter-Name")) != counter:
                continue
            name = row.get("Kernel_Name", row.get("Kernel-Name", ""))
            vals.setdefault(name, []).append(float(row.get("Counter_Value", row.get("Counter-Value"))))
    return vals


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    stats_csv = find(os.path.join(src, "trace", "**", "*kernel_stats.csv"))
    out = {}
    if stats_csv:
        shutil.copy(stats_csv, os.path.join(dst, "kernel_stats.csv"))
        with open(stats_csv) as f:
            for row in csv.DictReader(f):
                out[row["Name"]] = dict(calls=int(row["Calls"]), avg_ns=float(row["AverageNs"]),
                                        min_ns=float(row["MinNs"]), max_ns=float(row["MaxNs"]))
    fetch = per_kernel_counter(find(os.path.join(src, "fetch", "**", "*counter_collection.csv")),
                               "FETCH_SIZE")
    write = per_kernel_counter(find(os.path.join(src, "write", "**", "*counter_collection.csv")),
                               "WRITE_SIZE")
    for name, v in fetch.items():
        d = out.setdefault(name, {})
        d["fetch_bytes_avg"] = statistics.mean(v) * 1024 * 2
        d["fetch_size_kb_raw_avg"] = statistics.mean(v)
    for name, v in write.items():
        d = out.setdefault(name, {})
        d["write_bytes_avg"] = statistics.mean(v) * 1024
    for d in out.values():
        if "fetch_bytes_avg" in d and "write_bytes_avg" in d:
            d["hbm_bytes_avg"] = d["fetch_bytes_avg"] + d["write_bytes_avg"]
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    for name, d in sorted(out.items(), key=lambda kv: -kv[1].get("avg_ns", 0))[:8]:
        print(f"{name[:90]:90s} {d}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
