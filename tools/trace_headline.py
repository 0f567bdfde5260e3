"""The headline launches of one `bench.py` run from its rocprofv3 kernel-trace database:
per launch of the C2 cycle kernel (in dispatch order) its duration and the gap from the previous
launch's end, so the timed window's first-launch and clock effects show.

    python tools/trace_headline.py RUN_results.db [first] [count]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    count = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    start = "start" if "start" in cols else "start_ns"
    end = "end" if "end" in cols else "end_ns"
    rows = con.execute(f"select name, grid_x, {start}, {end} from kernels order by {start}").fetchall()
    prev = None
    k = 0
    for name, gx, s, e in rows:
        if "moments_kernel<double, 1, true" not in name:
            prev = e
            continue
        if first <= k < first + count:
            gap = (s - prev) / 1000 if prev is not None else float("nan")
            print(f"{k:4d} grid {gx:6d} dur {(e - s) / 1000:7.2f} us  gap {gap:9.2f} us")
        prev = e
        k += 1
    print("launches", k)


if __name__ == "__main__":
    main()
