"""Per-workgroup phase timeline of one moments / cycle launch (needs the PROBE=4 build of
libccmpc.so copied over the real one; see tools/probe_variants.sh).

Slots (s_memrealtime, 100 MHz): 0 start, 1 located, 2 wave 0's stream loop done,
3 combined + published, 4 tree climbed (or gave up), 5 finalised, 6 half-spaces done.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd"), os.path.join(ROOT, "tools")]

import torch  # noqa: E402

from ccmpc import _lib, engine  # noqa: E402
from probe_moments import CONFIGS, build  # noqa: E402

SLOTS, MAXWG = 8, 8192


def stats(x):
    x = np.asarray(x, float) / 100.0  # us
    if x.size == 0:
        return "-"
    return f"min {x.min():6.2f} med {np.median(x):6.2f} max {x.max():6.2f} (n={x.size})"


def one(name, what, dev, lib, back_to_back=1):
    store, cyc = build(name, dev)
    fn = cyc.run if what == "cycle" else (lambda: engine.moments(store, cyc.mean, cyc.cov, cyc.ws))
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    buf = np.zeros(MAXWG * SLOTS, np.uint64)
    assert lib.ccmpc_probe_timestamps(None, 1) == 0
    for _ in range(back_to_back):  # the table keeps the last launch's stamps
        fn()
    torch.cuda.synchronize()
    assert lib.ccmpc_probe_timestamps(buf.ctypes.data_as(ctypes.c_void_p), 0) == 0
    ts = buf.reshape(MAXWG, SLOTS).astype(np.int64)
    live = ts[:, 0] > 0
    wg = np.flatnonzero(live)
    ts = ts[live]
    t0 = ts[:, 0].min()
    rel = np.where(ts > 0, ts - t0, -1)
    end = rel[:, :7].max()
    fin = rel[:, 5] >= 0
    print(f"== {name} {what} (last of {back_to_back} back-to-back): {live.sum()} WGs, "
          f"kernel span {end / 100:.2f} us")
    print("  start      ", stats(rel[:, 0]))
    print("  locate     ", stats(rel[:, 1] - rel[:, 0]))
    print("  loop end   ", stats(rel[:, 2]))
    print("  loop dur   ", stats(rel[:, 2] - rel[:, 1]))
    print("  combine    ", stats(rel[:, 3] - rel[:, 2]))
    print("  climb(non) ", stats((rel[:, 4] - rel[:, 3])[~fin]))
    print("  climb(last)", stats((rel[:, 4] - rel[:, 3])[fin]))
    if os.environ.get("PROBE16"):  # PROBE=20 build: slot 7 = the root gather's end
        g = fin & (rel[:, 7] >= 0)
        print("  gather     ", stats((rel[:, 7] - rel[:, 4])[g]))
        print("  finalize   ", stats((rel[:, 5] - rel[:, 7])[g]))
    print("  finalise   ", stats((rel[:, 5] - rel[:, 4])[fin]))
    print("  fin at     ", stats(rel[fin, 5]))
    if what == "cycle":
        print("  halfspaces ", stats((rel[:, 6] - rel[:, 5])[fin]))
        order = np.argsort(rel[:, 0])
        print("  slowest starters:", [int(b) for b in order[-10:]])
    print("  end at     ", stats(np.maximum(rel[:, 4], rel[:, 6])))
    if os.environ.get("BY_XCD"):  # dispatch places workgroup i on XCD i % 8
        for x in range(8):
            m = (wg % 8) == x
            print(f"  xcd {x}: start {stats(rel[m, 0])} | loop dur {stats((rel[:, 2] - rel[:, 1])[m])}")


def main():
    """python tools/probe_phases.py [NAME:moments|cycle ...] (default: every config's moments,
    then the C2 cycle)."""
    dev = torch.device("cuda:0")
    lib = _lib.load()
    lib.ccmpc_probe_timestamps.restype = ctypes.c_int
    lib.ccmpc_probe_timestamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    jobs = [a.split(":") for a in sys.argv[1:]] or (
        [(n, "moments") for n in CONFIGS] + [("C2", "cycle")])
    for name, what in jobs:
        one(name, what, dev, lib, back_to_back=5)


if __name__ == "__main__":
    main()
