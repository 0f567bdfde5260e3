"""Workgroup placement vs finish time of one moments launch (PROBE=4 build copied over the
real libccmpc.so, as tools/probe_timeline.sh does).  Slot 7 holds XCC_ID:HW_ID of the
workgroup's first wave; the per-CU workgroup count is set against each workgroup's stream
loop duration and end time.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd"), os.path.join(ROOT, "tools")]

import torch  # noqa: E402

from ccmpc import _lib, engine  # noqa: E402
from probe_moments import build  # noqa: E402

SLOTS, MAXWG = 8, 8192


def main(name="C4", what="moments"):
    dev = torch.device("cuda:0")
    lib = _lib.load()
    lib.ccmpc_probe_timestamps.restype = ctypes.c_int
    lib.ccmpc_probe_timestamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    store, cyc = build(name, dev)
    fn = cyc.run if what == "cycle" else (lambda: engine.moments(store, cyc.mean, cyc.cov, cyc.ws))
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    for rep in range(3):
        buf = np.zeros(MAXWG * SLOTS, np.uint64)
        assert lib.ccmpc_probe_timestamps(None, 1) == 0
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        assert lib.ccmpc_probe_timestamps(buf.ctypes.data_as(ctypes.c_void_p), 0) == 0
        ts = buf.reshape(MAXWG, SLOTS)
        live = ts[:, 0] > 0
        ts = ts[live]
        hw = (ts[:, 7] & 0xFFFFFFFF).astype(np.int64)
        xcc = (ts[:, 7] >> np.uint64(32)).astype(np.int64) & 0xF
        cu = (hw >> 8) & 0xF
        sh = (hw >> 12) & 0x1
        se = (hw >> 13) & 0x7
        key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
        t = ts[:, :7].astype(np.int64)
        t0 = t[:, 0].min()
        rel = np.where(t > 0, t - t0, -1) / 100.0
        end = np.maximum(rel[:, 4], rel[:, 2])
        uk, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
        per_wg = cnt[inv]
        print(f"== {name} {what} rep {rep}: {len(ts)} WGs on {len(uk)} CUs, span {end.max():.2f} us")
        print("   WGs per CU histogram:", dict(zip(*np.unique(cnt, return_counts=True))))
        print("   WGs per XCC:", np.bincount(xcc, minlength=8).tolist())
        for c in np.unique(per_wg):
            m = per_wg == c
            ld = rel[m, 2] - rel[m, 1]
            print(f"   CU with {c} WGs: n={m.sum():4d}  start med {np.median(rel[m, 0]):6.2f}"
                  f"  loop med {np.median(ld):6.2f} max {ld.max():6.2f}"
                  f"  end med {np.median(end[m]):6.2f} max {end[m].max():6.2f}")
        q = np.percentile(end, [10, 50, 90, 99, 100])
        print("   end percentiles 10/50/90/99/100:", np.round(q, 2).tolist())
        q = np.percentile(rel[:, 0], [10, 50, 90, 99, 100])
        print("   start percentiles 10/50/90/99/100:", np.round(q, 2).tolist())


if __name__ == "__main__":
    main(*sys.argv[1:])
