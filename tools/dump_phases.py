"""Raw per-workgroup phase stamps (+ hardware ids, slot 7) of one moments / cycle launch to an
.npz for offline analysis (PROBE=4 build): python tools/dump_phases.py C4 moments out.npz"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd"), os.path.join(ROOT, "tools")]

import torch  # noqa: E402

from ccmpc import _lib, engine  # noqa: E402
from probe_moments import build  # noqa: E402


def main():
    name, what, out = sys.argv[1], sys.argv[2], sys.argv[3]
    dev = torch.device("cuda:0")
    lib = _lib.load()
    lib.ccmpc_probe_timestamps.restype = ctypes.c_int
    lib.ccmpc_probe_timestamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    store, cyc = build(name, dev)
    fn = cyc.run if what == "cycle" else (lambda: engine.moments(store, cyc.mean, cyc.cov, cyc.ws))
    reps = []
    for r in range(6):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        assert lib.ccmpc_probe_timestamps(None, 1) == 0
        fn()
        torch.cuda.synchronize()
        buf = np.zeros(8192 * 8, np.uint64)
        assert lib.ccmpc_probe_timestamps(buf.ctypes.data_as(ctypes.c_void_p), 0) == 0
        reps.append(buf.reshape(8192, 8).copy())
    np.savez(out, ts=np.stack(reps), counts=np.asarray(store.counts),
             offsets=np.asarray(store.offsets))
    print("saved", out)


if __name__ == "__main__":
    main()
