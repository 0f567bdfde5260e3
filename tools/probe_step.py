"""One drop-in planning step on one clock (needs the PROBE=4 build, via
CCMPC_LIB=cc-mpc_amd/csrc/build_p4/libccmpc.so): every workgroup of the sampler, the three
bucketing kernels and the Minkowski cycle stamps s_memrealtime (100 MHz) at its phase
boundaries, so one replay of the captured step graph shows each kernel's span, its phases and
the gaps between kernels.

    python tools/probe_step.py [--direct] [--N 5000] [--O 4]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def med(x):
    return f"{np.median(x) / 100:6.2f}"


def table(fn, *args, wg=4096):
    buf = np.zeros(wg * 8, np.uint64)
    assert fn(buf.ctypes.data_as(ctypes.c_void_p), *args) == 0
    ts = buf.reshape(wg, 8).astype(np.int64)
    return ts[ts[:, 0] > 0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--direct", action="store_true", help="bound C-ABI calls, not the graph")
    ap.add_argument("--N", type=int, default=5000)
    ap.add_argument("--O", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from ccmpc import engine, episode, planner
    dev = torch.device("cuda", 0)
    O, N, ph = a.O, a.N, 8
    init, pmf, gmm = episode.synthetic_gmm(O, T=ph, seed=20251015)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]]) for o in range(O)]
    K = [int(np.count_nonzero(pmf[o] > 0.1)) for o in range(O)]
    eps = np.full((O, max(K)), 0.05 / O)
    ref = np.array([[165.0 + 4.0 * (t + 1), -72.0 + 0.5 * (t + 1)] for t in range(ph)])
    agent = planner.MidlevelAgent(prediction_horizon=ph, device=dev)
    for s in range(3):
        agent.predict_and_constrain(episode.Params(O, K, 0), dict(
            init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=s), eps, ph, ref, minpos, pasts)
    g = next(iter(agent._graphs.values()))
    lib = engine._lib.load()
    for name, nargs in (("ccmpc_probe_sampler_timestamps", 2), ("ccmpc_probe_fused_timestamps", 3),
                        ("ccmpc_probe_bucket_timestamps", 3), ("ccmpc_probe_timestamps", 2),
                        ("ccmpc_probe_l4_split_timestamps", 3)):
        f = getattr(lib, name)
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * (nargs - 1)
    for rep in range(a.reps):
        assert lib.ccmpc_probe_sampler_timestamps(None, 1) == 0
        for w in range(5):
            assert lib.ccmpc_probe_fused_timestamps(None, w, 1) == 0
        for w in range(3):
            assert lib.ccmpc_probe_bucket_timestamps(None, w, 1) == 0
        assert lib.ccmpc_probe_timestamps(None, 1) == 0
        for w in range(2):
            assert lib.ccmpc_probe_l4_split_timestamps(None, w, 1) == 0
        torch.cuda.synchronize()
        g.launch(direct=a.direct)
        g.wait()
        torch.cuda.synchronize()
        ks = [("sampler", table(lib.ccmpc_probe_sampler_timestamps, 0),
               ["staged", "z", "actions", "chain"]),
              ("latents", table(lib.ccmpc_probe_fused_timestamps, 0, 0), ["drawn"]),
              ("place", table(lib.ccmpc_probe_fused_timestamps, 1, 0),
               ["loaded/counted", "acted", "terms/sincos", "chained", "summed"]),
              ("rares", table(lib.ccmpc_probe_fused_timestamps, 2, 0),
               ["loaded", "centres", "keyed", "bins", "ranked", "copied"]),
              ("r.keys", table(lib.ccmpc_probe_fused_timestamps, 3, 0),
               ["loaded", "superblocks", "centres", "keyed"]),
              ("r.copy", table(lib.ccmpc_probe_fused_timestamps, 4, 0),
               ["loaded", "counted", "ranked", "copied"]),
              ("b.stats", table(lib.ccmpc_probe_bucket_timestamps, 0, 0),
               ["loaded", "published", "chunk last", "chunk done", "last", "done"]),
              ("b.hist", table(lib.ccmpc_probe_bucket_timestamps, 1, 0),
               ["loaded", "published", "chunk last", "chunk done", "last", "done"]),
              ("b.scatter", table(lib.ccmpc_probe_bucket_timestamps, 2, 0),
               ["loaded", "done"]),
              ("cycle", table(lib.ccmpc_probe_timestamps, 0, wg=8192), None),
              ("l4.pass1", table(lib.ccmpc_probe_l4_split_timestamps, 0, 0),
               ["loop", "published", "done"]),
              ("l4.pass2", table(lib.ccmpc_probe_l4_split_timestamps, 1, 0),
               ["located", "loop", "done"])]
        if not len(ks[-1][1]):      # one launch (l4_fused_kernel): its stamps are table 0's
            ks[-2] = ("l4.fused", ks[-2][1], ["p1 loop", "p1 published", "p1 done", "p2 prep",
                                              "theta seen", "p2 done"])
        ks = [k for k in ks if len(k[1])]
        t0 = ks[0][1][:, 0].min()
        print(f"--- replay {rep} ({'direct' if a.direct else 'graph'}), N={N}, times in us "
              "from the first kernel's first workgroup start")
        prev_end = None
        for name, ts, slots in ks:
            if len(ts) == 0:
                print(f"{name:10s} no stamps")
                continue
            nz = np.where(ts[:, :7] > 0, ts[:, :7], np.nan)
            first, last = np.nanmin(nz[:, 0]), np.nanmax(nz)
            starts = ts[:, 0]
            gap = "" if prev_end is None else f" gap {(first - prev_end) / 100:5.2f}"
            print(f"{name:10s} {len(ts):4d} WGs  first start {(first - t0) / 100:6.2f}  "
                  f"last start {(starts.max() - t0) / 100:6.2f}  last end "
                  f"{(last - t0) / 100:6.2f}  span {(last - first) / 100:5.2f}{gap}")
            if slots:
                cols = []
                for k, sname in enumerate(slots, start=1):
                    sel = ts[:, k] > 0
                    if sel.any():
                        d = ts[sel, k] - ts[sel, k - 1]
                        cols.append(f"{sname} {med(d)} (max {d.max() / 100:5.2f}, n {sel.sum()})")
                print("           " + " | ".join(cols))
            prev_end = last


if __name__ == "__main__":
    main()
