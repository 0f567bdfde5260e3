"""Per-workgroup phase timeline of ccmpc_l4 on the drop-in step's bucketed store (needs the
PROBE=4 build, via CCMPC_LIB=cc-mpc_amd/csrc/build_p4/libccmpc.so).  Slots (100 MHz):
0 start, 1 pass 1 done, 2 theta (block sum), 3 t = 0 variance done, 4 pass 2 done, 5 maxima."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def stats(x):
    x = np.asarray(x, float) / 100.0
    return f"min {x.min():6.2f} med {np.median(x):6.2f} max {x.max():6.2f}"


def main():
    from ccmpc import engine, episode, planner
    dev = torch.device("cuda", 0)
    O, N, ph = 4, 5000, 8
    init, pmf, gmm = episode.synthetic_gmm(O, T=ph, seed=20251015)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]]) for o in range(O)]
    K = [int(np.count_nonzero(pmf[o] > 0.1)) for o in range(O)]
    eps = np.full((O, max(K)), 0.05 / O)
    ref = np.array([[165.0 + 4.0 * (t + 1), -72.0 + 0.5 * (t + 1)] for t in range(ph)])
    agent = planner.MidlevelAgent(prediction_horizon=ph, device=dev)
    agent.predict_and_constrain(episode.Params(O, K, 0), dict(init_state=init, latent_pmf=pmf,
                                gmm=gmm, N=N, seed=1), eps, ph, ref, minpos, pasts)
    g = next(iter(agent._graphs.values()))
    lib, p, o, i, st = engine._lib.load(), engine._p, g.out, g.inp, g.store
    q = g.out_l4s[0]
    lib.ccmpc_probe_l4_timestamps.restype = ctypes.c_int
    lib.ccmpc_probe_l4_timestamps.argtypes = [ctypes.c_void_p, ctypes.c_int]

    def l4():
        engine._lib.check(lib.ccmpc_l4(
            p(st.pos), engine.F32, st.ld, ph, p(st.origin), p(o.d("off")), p(o.d("cnt")), g.C,
            p(i.d("past")), p(i.d("bbox")), p(q.d("A")), p(q.d("b")), p(q.d("yaw_mean")),
            p(q.d("yaw0_var")), None, None, engine._stream()), "ccmpc_l4")
    for _ in range(5):
        l4()
    torch.cuda.synchronize()
    assert lib.ccmpc_probe_l4_timestamps(None, 1) == 0
    l4()
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 8, np.uint64)
    assert lib.ccmpc_probe_l4_timestamps(buf.ctypes.data_as(ctypes.c_void_p), 0) == 0
    ts = buf.reshape(4096, 8).astype(np.int64)
    ts = ts[ts[:, 0] > 0]
    rel = ts - ts[:, 0].min()
    print(f"{len(ts)} WGs, span {rel.max() / 100:.2f} us")
    print("  start     ", stats(rel[:, 0]))
    print("  pass 1    ", stats(rel[:, 1] - rel[:, 0]))
    print("  theta sum ", stats(rel[:, 2] - rel[:, 1]))
    print("  t0 var    ", stats(rel[:, 3] - rel[:, 2]))
    print("  pass 2    ", stats(rel[:, 4] - rel[:, 3]))
    print("  maxima    ", stats(rel[:, 5] - rel[:, 4]))
    print("  end at    ", stats(rel[:, 5]))
    counts = g.out.d("cnt").cpu().numpy()
    order = np.argsort(rel[:, 5])[::-1][:12]
    print("  slowest (wg = cell*T + t: cell count, start, pass1, end):",
          [(int(w), int(counts[w // ph]), round(rel[w, 0] / 100, 1),
            round((rel[w, 1] - rel[w, 0]) / 100, 1), round(rel[w, 5] / 100, 1)) for w in order])
    order = np.argsort(rel[:, 5])[:6]
    print("  fastest:", [(int(w), int(counts[w // ph]), round(rel[w, 0] / 100, 1),
                          round((rel[w, 1] - rel[w, 0]) / 100, 1), round(rel[w, 5] / 100, 1))
                         for w in order])


if __name__ == "__main__":
    main()
