"""The planning QP's batch (bench.py planning_qp scenes) under method / policy switches (GPU box):
kernel time, verdicts and iteration counts per setting, so the active-set pass's share and its
hand-overs to the IPM show.

    python tools/qp_probe.py [T] [scenes]

QP_ONE=1: one solve per setting, no timing (for the CCMPC_QP_TRACE build's printf phases).
QP_FIRST=k: start at the batch's scene k (QP_ONE with scenes = 1: that scene alone).
QP_ITERS=1: print every scene's verdict and iteration count (gi default).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    scenes = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    from ccmpc import cycle, engine, mpc, synthetic
    dev = torch.device("cuda", 0)
    cells, K, cps, x0s, goals, refs = [], [], [], [], [], []
    first = int(os.environ.get("QP_FIRST", "0"))   # the batch's scenes first .. first + scenes - 1
    for sc in range(first, first + scenes):
        c, k, ref, goal, x0, _ = synthetic.crossing_scene(20251015 + 5000 + sc, O=2, N=5000, T=T)
        cells += c
        K.append(k)
        cps.append(len(c))
        refs.append(ref)
        goals.append(goal)
        x0s.append(x0)
    store = engine.ParticleStore.from_cells(cells, device=dev)
    cyc = cycle.MinkowskiCycle(store, [k for ks in K for k in ks], np.array(refs), scene_K=K)
    cyc.run()
    xbar, gamma = mpc.ltv(np.array(x0s), T, lon=3.7)
    goal_t = torch.as_tensor(np.array(goals), device=dev)
    ref_t = torch.as_tensor(np.array(refs), device=dev)
    base = None
    for name, env in (("ipm", {"CCMPC_QP_METHOD": "ipm"}), ("gi (default)", {}),
                      ("gi nostep=0", {"CCMPC_QP_GI_NOSTEP": "0"}),
                      ("gi nostep=1", {"CCMPC_QP_GI_NOSTEP": "1"})):
        for k in ("CCMPC_QP_METHOD", "CCMPC_QP_GI_NOSTEP"):
            os.environ.pop(k, None)
        os.environ.update(env)
        qp = mpc.PlanningQP(cps, T)
        fn = lambda: qp.solve(gamma, xbar, goal_t, ref_t, cyc.rec)  # noqa: E731
        if os.environ.get("QP_ONE"):
            print(f"--- {name}", flush=True)
            fn()
            torch.cuda.synchronize()
            t = 0.0
        else:
            t = bench.time_kernel_live(fn, dev, per_graph=5, replays=5)
            fn()
        st, it = qp.status.cpu().numpy(), qp.iters.cpu().numpy()
        if os.environ.get("QP_ITERS") and name == "gi (default)":
            print("scene status iters:", [(i, int(st[i]), int(it[i])) for i in range(len(st))])
        u = qp.u.cpu().numpy()
        ok = st == mpc.QP_OK
        line = (f"{name:14s} {t * 1e6:8.1f} us  solved {ok.sum():3d}  infeasible "
                f"{(st == mpc.QP_MAXITER).sum():3d}  iters ok max {it[ok].max() if ok.any() else -1} "
                f"median {np.median(it[ok]) if ok.any() else -1}  not-ok iters max "
                f"{it[~ok].max() if (~ok).any() else -1}")
        if base is None:
            base = (st, u)
        else:
            same = np.array_equal(st, base[0])
            du = np.abs(u[ok] - base[1][ok]).max() if ok.any() else 0.0
            line += f"  verdicts == ipm: {same}  max |du| {du:.2e}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
