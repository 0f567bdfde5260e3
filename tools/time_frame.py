"""One planning frame at the C2 shape (4 OVs x 5000, ph = T = 8, the Minkowski step + the QP)
on the host clock: compute_prediction_controls (the QP captured inside the step graph) against
the same frame as predict_and_constrain followed by solve_planning_qp (GPU box, repo root)."""
import os
import sys
import time

ROOT = os.getcwd()
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]
import numpy as np
import torch

from ccmpc import episode, planner

O, N, ph = 4, 5000, 8
dev = torch.device("cuda", 0)
init, pmf, gmm = episode.synthetic_gmm(O, T=ph, seed=20251015)
minpos = np.array([150.0, -120.0])
pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]]) for o in range(O)]
K = [int(np.count_nonzero(pmf[o] > 0.1)) for o in range(O)]
x_init = np.array([100.0, -20.0, 0.0, 6.0])       # clear of the OVs: every frame feasible
ref = np.stack([100.0 + 3.0 * np.arange(1, ph + 1), np.full(ph, -20.0)], 1)
goal = np.array([126.0, -20.0])
agent = planner.MidlevelAgent(prediction_horizon=ph, device=dev)


def sampler(i):
    return dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=i)


def frame(i):
    return agent.compute_prediction_controls(0, ph, True, sampler(i), minpos, pasts, x_init,
                                             goal, ref)


def split(i):
    eps = np.full((O, max(K)), 0.05 / O)
    params = episode.Params(O, K, 0)
    agent.predict_and_constrain(params, sampler(i), eps, ph, ref, minpos, pasts)
    return agent.solve_planning_qp(x_init, goal, ref, ph, lon=agent.ego_lon)


for name, fn in (("frame (QP inside the step graph)", frame), ("split (step, then QP)", split),
                 ("frame (QP inside the step graph)", frame), ("split (step, then QP)", split)):
    for i in range(30):
        fn(i)
    ts = []
    for i in range(300):
        t0 = time.perf_counter()
        fn(100 + i)
        ts.append(time.perf_counter() - t0)
    ts = np.array(ts) * 1e6
    print(f"{name:36s} median {np.median(ts):7.1f} us  p90 {np.percentile(ts, 90):7.1f} us",
          flush=True)
frame(7)
ca = agent.last_ctrl["u"].copy()
split(7)
cb = agent.solve_planning_qp(x_init, goal, ref, ph, lon=agent.ego_lon)["u"]
print("same u:", np.array_equal(ca, cb), float(np.abs(ca - cb).max()))
