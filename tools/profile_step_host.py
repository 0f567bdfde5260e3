"""Host-side profile of the planning step (the drop-in C2 step, predict_and_constrain at
Tsh == ph): cProfile over 300 steps, the functions by own time (GPU box, repo root)."""
import cProfile
import os
import pstats
import sys
import time

ROOT = "/root/repo" if os.path.exists("/root/repo/bench.py") else os.getcwd()
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
eps = np.full((O, max(K)), 0.05 / O)
ref = np.array([[165.0 + 4.0 * (t + 1), -72.0 + 0.5 * (t + 1)] for t in range(ph)])
agent = planner.MidlevelAgent(prediction_horizon=ph, device=dev)
params = episode.Params(O, K, 0)


def step(i):
    return agent.predict_and_constrain(params, dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N,
                                                    seed=i), eps, ph, ref, minpos, pasts)


for i in range(30):
    step(i)
n = 300
t0 = time.perf_counter()
for i in range(n):
    step(100 + i)
print(f"plain: {(time.perf_counter() - t0) / n * 1e6:.1f} us/step")
pr = cProfile.Profile()
pr.enable()
for i in range(n):
    step(1000 + i)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(40)
