"""In-process A/B of the planning step's copy-out + signal forms (GPU box, repo root):
CCMPC_STEP_FUSED_SIGNAL=1 (one single-workgroup copy + signal kernel) against 0 (the multi-block
copy kernel, then ccmpc_signal_host), alternating agents, C2 shape.  Prints the host time per
drop-in step and the launch -> records latency, medians."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ccmpc import episode, planner  # noqa: E402

dev = torch.device("cuda", 0)
O, N, ph = 4, 5000, 8
init, pmf, gmm = episode.synthetic_gmm(O, T=ph, seed=20251015)
minpos = np.array([150.0, -120.0])
pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]]) for o in range(O)]
K = [int(np.count_nonzero(pmf[o] > 0.1)) for o in range(O)]
eps = np.full((O, max(K)), 0.05 / O)
ref = np.array([[165.0 + 4.0 * (t + 1), -72.0 + 0.5 * (t + 1)] for t in range(ph)])
params = episode.Params(O, K, 0)
agents = {}
for v in ("1", "0"):
    os.environ["CCMPC_STEP_FUSED_SIGNAL"] = v
    a = planner.MidlevelAgent(prediction_horizon=ph, device=dev)
    for i in range(20):
        a.predict_and_constrain(params, dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N,
                                             seed=i), eps, ph, ref, minpos, pasts)
    agents[v] = a
res = {v: ([], []) for v in agents}
for rnd in range(6):
    for v, a in agents.items():
        g = next(iter(a._graphs.values()))
        for i in range(100):
            t0 = time.perf_counter()
            a.predict_and_constrain(params, dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N,
                                                 seed=1000 + i), eps, ph, ref, minpos, pasts)
            res[v][0].append(time.perf_counter() - t0)
        for i in range(100):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.launch()
            g.wait()
            res[v][1].append(time.perf_counter() - t0)
for v, (st, rp) in res.items():
    print(f"FUSED_SIGNAL={v}: step {statistics.median(st) * 1e6:.1f} us, launch->records "
          f"{statistics.median(rp) * 1e6:.1f} us")
