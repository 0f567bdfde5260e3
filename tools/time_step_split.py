import os, sys, time
ROOT = "/root/repo" if os.path.exists("/root/repo/bench.py") else os.getcwd()
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]
import numpy as np, torch
from ccmpc import episode, planner, step
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
for i in range(30):
    agent.predict_and_constrain(params, dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=i), eps, ph, ref, minpos, pasts)
g = next(iter(agent._graphs.values()))
# instrument
marks = {}
orig_launch, orig_wait, orig_snap, orig_set = g.launch, g.wait, g.out.snapshot, g.set_inputs
def wrap(name, f):
    def w(*a, **k):
        t0 = time.perf_counter(); r = f(*a, **k); marks[name] = marks.get(name, 0) + time.perf_counter() - t0; return r
    return w
g.launch, g.wait, g.out.snapshot, g.set_inputs = wrap("launch", orig_launch), wrap("wait", orig_wait), wrap("snapshot", orig_snap), wrap("set_inputs", orig_set)
for name in ("_cell_risk_host", "_step_tuple", "_src_cells_host"):
    if hasattr(agent, name):
        setattr(agent, name, wrap(name.strip("_"), getattr(agent, name)))
n = 300
t0 = time.perf_counter()
for i in range(n):
    agent.predict_and_constrain(params, dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=100+i), eps, ph, ref, minpos, pasts)
tot = (time.perf_counter() - t0) / n
print(f"total {tot*1e6:.1f} us/step")
for k, v in marks.items(): print(f"  {k:12s} {v/n*1e6:7.1f} us")
print(f"  other        {(tot - sum(marks.values())/n)*1e6:7.1f} us")
