"""Diagnostic: GPU QP vs oracle per scene at a given T, with KKT residuals of both points."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from ccmpc import mpc
from oracle import mpc_oracle as mo
import test_gpu_mpc as tg
T = int(sys.argv[1]); seeds = list(range(200, 216))
gpu = torch.device("cuda", 0)
rec, cps, o_recs, refs, goals, x0s = tg._scene_inputs(seeds, T, gpu)
xbar, gamma = mpc.ltv(x0s, T, lon=3.7)
qp = mpc.PlanningQP(cps, T)
u, X, cost, st, it = qp.solve(gamma, xbar, torch.as_tensor(goals, device=gpu), torch.as_tensor(refs, device=gpu), rec)
u, st, it = u.cpu().numpy(), st.cpu().numpy(), it.cpu().numpy()
prm = mpc.MPCParams.reference_defaults().as_dict()
for i, s in enumerate(seeds):
    w = tg._oracle_solve(x0s[i], T, goals[i], refs[i], o_recs[i], "halfspace", prm)
    if not w["feasible"]:
        print(s, "infeasible", st[i], it[i]); continue
    kg = mo.kkt_residuals(w["H"], w["f"], w["G"], w["h"], u[i])[:3]
    ko = mo.kkt_residuals(w["H"], w["f"], w["G"], w["h"], w["u"], w["lam"])[:3]
    og = 0.5 * u[i] @ w["H"] @ u[i] + w["f"] @ u[i]; oo = 0.5 * w["u"] @ w["H"] @ w["u"] + w["f"] @ w["u"]
    print(s, st[i], it[i], "du %.2e" % np.abs(u[i] - w["u"]).max(), "gpuKKT", ["%.1e" % v for v in kg],
          "orcKKT", ["%.1e" % v for v in ko], "obj gpu %.6f orc %.6f" % (og, oo))
