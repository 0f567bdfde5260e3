"""Debug probe: one scene's ccmpc_mpc_qp with a given max_iter; run it against the
CCMPC_QP_TRACE build to see the IPM's residuals per iteration.
usage: qp_debug.py SEED KIND(h|a) MAX_ITER..."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from ccmpc import cycle, engine, mpc
from _qp_inputs import crossing_scene
dev = torch.device("cuda", 0)
T = 8
seed, kind = int(sys.argv[1]), sys.argv[2]
MIS = [int(a) for a in sys.argv[3:]] or [60]
ovs, cells, K, ref, goal, x0 = crossing_scene(seed, T=T)
store = engine.ParticleStore.from_cells(cells, device=dev)
cyc = (cycle.MinkowskiCycle if kind == "h" else cycle.AffineCycle)(store, K, ref)
cyc.run()
xbar, gamma = mpc.ltv(x0[None], T, lon=3.7)
g = torch.as_tensor(goal[None], device=dev)
r = torch.as_tensor(ref[None], device=dev)
for mi in MIS:
    qp = mpc.PlanningQP([len(cells)], T, max_iter=mi, u_order=int(os.environ.get("ORDER", "0")),
                        kind=mpc.REC_HALFSPACE if kind == "h" else mpc.REC_AFFINE)
    u, X, cost, st, it = qp.solve(gamma, xbar, g, r, cyc.rec)
    print(seed, kind, mi, int(st[0]), int(it[0]), float(cost[0]), u[0].cpu().numpy().round(3))
