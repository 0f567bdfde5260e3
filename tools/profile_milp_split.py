"""Host / device split of the v8 MILP frame (bench.py's v8_milp scenes, GPU box, repo root):
wall time per frame and, summed over its rounds, the host-side pieces (records, violations and
the tree) against the round trip of the batched QP (copy-in, solve, copy-out, poll)."""
import os
import sys
import time

ROOT = os.getcwd()
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]
import torch  # noqa: E402

from ccmpc import milp, ovehicle, synthetic  # noqa: E402
from ccmpc.standins import AttrDict  # noqa: E402

acc = {}


def timed(cls, name):
    f = getattr(cls, name)

    def w(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
        return r
    setattr(cls, name, w)


for cls, name in ((milp.MilpBnB, "_records"), (milp.MilpBnB, "_violations"),
                  (milp._RoundIO, "run"), (milp.MilpBnB, "_solve_batch"),
                  (milp.MilpBnB, "solve"), (milp.MidlevelAgentV8, "compute_obstacle_constraints")):
    timed(cls, name)

dev = torch.device("cuda", 0)
T, O = 8, 2
cases = []
for seed in range(20, 28):
    cells, K, ref, goal, x_init, pasts = synthetic.crossing_scene(seed, O=O, N=600, T=T, K=1,
                                                                  lateral=6.0)
    ovs = ovehicle.scene_from_positions([[c] for c in cells], [p.reshape(1, 2) for p in pasts],
                                        device=dev)
    agent = milp.MidlevelAgentV8(prediction_horizon=T, control_horizon=T, device=dev)
    params = AttrDict(x_init=x_init, goal=goal, diag=milp.ego_diag(3.7, 1.79), O=O, K=K)
    agent.do_highlevel_control(params, ovs)
    cases.append((agent, params, ovs))
torch.cuda.synchronize(dev)
for rep in range(3):
    acc.clear()
    t0 = time.perf_counter()
    for agent, params, ovs in cases:
        agent.do_highlevel_control(params, ovs)
    wall = time.perf_counter() - t0
    print(f"rep {rep}: {1e3 * wall / len(cases):.3f} ms per frame; per frame: " +
          ", ".join(f"{k} {1e3 * v / len(cases):.3f}" for k, v in acc.items()), flush=True)
