"""Host split of one planning frame (tools/time_frame.py's scene, GPU box, repo root): where
compute_prediction_controls spends its host time -- before the graph launch, the launch call,
waiting for the records, the 9-tuple, waiting for the QP, the rest."""
import os
import sys
import time

ROOT = os.getcwd()
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ccmpc import episode, mpc, planner, step  # noqa: E402

O, N, ph = 4, 5000, 8
dev = torch.device("cuda", 0)
init, pmf, gmm = episode.synthetic_gmm(O, T=ph, seed=20251015)
minpos = np.array([150.0, -120.0])
pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]]) for o in range(O)]
x_init = np.array([100.0, -20.0, 0.0, 6.0])
ref = np.stack([100.0 + 3.0 * np.arange(1, ph + 1), np.full(ph, -20.0)], 1)
goal = np.array([126.0, -20.0])
agent = planner.MidlevelAgent(prediction_horizon=ph, device=dev)
marks = []
pc = time.perf_counter


def wrap(cls, name, tag):
    f = getattr(cls, name)

    def g(*a, **k):
        marks.append((tag + ">", pc()))
        r = f(*a, **k)
        marks.append((tag + "<", pc()))
        return r
    setattr(cls, name, g)


wrap(step.StepGraph, "launch", "launch")
wrap(step.StepGraph, "wait", "records")
wrap(mpc.PlanningQPStep, "wait", "qp")
wrap(planner.MidlevelAgent, "_step_tuple", "tuple")
wrap(planner.MidlevelAgent, "_graph_step", "graph_step")
wrap(step.StepGraph, "set_inputs", "set_inputs")
wrap(mpc.PlanningQPStep, "prepare", "prepare")
wrap(planner.MidlevelAgent, "_cell_risk_host", "risk")
wrap(step.Pack, "snapshot", "snapshot")
wrap(planner.HalfSpaceList, "__init__", "hslist")


def frame(i):
    return agent.compute_prediction_controls(0, ph, True, dict(init_state=init, latent_pmf=pmf,
                                             gmm=gmm, N=N, seed=i), minpos, pasts, x_init,
                                             goal, ref)


for i in range(50):
    frame(i)
acc = {}
for i in range(300):
    marks.clear()
    t0 = pc()
    frame(100 + i)
    t1 = pc()
    m = dict(marks)
    seg = {"pre-launch": m["launch>"] - t0, "  to _graph_step": m["graph_step>"] - t0,
           "  risk": m["risk<"] - m["risk>"], "  set_inputs": m["set_inputs<"] - m["set_inputs>"],
           "  qp prepare": m["prepare<"] - m["prepare>"],
           "  rest of _graph_step": (m["launch>"] - m["graph_step>"]) - (m["risk<"] - m["risk>"])
           - (m["set_inputs<"] - m["set_inputs>"]) - (m["prepare<"] - m["prepare>"]), "launch call": m["launch<"] - m["launch>"],
           "launch -> wait": m["records>"] - m["launch<"],
           "records wait": m["records<"] - m["records>"],
           "  snapshot": m["snapshot<"] - m["snapshot>"],
           "  records< -> snapshot>": m["snapshot>"] - m["records<"],
           "  snapshot< -> hslist>": m["hslist>"] - m["snapshot<"],
           "  hslist": m["hslist<"] - m["hslist>"],
           "  hslist< -> tuple>": m["tuple>"] - m["hslist<"],
           "records -> tuple": m["tuple>"] - m["records<"],
           "tuple": m["tuple<"] - m["tuple>"], "tuple -> qp wait": m["qp>"] - m["tuple<"],
           "qp wait": m["qp<"] - m["qp>"], "after qp": t1 - m["qp<"], "total": t1 - t0}
    for k, v in seg.items():
        acc.setdefault(k, []).append(v * 1e6)
for k, v in acc.items():
    print(f"{k:18s} median {np.median(v):7.1f} us")

if len(sys.argv) > 1 and sys.argv[1] == "profile":
    import cProfile
    import pstats
    prof = cProfile.Profile()
    prof.enable()
    for i in range(300):
        frame(1000 + i)
    prof.disable()
    pstats.Stats(prof).sort_stats("tottime").print_stats(40)
