"""cProfile of the v8 MILP frames (bench.py's v8_milp scenes, GPU box, repo root) in steady
state, each frame on a fresh scene: where the host's share of a frame goes.    python tools/profile_milp_host.py"""
import cProfile
import os
import pstats
import sys

ROOT = os.getcwd()
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]
import torch  # noqa: E402

from ccmpc import milp, ovehicle, synthetic  # noqa: E402
from ccmpc.standins import AttrDict  # noqa: E402

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
    agent.do_highlevel_control(params, ovs)
    cases.append((agent, params, (cells, pasts)))
torch.cuda.synchronize(dev)


def fresh(cp):   # a new scene of the same particles (its L4 computed inside the frame)
    cells, pasts = cp
    return ovehicle.scene_from_positions([[c] for c in cells], [p.reshape(1, 2) for p in pasts],
                                         device=dev)


def frames():
    for _ in range(20):
        for agent, params, cp in cases:
            agent.do_highlevel_control(params, fresh(cp))


cProfile.run("frames()", "/tmp/milp.prof")
st = pstats.Stats("/tmp/milp.prof")
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumtime").print_stats(25)
