"""Synthetic planning-step scenes for the QP tests: ccmpc.synthetic.crossing_scene (obstacle
clouds that cross the ego's path, so half-spaces bind), wrapped as the oracle's OVehicles."""
import numpy as np

from ccmpc import synthetic
from oracle import ccmpc_oracle as orc


def crossing_scene(seed, O=2, N=400, T=8, K=2, lateral=8.0):
    """(ovehicles for the oracle, per-cell clouds, K list, ref, goal, x_init)."""
    cells, Ks, ref, goal, x_init, pasts = synthetic.crossing_scene(seed, O=O, N=N, T=T, K=K,
                                                                   lateral=lateral)
    ovs, c0 = [], 0
    for o, k in enumerate(Ks):
        mine = cells[c0:c0 + k]
        c0 += k
        past = pasts[o].reshape(1, 2)
        yaws = [orc._step_yaws(c, past[-1], T) for c in mine]
        centres = np.array([c[:, T - 1].mean(0) for c in mine])
        ovs.append(orc.OVehicle(T, past, np.full(k, 1.0 / k), list(mine), yaws, centres,
                                np.array([4.5, 2.5])))
    return ovs, cells, Ks, ref, goal, x_init
