"""Synthetic planning-step scenes for the QP tests: ccmpc.synthetic.crossing_scene (obstacle
clouds that cross the ego's path, so half-spaces bind), wrapped as the oracle's OVehicles."""
import functools

import numpy as np

from ccmpc import synthetic
from oracle import ccmpc_oracle as orc
from oracle import mpc_oracle as mo

LON = 3.7


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


@functools.lru_cache(maxsize=None)
def classify(seed, T=8, order="F"):
    """'infeasible', 'binding' (an obstacle half-space is active at the optimum) or 'free':
    the oracle's QP on the scene's oracle records."""
    ovs, cells, K, ref, goal, x0 = crossing_scene(seed, T=T)
    out = orc.minkowski_generator(ovs, T, T, ref, with_l4=False)
    xbar, _, G, _, _ = mo.VehicleModel(T, 0.5, 0.5 * LON, LON).get_optimization_ltv(
        x0, np.zeros(2))
    r = mo.solve_step(G, xbar, T, T, goal, ref, out["records"], "halfspace",
                      mo.DEFAULT_PARAMS, order=order)
    if not r["feasible"]:
        return "infeasible"
    return "binding" if any(a >= 6 * T for a in r["active"]) else "free"


def pick_seeds(kind, count, start=0, T=8, limit=400):
    """The first `count` seeds from `start` whose scene classifies as `kind`."""
    out = []
    for s in range(start, start + limit):
        if classify(s, T) == kind:
            out.append(s)
            if len(out) == count:
                return out
    raise RuntimeError(f"fewer than {count} {kind!r} scenes in seeds {start}..{start + limit}")
