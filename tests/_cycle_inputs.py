"""Rebuild the per-OV inputs of a golden cycle fixture (tests/golden/make_golden.py:make_ovs)."""
import numpy as np

from oracle import ccmpc_oracle as orc


def cells_from_fixture(g):
    counts = g["counts"]
    pos = g["positions"]
    out, o = [], 0
    for c in counts:
        out.append(pos[o:o + c])
        o += c
    return out


def ovehicles_from_fixture(g):
    T = int(g["T"])
    K = [int(k) for k in g["K"]]
    cells = cells_from_fixture(g)
    ovs, j = [], 0
    for o, k in enumerate(K):
        mine = cells[j:j + k]
        j += k
        pmf = np.array([c.shape[0] for c in mine], float)
        pmf /= pmf.sum()
        past = np.asarray(g["past"][o]).reshape(1, 2)
        yaws = [orc._step_yaws(c, past[-1], T) for c in mine]
        centres = np.array([c[:, T - 1].mean(0) for c in mine])
        ovs.append(orc.OVehicle(T, past, pmf, list(mine), yaws, centres, np.array([4.5, 2.5])))
    return ovs
