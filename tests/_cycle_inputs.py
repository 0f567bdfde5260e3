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


REFLOOP = ["refloop_o2_t8", "refloop_o1_t12", "refloop_o3_t12", "refloop_o2_t40",
           "refloop_shrink_t7"]


def refloop_inputs(g):
    """A refloop_* fixture (the reference's own generator loops, make_golden.py
    pin_generator_glue): (K, T, ph, cells per OV, yaws per OV (the ones the reference read),
    ideal clouds per cell or None)."""
    T, ph = int(g["T"]), int(g["ph"])
    K = [int(k) for k in g["K"]]
    cells = cells_from_fixture(g)
    yaws, out_c, out_y, j, y0 = g["yaws"], [], [], 0, 0
    for k in K:
        out_c.append(cells[j:j + k])
        ys = []
        for c in cells[j:j + k]:
            ys.append(yaws[y0:y0 + c.shape[0]])
            y0 += c.shape[0]
        out_y.append(ys)
        j += k
    ideal = None
    if "ideal" in g.files:
        ideal, o = [], 0
        for n in g["ideal_counts"]:
            ideal.append(g["ideal"][o:o + n])
            o += n
    return K, T, ph, out_c, out_y, ideal


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
