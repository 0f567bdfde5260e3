"""v8 MILP big-M obstacle rows (v8/__init__.py:692-724) on the host: BigMRows' expression
list, sparse form and numeric check agree with the oracle restatement (built on the oracle's
golden-pinned L4 over-approximation)."""
import numpy as np
import pytest

from oracle import ccmpc_oracle as orc
from ccmpc import milp


def _scene(seed=0, T=8, K=(2, 1), N=400):
    rng = np.random.default_rng(seed)
    ovs = []
    for o, k_o in enumerate(K):
        past = np.array([[10.0 * o, 5.0]])
        cells = [past[0] + np.cumsum(rng.normal([1.0, 0.3 * k], 0.2, size=(N, T, 2)), axis=1)
                 for k in range(k_o)]
        ovs.append(orc.OVehicle(T, past, np.ones(k_o) / k_o, cells,
                                [orc._step_yaws(c, past[-1], T) for c in cells],
                                np.zeros((k_o, 2)), np.array([4.5, 2.5])))
    return ovs


def _rows_from_oracle(ovs, T, diag):
    _, A_u, b_u = orc.vertices_and_l4(ovs, T)
    A = np.stack([A_u[t][k][o] for o, ov in enumerate(ovs) for k in range(ov.n_states)
                  for t in range(T)]).reshape(-1, T, 4, 2)
    b = np.stack([b_u[t][k][o] for o, ov in enumerate(ovs) for k in range(ov.n_states)
                  for t in range(T)]).reshape(-1, T, 4)
    return A, b


@pytest.mark.parametrize("T_ctrl", [8, 5])
def test_bigm_rows_match_oracle(T_ctrl):
    ph, diag = 8, milp.ego_diag(4.7, 1.9)
    ovs = _scene(T=ph)
    A, b = _rows_from_oracle(ovs, ph, diag)
    rows = milp.BigMRows(A, b, diag, T_ctrl)
    want, holds = orc.milp_obstacle_rows(ovs, T_ctrl, ph, diag)
    assert len(rows) == len(want) * 5
    rng = np.random.default_rng(1)
    for trial in range(4):
        xy = rng.normal([5.0, 5.0], 8.0, size=(T_ctrl, 2))
        delta = rng.integers(0, 2, size=(rows.n_cells, T_ctrl, 4)).astype(float)
        ref = holds(xy, delta)
        got = [bool(v) for v in rows.expr(xy, delta)]
        assert got == ref
        r, c, v, h = rows.coo()
        z = np.concatenate([xy.ravel(), delta.ravel()])
        Gz = np.zeros(h.size)
        np.add.at(Gz, r, v * z[c])
        assert [bool(x) for x in Gz >= h - 1e-9 * np.abs(h)] == ref
        sat = rows.satisfied(xy, delta)
        per_ct = np.asarray(ref).reshape(rows.n_cells, T_ctrl, 5).all(-1)
        np.testing.assert_array_equal(sat, per_ct)


def test_outside_is_the_best_delta_choice():
    ph, diag = 8, 1.5
    ovs = _scene(seed=3, T=ph)
    A, b = _rows_from_oracle(ovs, ph, diag)
    rows = milp.BigMRows(A, b, diag, ph)
    rng = np.random.default_rng(2)
    xy = rng.normal([5.0, 5.0], 10.0, size=(ph, 2))
    face = np.einsum("ctlj,tj->ctl", rows.A, xy) >= rows.rhs
    # delta = 1 exactly on the faces that hold: feasible iff some face holds
    np.testing.assert_array_equal(rows.satisfied(xy, face.astype(float)), rows.outside(xy))
