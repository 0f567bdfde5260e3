"""v8's MILP (v8/__init__.py:692-838): the big-M obstacle disjunction over the
L4 faces with v8's compute_objective, solved on the GPU by ccmpc.milp.BranchAndBound (batched
mpc_qp_kernel launches per round) against the oracle's exact optimum (oracle/mpc_oracle.py
milp_bnb, SciPy QPs; milp_enumerate over every face assignment where that is small).

Parity bar: the MILP optimum is unique on these scenes, so u within 1e-6 (1 + |u|), the cost
within 1e-8 relative; the faces: every face the GPU chose holds at the oracle's optimum, and
the oracle's at the GPU's (both satisfy all disjunctions).  CPLEX itself is absent (unpinned)."""
import numpy as np
import pytest

from oracle import mpc_oracle as mo
from test_milp import _box_rows, _ego_model

pytestmark = pytest.mark.gpu

X0 = (0.0, 0.0, 0.0, 6.0)


def _rows(A, rhs):
    from ccmpc import milp
    return milp.BigMRows(A, rhs, 0.0, A.shape[1])     # rhs already holds + diag


def _check(got, want, A, rhs, T):
    assert got is not None and want is not None
    tol = 1e-6 * (1.0 + np.abs(want["u"]).max())
    assert np.abs(got["u"] - want["u"]).max() <= tol, np.abs(got["u"] - want["u"]).max()
    assert got["cost"] == pytest.approx(want["cost"], rel=1e-8)
    for X, faces in ((want["X"], got["faces"]), (got["X"], want["faces"])):
        a = np.einsum("ctlj,tj->ctl", A[:, :T], X[:, :2])
        chosen = np.take_along_axis(a - rhs[:, :T], faces[..., None], -1)[..., 0]
        assert np.all(chosen >= -1e-5), chosen.min()
    assert np.all(mo.disjunction_slack(A[:, :T], rhs[:, :T], got["X"]) <= 1e-6)


SCENES = {
    "one_box_T4": (4, [lambda t: (8.0 + 1.5 * t, 0.3)]),
    "one_box_T6": (6, [lambda t: (9.0 + 1.0 * t, -0.4)]),
    "two_boxes_T6": (6, [lambda t: (8.0 + 1.5 * t, 0.3), lambda t: (16.0, 4.0 - 0.5 * t)]),
    "two_boxes_T8": (8, [lambda t: (10.0 + 1.0 * t, 0.2), lambda t: (22.0, -3.5 + 0.6 * t)]),
    "static_box_T8": (8, [lambda t: (14.0, 0.3)]),                 # the ego swerves past it
    "static_pair_T8": (8, [lambda t: (14.0, 0.3), lambda t: (20.0, -4.0)]),
}


@pytest.mark.parametrize("name", list(SCENES))
def test_branch_and_bound_matches_oracle_optimum(gpu, name):
    from ccmpc import milp
    T, centres = SCENES[name]
    A, rhs = _box_rows(T, centres)
    goal = np.array([6.0 * T * 0.5 + 8.0, 0.0])
    xbar, G = _ego_model(T, X0)
    want = mo.milp_bnb(G, xbar, T, goal, A, rhs)
    bnb = milp.BranchAndBound(_rows(A, rhs), T, X0, goal, device=gpu)
    got = bnb.solve()
    _check(got, want, A, rhs, T)
    assert got["launches"] <= got["nodes"]
    if T == 4 and len(centres) == 1:              # small enough to enumerate (256 QPs)
        e = mo.milp_enumerate(G, xbar, T, goal, A, rhs)
        _check(got, e, A, rhs, T)


def test_branch_and_bound_batches_are_one_launch_per_round(gpu):
    """Batch size 1 (one node per launch) and 64 reach the same optimum; the batched form
    needs fewer launches."""
    from ccmpc import milp
    T, centres = SCENES["two_boxes_T6"]
    A, rhs = _box_rows(T, centres)
    goal = np.array([20.0, 0.0])
    r1 = milp.BranchAndBound(_rows(A, rhs), T, X0, goal, batch=1, device=gpu).solve()
    r64 = milp.BranchAndBound(_rows(A, rhs), T, X0, goal, batch=64, device=gpu).solve()
    np.testing.assert_allclose(r64["u"], r1["u"], atol=1e-9)
    assert r64["launches"] < r1["launches"]


def test_infeasible_milp_is_reported(gpu):
    """A box the ego cannot avoid (too close, too wide): no face assignment is feasible, the
    solve returns None (do_highlevel_control's InSimulationException path, :862-873)."""
    from ccmpc import milp
    T = 4
    A, rhs = _box_rows(T, [lambda t: (3.0 * (t + 1) + 0.5, 0.3)], half=(2.0, 6.0))
    xbar, G = _ego_model(T, X0)
    assert mo.milp_bnb(G, xbar, T, np.array([20.0, 0.0]), A, rhs) is None
    assert milp.BranchAndBound(_rows(A, rhs), T, X0, np.array([20.0, 0.0]),
                               device=gpu).solve() is None


@pytest.mark.parametrize("O,T", [(1, 6), (2, 8)])
def test_v8_do_highlevel_control_on_device_l4(gpu, O, T):
    """MidlevelAgentV8.do_highlevel_control: the big-M rows over the device L4 faces of
    crossing OV clouds (v8/__init__.py:692-724), v8's objective, the MILP on the GPU -- the
    oracle's branch and bound on the same rows gives the same u, and the same verdict where
    no face assignment is feasible; U_star / X_star / cost as the reference returns them
    (U = u.reshape(T, nu))."""
    from ccmpc import milp, ovehicle, synthetic
    from ccmpc.standins import AttrDict
    n_cmp = 0
    for seed in range(20, 28):
        cells, K, ref, goal, x_init, pasts = synthetic.crossing_scene(seed, O=O, N=600, T=T,
                                                                      K=1, lateral=6.0)
        ovs = ovehicle.scene_from_positions([[c] for c in cells],
                                            [p.reshape(1, 2) for p in pasts], device=gpu)
        agent = milp.MidlevelAgentV8(prediction_horizon=T, control_horizon=T, device=gpu)
        params = AttrDict(x_init=x_init, goal=goal, diag=milp.ego_diag(3.7, 1.79), O=O, K=K)
        out, err = agent.do_highlevel_control(params, ovs)
        rows = agent.compute_obstacle_constraints(params, ovs, None, None, None, None)[0]
        xbar, _, G, _, _ = mo.VehicleModel(T, 0.5, 1.85, 3.7).get_optimization_ltv(
            x_init, np.zeros(2))
        want = mo.milp_bnb(G, xbar, T, goal, rows.A, rows.rhs)
        if want is None:
            assert err is not None and out.U_star is None
            continue
        assert err is None
        got = dict(u=out.U_star.reshape(-1), X=out.X_star, cost=out.cost, faces=out.faces)
        _check(got, want, rows.A, rows.rhs, T)
        assert out.cost == pytest.approx(milp.compute_objective(out.X_star, out.U_star, goal),
                                         rel=1e-9)
        n_cmp += 1
    assert n_cmp >= 2
