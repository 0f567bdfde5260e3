"""CPU checks of the planning-QP oracle (oracle/mpc_oracle.py): the LTV restatement against the
closed form the HIP kernel uses, the dense QP against the objective as the reference writes
it, and the oracle's solutions against the KKT conditions (a solver-independent certificate;
CPLEX itself is absent, so parity against it is unpinned)."""
import math

import numpy as np
import pytest

from oracle import ccmpc_oracle as orc
from oracle import mpc_oracle as mo
from _qp_inputs import (SEEDS, check_farkas, classify, crossing_scene, farkas_certificate,
                        pick_seeds)

P = mo.DEFAULT_PARAMS


def closed_form_ltv(x0, T, Ts, l_r, L):
    """ccmpc_mpc_ltv's formulas (qp.hip): straight nominal path, Ad = I + Ts A,
    Bd = Ts B + Ts^2/2 A B, Gamma(t, k) = (I + (t - k) Ts A) Bd."""
    x, y, psi, v = x0
    c, s = math.cos(psi), math.sin(psi)
    db = 1.0 if l_r == L else 1.0 / (L / l_r)
    A = np.zeros((4, 4))
    A[0, 2], A[0, 3], A[1, 2], A[1, 3] = -v * s, c, v * c, s
    B = np.zeros((4, 2))
    B[0, 1], B[1, 1], B[2, 1], B[3, 0] = -v * s * db, v * c * db, v / L, 1.0
    Bd = Ts * B + 0.5 * Ts * Ts * A @ B
    G = np.zeros((4 * T, 2 * T))
    for t in range(T):
        for k in range(t + 1):
            G[4 * t:4 * t + 4, 2 * k:2 * k + 2] = (np.eye(4) + (t - k) * Ts * A) @ Bd
    xb = np.array([[x + v * c * Ts * i, y + v * s * Ts * i, psi, v] for i in range(1, T + 1)])
    return xb.ravel(), G


@pytest.mark.parametrize("T,x0", [(8, [165.0, -60.0, 0.124, 8.0]),
                                  (12, [10.0, 5.0, -2.1, 3.5]),
                                  (3, [0.0, 0.0, 1.0, 0.0])])
def test_ltv_restatement_matches_closed_form(T, x0):
    vm = mo.VehicleModel(T, 0.5, l_r=0.5 * 3.7, L=3.7)
    xbar, ubar, G, nx, nu = vm.get_optimization_ltv(np.array(x0), np.zeros(2))
    xb_c, G_c = closed_form_ltv(x0, T, 0.5, 0.5 * 3.7, 3.7)
    assert (nx, nu) == (4, 2) and not ubar.any()
    np.testing.assert_allclose(xbar, xb_c, rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(G, G_c, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("order", ["F", "C"])
def test_dense_qp_equals_objective_as_written(order):
    T = 8
    ovs, cells, K, ref, goal, x0 = crossing_scene(1, T=T)
    out = orc.minkowski_generator(ovs, T, T, ref, with_l4=False)
    xbar, _, G, _, _ = mo.VehicleModel(T, 0.5, 1.85, 3.7).get_optimization_ltv(x0, np.zeros(2))
    Gf, c = mo.state_map(G, xbar, T, T)
    rows = mo.obstacle_rows(out["records"], "halfspace", T)
    H, f, k, GG, h = mo.assemble_qp(Gf, c, T, goal, ref, rows, P, order=order)
    rng = np.random.default_rng(0)
    for _ in range(5):
        u = rng.normal(0, 1, 2 * T)
        want = mo.objective_value(u, Gf, c, T, goal, ref, P, order=order)
        assert abs(0.5 * u @ H @ u + f @ u + k - want) <= 1e-9 * abs(want)
        # the rows say what the constraints say: n.x_t >= d (side +1) / <= d (side -1)
        X = (Gf @ u + c).reshape(T, 4)
        lhs = GG @ u - h
        base = 4 * T + 2 * T
        for i, r in enumerate(out["records"]):
            val = r["n"] @ X[r["t"], :2] - r["d"]
            assert math.isclose(lhs[base + i], -val if r["side"] == 1 else val,
                                rel_tol=1e-9, abs_tol=1e-7)


def test_order_f_pairs_u_t_with_u_t_plus_T():
    """cvxpy's column-major reshape: U_t = (u[t], u[T + t]) (the reference's effective
    objective); order 'C' pairs (u[2t], u[2t+1])."""
    T = 4
    G = np.zeros((4 * T, 2 * T))
    c = np.zeros(4 * T)
    p = dict(P, w_joint=0.0, w_ch_accel=0.0, w_ch_joint=0.0, w_ch_turning=0.0)
    u = np.zeros(2 * T)
    u[T] = 1.0                                   # U_0 steering under 'F', U_2 accel under 'C'
    f_cost = mo.objective_value(u, G, c, T, [0, 0], [[0, 0]], p, order="F")
    c_cost = mo.objective_value(u, G, c, T, [0, 0], [[0, 0]], p, order="C")
    assert f_cost == pytest.approx(p["w_turning"]) and c_cost == pytest.approx(p["w_accel"])


@pytest.mark.parametrize("i", range(4))
def test_oracle_solution_satisfies_kkt(i):
    T = 8
    seed = pick_seeds("binding", 4)[i]
    ovs, cells, K, ref, goal, x0 = crossing_scene(seed, T=T)
    out = orc.minkowski_generator(ovs, T, T, ref, with_l4=False)
    xbar, _, G, _, _ = mo.VehicleModel(T, 0.5, 1.85, 3.7).get_optimization_ltv(x0, np.zeros(2))
    r = mo.solve_step(G, xbar, T, T, goal, ref, out["records"], "halfspace", P)
    assert r["feasible"]
    prim, stat, comp, lam = mo.kkt_residuals(r["H"], r["f"], r["G"], r["h"], r["u"], r["lam"])
    assert prim < 1e-12 and stat < 1e-10 and comp < 1e-10 and lam.min() >= -1e-10
    assert any(a >= 6 * T for a in r["active"])   # an obstacle half-space binds
    # no feasible point does better (strict convexity: the KKT point is the minimiser)
    rng = np.random.default_rng(seed)
    for _ in range(50):
        v = r["u"] + rng.normal(0, 1e-2, 2 * T)
        if np.all(r["G"] @ v <= r["h"]):
            assert mo.objective_value(v, r["Gf"], r["c"], T, goal, ref, P) >= r["cost"] - 1e-9


@pytest.mark.parametrize("T", [8, 12])
def test_pinned_verdicts(T):
    """The oracle still classifies every pinned seed as recorded in _qp_inputs.SEEDS."""
    for kind, seeds in SEEDS[T].items():
        for s in seeds:
            assert classify(s, T) == kind, (T, s, kind)


@pytest.mark.parametrize("seed", SEEDS[8]["infeasible"][:3])
def test_infeasible_scenes_have_a_farkas_certificate(seed):
    """Infeasibility proven independently of the oracle's phase-1 LP: a Farkas vector y >= 0,
    G^T y = 0, h . y < 0 for the QP's inequality rows (the reference's CPLEX failure path,
    v8ideal/__init__.py:3099-3110)."""
    T = 8
    ovs, cells, K, ref, goal, x0 = crossing_scene(seed, T=T)
    out = orc.minkowski_generator(ovs, T, T, ref, with_l4=False)
    xbar, _, G, _, _ = mo.VehicleModel(T, 0.5, 1.85, 3.7).get_optimization_ltv(x0, np.zeros(2))
    r = mo.solve_step(G, xbar, T, T, goal, ref, out["records"], "halfspace", P)
    assert not r["feasible"]
    y = farkas_certificate(r["G"], r["h"])
    assert y is not None and check_farkas(r["G"], r["h"], y)


@pytest.mark.parametrize("seed", SEEDS[8]["binding"][:3])
def test_feasible_scenes_have_no_farkas_certificate(seed):
    T = 8
    ovs, cells, K, ref, goal, x0 = crossing_scene(seed, T=T)
    out = orc.minkowski_generator(ovs, T, T, ref, with_l4=False)
    xbar, _, G, _, _ = mo.VehicleModel(T, 0.5, 1.85, 3.7).get_optimization_ltv(x0, np.zeros(2))
    r = mo.solve_step(G, xbar, T, T, goal, ref, out["records"], "halfspace", P)
    assert r["feasible"] and np.all(r["G"] @ r["u"] <= r["h"] + 1e-9)
    assert farkas_certificate(r["G"], r["h"]) is None


def test_shrinking_step_state_map_keeps_the_first_step_model():
    """T < T_full: x = Gamma_full[rows, cols_future] u + x_bar + Gamma_full[rows, :past] u_prev
    (:2858-2891), i.e. the full-horizon state of the controls (u_prev, u)."""
    Tf, T = 8, 5
    x0 = np.array([165.0, -60.0, 0.124, 8.0])
    xbar, _, G, _, _ = mo.VehicleModel(Tf, 0.5, 1.85, 3.7).get_optimization_ltv(x0, np.zeros(2))
    rng = np.random.default_rng(1)
    u_prev = rng.normal(0, 1, 2 * (Tf - T))
    u = rng.normal(0, 1, 2 * T)
    Gf, c = mo.state_map(G, xbar, T, Tf, u_prev=u_prev)
    full = G @ np.concatenate((u_prev, u)) + xbar
    np.testing.assert_allclose(Gf @ u + c, full[4 * (Tf - T):], rtol=1e-12, atol=1e-9)
