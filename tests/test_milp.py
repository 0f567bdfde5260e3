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


def _box_rows(T, centres, half=(2.0, 1.2), diag=1.0):
    """L4-shaped rows of axis-aligned boxes: A (C, T, 4, 2), rhs = b + diag (C, T, 4); the
    obstacle is {x : A x <= b}, a face row asks a_l . x_t >= rhs_l (outside face l)."""
    A = np.tile(np.array([[1.0, 0.0], [0.0, 1.0], [-1.0, 0.0], [0.0, -1.0]]),
                (len(centres), T, 1, 1))
    b = np.zeros((len(centres), T, 4))
    for c, ctr in enumerate(centres):
        for t in range(T):
            px, py = ctr(t)
            b[c, t] = [px + half[0], py + half[1], -px + half[0], -py + half[1]]
    return A, b + diag


def _ego_model(T, x0=(0.0, 0.0, 0.0, 6.0)):
    from oracle import mpc_oracle as mo
    xbar, _, G, _, _ = mo.VehicleModel(T, 0.5, 1.85, 3.7).get_optimization_ltv(
        np.array(x0), np.zeros(2))
    return xbar, G


def test_v8_objective_is_the_qp_with_v8_weights():
    """v8's compute_objective (v8/__init__.py:727-753) equals the QP's objective under
    v8_qp_params (w_ref = 0, R2 off-diagonal w_ch_joint / 2, U row-major), and the product's
    mirror (ccmpc.milp.compute_objective) is the same expression."""
    from oracle import mpc_oracle as mo
    T = 6
    xbar, G = _ego_model(T)
    Gf, c = mo.state_map(G, xbar, T, T)
    goal = np.array([30.0, 1.0])
    H, f, k, _, _ = mo.assemble_qp(Gf, c, T, goal, goal.reshape(1, 2), [], mo.v8_qp_params(),
                                   order="C")
    rng = np.random.default_rng(3)
    for _ in range(5):
        u = rng.normal(0, 0.5, 2 * T)
        X, U = (Gf @ u + c).reshape(T, 4), u.reshape(T, 2)
        want = mo.v8_compute_objective(X, U, goal)
        assert 0.5 * u @ H @ u + f @ u + k == pytest.approx(want, rel=1e-12)
        assert milp.compute_objective(X, U, goal) == pytest.approx(want, rel=1e-14)


def test_oracle_branch_and_bound_is_the_enumerated_optimum():
    """The oracle's best-first branch and bound returns the optimum of the enumeration over
    every face assignment (L^(C T) convex QPs), on a box in the ego's path at every step."""
    from oracle import mpc_oracle as mo
    T = 4
    xbar, G = _ego_model(T)
    A, rhs = _box_rows(T, [lambda t: (8.0 + 1.5 * t, 0.3)])      # slower, just ahead
    goal = np.array([20.0, 0.0])
    e = mo.milp_enumerate(G, xbar, T, goal, A, rhs)
    b = mo.milp_bnb(G, xbar, T, goal, A, rhs)
    assert e is not None and b is not None
    np.testing.assert_allclose(b["u"], e["u"], atol=1e-7)
    assert b["cost"] == pytest.approx(e["cost"], rel=1e-9)
    assert b["nodes"] < 4 ** T        # the bound prunes
    slack = mo.disjunction_slack(A, rhs, b["X"])
    assert np.all(slack <= 1e-6)      # every disjunction holds at the optimum


def _road_scene(T):
    """Two road polytopes along x (A x <= b): a narrow non-junction lane and a wide junction
    box overlapping it, and the ego model of _ego_model."""
    lane = (np.array([[1.0, 0.0], [-1.0, 0.0], [0.0, 1.0], [0.0, -1.0]]),
            np.array([9.0, 5.0, 1.8, 1.8]))
    box = (np.array([[1.0, 0.0], [-1.0, 0.0], [0.0, 1.0], [0.0, -1.0]]),
           np.array([60.0, -6.0, 6.0, 6.0]))
    return [lane, box], np.array([False, True])


def _road_base(T, sbig):
    """Half-spaces that make the polytope choice matter: a '<=' row slowing the ego (x_t <=
    2.5 + 3.2 t, which the junction box x >= 6 cannot meet before t = 1) and from t = 2 a '>='
    row below it; with sbig the lane's S_t = M_big relaxes the first and breaks the second."""
    base = []
    for t in range(T):
        base.append(dict(t=t, n=np.array([1.0, 0.0]), rhs=2.5 + 3.2 * t, side=-1, sbig=sbig))
        if t >= 2:
            base.append(dict(t=t, n=np.array([0.0, 1.0]), rhs=-1.0 - 0.1 * t, side=1,
                             sbig=sbig))
    return np.array([3.0 * T + 4.0, 3.0]), base


@pytest.mark.parametrize("T,sbig", [(2, True), (3, True), (3, False), (4, True)])
def test_one_polytope_per_step_is_enough(T, sbig):
    """MilpBnB branches on ONE road polytope per step; the reference's Omicron[:, t] may take
    any non-empty subset.  The oracle's literal MILP (every subset, every unchosen row with its
    + M_big relaxation) has the same optimum as the one-polytope restriction, on a scene whose
    half-spaces carry S_t (sbig: the affine / scale-ideal rows, both sides) or not."""
    from oracle import mpc_oracle as mo
    segs, mask = _road_scene(T)
    xbar, G = _ego_model(T, (0.0, 0.0, 0.0, 6.0))
    goal, base = _road_base(T, sbig)
    p = mo.DEFAULT_PARAMS
    ref = np.stack([np.linspace(1.0, goal[0], T), np.zeros(T)], 1)
    full = mo.road_milp_enumerate(G, xbar, T, goal, ref, p, base=base, segs=segs, mask=mask,
                                  subsets=True)
    one = mo.road_milp_enumerate(G, xbar, T, goal, ref, p, base=base, segs=segs, mask=mask,
                                 subsets=False)
    assert full is not None and one is not None
    assert one["cost"] == pytest.approx(full["cost"], rel=1e-9, abs=1e-9)
    np.testing.assert_allclose(one["u"], full["u"], atol=1e-6)


def test_road_segments_padding():
    segs, mask = _road_scene(2)
    tri = (np.array([[1.0, 0.0], [0.0, 1.0], [-1.0, -1.0]]), np.array([1.0, 1.0, 0.0]))
    rs = milp.RoadSegments(dict(polytopes=segs + [tri], mask=[False, True, True]))
    assert (rs.I, rs.F) == (3, 4)
    assert rs.live.sum() == 11 and not rs.live[2, 3]
    assert rs.any_open
    with pytest.raises(ValueError):
        milp.RoadSegments(dict(polytopes=[(np.zeros((2, 2)), np.zeros(3))], mask=[False]))


class _OracleBnB(milp.MilpBnB):
    """MilpBnB's tree with each node's relaxation solved by the oracle's QP from the very
    records the GPU launch would get (host-only: the branching, relaxation and feasibility
    logic on CPU)."""

    def __init__(self, G, xbar, T, goal, ref, p, order, **kw):
        from oracle import mpc_oracle as mo
        self._mo, self._p, self._order = mo, p, order
        self._Gf, self._c = mo.state_map(G, xbar, T, T)
        self._host_init(T, goal, ref, None, 0, T, kw.get("base"), kw.get("faces"),
                        kw.get("segments"), kw.get("M_big", milp.M_BIG), 64, 1e-7, 100000)

    def _solve_batch(self, nodes):
        mo, T = self._mo, self.T
        rec = self._records(nodes)
        out = []
        for r in rec:
            rows = [(int(x["t_tau"]), (-1.0 if x["side"] == 1 else 1.0) * np.array(
                [x["n0"], x["n1"]]), (-1.0 if x["side"] == 1 else 1.0) * float(x["rhs"]))
                for x in r.reshape(-1) if x["status"] == 0]
            s = mo._road_node(self._Gf, self._c, T, self.goal, self.ref, rows, self._p,
                              self._order)
            out.append(s)
        ok = np.array([s is not None for s in out])
        u = np.array([s["u"] if s else np.zeros(2 * T) for s in out])
        X = np.array([s["X"] if s else np.zeros((T, 4)) for s in out])
        cost = np.array([s["cost"] if s else np.inf for s in out])
        self.stats["launches"] += 1
        return u, X, cost, ok


@pytest.mark.parametrize("T,sbig", [(3, True), (3, False), (4, True)])
def test_bnb_tree_on_oracle_qps_halfspaces(T, sbig):
    """The branch and bound's relaxation / branching / incumbent logic with oracle QPs: the
    same optimum as the oracle's literal MILP over every Omicron subset."""
    from oracle import mpc_oracle as mo
    segs, mask = _road_scene(T)
    goal, base = _road_base(T, sbig)
    xbar, G = _ego_model(T, (0.0, 0.0, 0.0, 6.0))
    ref = np.stack([np.linspace(1.0, goal[0], T), np.zeros(T)], 1)
    want = mo.road_milp_enumerate(G, xbar, T, goal, ref, mo.DEFAULT_PARAMS, base=base,
                                  segs=segs, mask=mask, subsets=True)
    rows = dict(n=np.zeros((2, T, 2)), rhs=np.zeros((2, T)), side=np.ones((2, T), int),
                live=np.zeros((2, T), bool), sbig=np.array([sbig, sbig]))
    for r in base:
        j, t = (0 if r["side"] == -1 else 1), r["t"]
        rows["n"][j, t], rows["rhs"][j, t], rows["side"][j, t] = r["n"], r["rhs"], r["side"]
        rows["live"][j, t] = True
    got = _OracleBnB(G, xbar, T, goal, ref, mo.DEFAULT_PARAMS, "F", base=rows,
                     segments=milp.RoadSegments(dict(polytopes=segs, mask=mask))).solve()
    assert got["cost"] == pytest.approx(want["cost"], rel=1e-9)
    np.testing.assert_allclose(got["u"], want["u"], atol=1e-6)


def test_bnb_tree_on_oracle_qps_v8_faces_and_road():
    """v8's face disjunctions and the road polytopes branched together (oracle QPs) against
    the oracle's enumeration of both; and the faces alone against milp_bnb."""
    from oracle import mpc_oracle as mo
    T = 3
    segs, mask = _road_scene(T)
    A, rhs = _box_rows(T, [lambda t: (6.5 + 1.0 * t, 0.6)])
    goal = np.array([14.0, 0.0])
    xbar, G = _ego_model(T, (0.0, 0.0, 0.0, 6.0))
    p = mo.v8_qp_params()
    want = mo.road_milp_enumerate(G, xbar, T, goal, goal.reshape(1, 2), p, faces=(A, rhs),
                                  segs=segs, mask=mask, order="C", subsets=False)
    got = _OracleBnB(G, xbar, T, goal, None, p, "C", faces=(A, rhs),
                     segments=milp.RoadSegments(dict(polytopes=segs, mask=mask))).solve()
    assert got["cost"] == pytest.approx(want["cost"], rel=1e-9)
    np.testing.assert_allclose(got["u"], want["u"], atol=1e-6)
    plain = _OracleBnB(G, xbar, T, goal, None, p, "C", faces=(A, rhs)).solve()
    ref = mo.milp_bnb(G, xbar, T, goal, A, rhs)
    assert plain["cost"] == pytest.approx(ref["cost"], rel=1e-9)


def test_round_violations_at_once_equal_per_node():
    """MilpBnB._violations_all (a round's nodes at once) against _violations node by node:
    the same bits, with and without base rows, for nodes with fixed faces."""
    T, C, L = 6, 3, 4
    rng = np.random.default_rng(7)
    faces = (rng.standard_normal((C, T, L, 2)), rng.standard_normal((C, T, L)))
    base = dict(n=rng.standard_normal((2, T, 2)), rhs=rng.standard_normal((2, T)),
                side=np.where(rng.random((2, T)) < 0.5, 1, -1),
                live=rng.random((2, T)) < 0.8, sbig=rng.random((2, T)) < 0.5)
    for b in (None, base):
        bnb = milp.MilpBnB.__new__(milp.MilpBnB)
        bnb._host_init(T, np.zeros(2), None, milp.v8_qp_params(), 0, T, b, faces, None,
                       milp.M_BIG, 64, 1e-7, 1000)
        nodes = [({}, {})] + [({(int(rng.integers(C)), int(rng.integers(T))): int(rng.integers(L))
                                for _ in range(k)}, {}) for k in range(1, 9)]
        X = rng.standard_normal((len(nodes), T, 4)) * 5.0
        got = bnb._violations_all(X, nodes)
        for Xi, (f, g), (tv, ch, fv) in zip(X, nodes, got):
            tv1, ch1, fv1 = bnb._violations(Xi, f, g)
            assert tv.tobytes() == tv1.tobytes() and fv.tobytes() == fv1.tobytes()
            assert ch == ch1
