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


def _road_segments():
    from ccmpc import milp
    from test_milp import _road_scene
    segs, mask = _road_scene(0)
    return segs, mask, milp.RoadSegments(dict(polytopes=segs, mask=mask))


@pytest.mark.parametrize("T,sbig", [(3, True), (3, False), (4, True), (5, True)])
def test_road_milp_on_halfspaces_matches_oracle(gpu, T, sbig):
    """Road boundaries on a v8ideal-style QP (the reference objective with its trajectory
    term, cvxpy's column-major U): the generator's half-spaces plus one road polytope per step
    (Omicron), the affine / scale-ideal rows carrying S_t (sbig) or not -- MilpBnB on the GPU
    against the oracle's literal MILP over every Omicron subset."""
    from ccmpc import milp, mpc
    from test_milp import _road_base
    segs, mask, rs = _road_segments()
    goal, base = _road_base(T, sbig)
    xbar, G = _ego_model(T, X0)
    ref = np.stack([np.linspace(1.0, goal[0], T), np.zeros(T)], 1)
    want = mo.road_milp_enumerate(G, xbar, T, goal, ref, mo.DEFAULT_PARAMS, base=base,
                                  segs=segs, mask=mask, subsets=True)
    rows = dict(n=np.zeros((2, T, 2)), rhs=np.zeros((2, T)), side=np.ones((2, T), int),
                live=np.zeros((2, T), bool), sbig=np.full((2, T), sbig))
    slot = {-1: 0, 1: 1}
    for r in base:
        j, t = slot[r["side"]], r["t"]
        rows["n"][j, t], rows["rhs"][j, t], rows["side"][j, t] = r["n"], r["rhs"], r["side"]
        rows["live"][j, t] = True
    g_xbar, g_gamma = mpc.ltv(np.array(X0).reshape(1, 4), T)
    got = milp.MilpBnB(T, g_gamma, g_xbar, goal, ref=ref,
                       params=mpc.MPCParams.reference_defaults(), u_order=mpc.U_ORDER_F,
                       base=rows, segments=rs, device=gpu).solve()
    assert got is not None and want is not None
    assert np.abs(got["u"] - want["u"]).max() <= 1e-6 * (1.0 + np.abs(want["u"]).max())
    assert got["cost"] == pytest.approx(want["cost"], rel=1e-8)
    # the GPU's polytope per step holds its optimum
    for t, i in enumerate(got["segments"]):
        A, b = segs[i]
        assert np.all(A @ got["X"][t, :2] <= b + 1e-6)


@pytest.mark.parametrize("T", [3])
def test_v8_road_milp_matches_oracle(gpu, T):
    """v8's MILP with road boundaries: the L4-face disjunctions (Delta) and the road polytopes
    (Omicron, S_t = M_big per non-junction polytope on the face rows, v8/__init__.py:676-702)
    branched together by BranchAndBound against the oracle's enumeration of both."""
    from ccmpc import milp
    segs, mask, rs = _road_segments()
    A, rhs = _box_rows(T, [lambda t: (6.5 + 1.0 * t, 0.6)])
    goal = np.array([14.0, 0.0])
    xbar, G = _ego_model(T, X0)
    want = mo.road_milp_enumerate(G, xbar, T, goal, goal.reshape(1, 2), mo.v8_qp_params(),
                                  faces=(A, rhs), segs=segs, mask=mask, order="C",
                                  subsets=False)
    got = milp.BranchAndBound(_rows(A, rhs), T, X0, goal, segments=rs, device=gpu).solve()
    assert got is not None and want is not None
    assert np.abs(got["u"] - want["u"]).max() <= 1e-6 * (1.0 + np.abs(want["u"]).max())
    assert got["cost"] == pytest.approx(want["cost"], rel=1e-8)
    plain = milp.BranchAndBound(_rows(A, rhs), T, X0, goal, device=gpu).solve()
    assert plain is None or plain["cost"] != pytest.approx(got["cost"], rel=1e-6)


def _planner_road_case(gpu, affine, seed):
    """One planning frame of MidlevelAgent(road_boundary_constraints=True) at ph = 4 through
    compute_prediction_controls, and the oracle's literal road MILP on the frame's records."""
    from ccmpc import episode, mpc, planner
    from ccmpc.standins import AttrDict
    ph, O = 4, 2
    init, pmf, gmm = episode.synthetic_gmm(O, T=ph, seed=seed)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]])
             for o in range(O)]
    x_init = np.array([172.0, -96.0, 0.0, 5.0])
    ref = np.stack([172.0 + 2.5 * np.arange(1, ph + 1), np.linspace(-95.0, -92.0, ph)], 1)
    goal = np.array([186.0, -91.0])        # up the junction box, out of the lane
    lane = (np.array([[1.0, 0.0], [-1.0, 0.0], [0.0, 1.0], [0.0, -1.0]]),
            np.array([180.0, -160.0, -96.0 + 0.6, 96.0 + 0.6]))
    box = (np.array([[1.0, 0.0], [-1.0, 0.0], [0.0, 1.0], [0.0, -1.0]]),
           np.array([230.0, -178.0, -96.0 + 8.0, 96.0 + 8.0]))
    segments = AttrDict(polytopes=[lane, box], mask=np.array([False, True]), goal=goal)
    agent = planner.MidlevelAgent(prediction_horizon=ph, road_boundary_constraints=True,
                                  device=gpu)
    sampler = dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=2000, seed=seed)
    err = None
    try:
        agent.compute_prediction_controls(0, ph, not affine, sampler, minpos, pasts, x_init,
                                          goal, ref, segments=segments)
    except planner.InSimulationException as e:
        err = e
    h = agent.last_records
    base = []
    for c in range(h.shape[0]):
        for r in h[c]:
            if int(r["status"]) != 0:
                continue
            if affine:
                t, d = int(r["t"]), float(r["rhs"])
            else:
                t, d = int(r["t_tau"]) >> 16, float(r["d"])
            base.append(dict(t=t, n=np.array([r["n0"], r["n1"]]), rhs=d, side=int(r["side"]),
                             sbig=affine))
    xb, _, G, _, _ = mo.VehicleModel(ph, 0.5, 1.85, 3.7).get_optimization_ltv(x_init,
                                                                               np.zeros(2))
    want = mo.road_milp_enumerate(G, xb, ph, goal, ref, mpc.MPCParams.reference_defaults()
                                  .as_dict(), base=base, segs=segments.polytopes,
                                  mask=segments.mask, subsets=True)
    return agent, err, want


@pytest.mark.parametrize("affine", [False, True], ids=["minkowski", "affine"])
def test_planner_road_boundaries_match_oracle_milp(gpu, affine):
    """road_boundary_constraints=True on the v8ideal planner (it used to refuse): the frame's
    generator records (Minkowski: no S_big; affine: + S_big on both sides) and the road
    polytopes as one MILP -- solve_planning_qp's branch and bound against the oracle's literal
    enumeration, the polytope per step holding the plan."""
    n_feasible = 0
    for seed in (3, 11):
        agent, err, want = _planner_road_case(gpu, affine, seed)
        if want is None:
            assert err is not None
            continue
        assert err is None, err
        got = agent.last_ctrl
        assert np.abs(got["u"] - want["u"]).max() <= 1e-6 * (1.0 + np.abs(want["u"]).max())
        assert got["cost"] == pytest.approx(want["cost"], rel=1e-8)
        assert list(got["polytopes"]) == [0, 1, 1, 1]     # the lane, then the junction box
        assert agent.last_bnb["nodes"] > 1                 # the road binds: it branched
        n_feasible += 1
    assert n_feasible >= 1


@pytest.mark.parametrize("T,Tf", [(3, 5), (4, 6)])
def test_road_milp_shrinking_horizon_matches_oracle(gpu, T, Tf):
    """The shrinking step's road MILP (Tsh < ph: the first step's LTV model kept, the executed
    controls u_prev moving the state, :2858-2891 / :3186): MilpBnB with T_full and u_prev --
    its rounds carry u_prev in their pinned input pack -- against the oracle's literal MILP on
    the same sliced model."""
    from ccmpc import milp, mpc
    from test_milp import _road_base
    segs, mask, rs = _road_segments()
    goal, base = _road_base(T, True)
    xbar, G = _ego_model(Tf, X0)
    ref = np.stack([np.linspace(1.0, goal[0], T), np.zeros(T)], 1)
    u_prev = np.tile([0.3, -0.02], Tf - T)
    want = mo.road_milp_enumerate(G, xbar, T, goal, ref, mo.DEFAULT_PARAMS, base=base,
                                  segs=segs, mask=mask, subsets=False, T_full=Tf,
                                  u_prev=u_prev)
    rows = dict(n=np.zeros((2, T, 2)), rhs=np.zeros((2, T)), side=np.ones((2, T), int),
                live=np.zeros((2, T), bool), sbig=np.full((2, T), True))
    slot = {-1: 0, 1: 1}
    for r in base:
        j, t = slot[r["side"]], r["t"]
        rows["n"][j, t], rows["rhs"][j, t], rows["side"][j, t] = r["n"], r["rhs"], r["side"]
        rows["live"][j, t] = True
    g_xbar, g_gamma = mpc.ltv(np.array(X0).reshape(1, 4), Tf)
    got = milp.MilpBnB(T, g_gamma, g_xbar, goal, ref=ref,
                       params=mpc.MPCParams.reference_defaults(), u_order=mpc.U_ORDER_F,
                       T_full=Tf, u_prev=u_prev, base=rows, segments=rs, device=gpu).solve()
    assert (got is None) == (want is None)
    if want is not None:
        assert np.abs(got["u"] - want["u"]).max() <= 1e-6 * (1.0 + np.abs(want["u"]).max())
        assert got["cost"] == pytest.approx(want["cost"], rel=1e-8)
