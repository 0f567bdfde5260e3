"""The drop-in surface: MidlevelAgent generator methods (9-tuples) and make_ovehicles on the
GPU, against the oracle restatement of v8ideal/__init__.py and ovehicle.py."""
import numpy as np
import pytest
import torch

from oracle import ccmpc_oracle as orc

pytestmark = pytest.mark.gpu


class Params:
    def __init__(self, O, K, frame):
        self.O, self.K, self.frame = O, np.asarray(K), frame


def _scene(seed, O=3, N=3000, T=8):
    from ccmpc import synthetic
    ovs, ref, pasts = synthetic.scene(seed, O=O, N=N, T=T)
    return ovs, ref, pasts


def _oracle_ovs(ov_cells, pasts, T):
    out = []
    for cells, p in zip(ov_cells, pasts):
        past = np.asarray(p, float).reshape(1, 2)
        out.append(orc.OVehicle(T, past, np.ones(len(cells)) / len(cells), cells,
                                [orc._step_yaws(c, past[-1], T) for c in cells],
                                np.zeros((len(cells), 2)), np.array([4.5, 2.5])))
    return out


def _check_minkowski(cons, want_recs):
    assert len(cons) == len(want_recs)
    for c, r in zip(cons, want_recs):
        assert (c.ov, c.k, c.t, c.tau) == (r["ov"], r["k"], r["t"], r["tau"])
        assert c.which == r["which"] and c.side == r["side"]
        np.testing.assert_allclose(c.n, r["n"], rtol=1e-12)
        assert c.d == pytest.approx(r["d"], rel=1e-10)


def test_minkowski_generator_full_tuple(gpu):
    from ccmpc import ovehicle, planner
    T = 8
    ov_cells, ref, pasts = _scene(31, T=T)
    K = [len(c) for c in ov_cells]
    ovs = ovehicle.scene_from_positions(ov_cells, pasts, device=gpu)
    agent = planner.MidlevelAgent(prediction_horizon=T, device=gpu)
    eps = orc.eps_ura_matrix(K)
    out = agent.compute_obstacle_constraints_GMM_Minkowski_idealprediction(
        Params(len(K), K, 100), ovs, None, None, None, eps, None, T, ref)
    assert len(out) == 9 and out[8] == 0
    cons, vertices, A_union, b_union, ovc, direct, smean, scov, _ = out
    want = orc.minkowski_generator(_oracle_ovs(ov_cells, pasts, T), T, T, ref)
    _check_minkowski(cons, want["records"])
    np.testing.assert_allclose(agent.prob_lower_save, want["prob_lower_save"], rtol=1e-9)
    assert ovc == want["OVconstraint"] and direct == [None] * len(K)
    for j in range(3):
        for o in range(len(K)):
            for k in range(K[o]):
                assert smean[j][o][k] == pytest.approx(want["ov_state_mean"][j][o][k], rel=1e-12)
                assert scov[j][o][k] == pytest.approx(float(want["ov_state_cov"][j][o][k]),
                                                      rel=1e-9)
    for t in range(T):
        for o in range(len(K)):
            for k in range(K[o]):
                np.testing.assert_allclose(A_union[t][k][o], want["A_union"][t][k][o], atol=1e-15)
                np.testing.assert_allclose(b_union[t][k][o], want["b_union"][t][k][o], rtol=1e-12)
    np.testing.assert_allclose(vertices[T - 1][0][0], want["vertices"][T - 1][0][0], rtol=1e-12)
    # save_moments content (the reference's pickle) matches the oracle's save_moments
    sm = agent.saved_moments(100)
    for o in range(len(K)):
        for k in range(K[o]):
            for t in range(T):
                np.testing.assert_allclose(sm["mean_p0p1"][o][k][t],
                                           want["moments"]["mean_p0p1"][o][k][t], rtol=1e-13)
                np.testing.assert_allclose(sm["cov_p0p1"][o][k][t],
                                           want["moments"]["cov_p0p1"][o][k][t], rtol=1e-10)


def test_shrinking_step_uses_ideal_rollout(gpu):
    """T < ph: predict_ideal from the previous step's device moments, then the Minkowski
    constraints on the rolled-out cloud (v8ideal/__init__.py:824-825, :885-888)."""
    from ccmpc import ovehicle, planner
    T, n_ideal, seed = 8, 20000, 5
    ov_cells, ref, pasts = _scene(44, O=2, N=2500, T=T)
    K = [len(c) for c in ov_cells]
    ovs = ovehicle.scene_from_positions(ov_cells, pasts, device=gpu)
    agent = planner.MidlevelAgent(prediction_horizon=T, n_ideal=n_ideal, seed=seed, device=gpu)
    eps = orc.eps_ura_matrix(K)
    agent.compute_obstacle_constraints_GMM_Minkowski_idealprediction(
        Params(len(K), K, 200), ovs, None, None, None, eps, None, T, ref)
    Tn = T - 1
    out = agent.compute_obstacle_constraints_GMM_Minkowski_idealprediction(
        Params(len(K), K, 210), ovs, None, None, None, eps, None, Tn, ref)
    # oracle: same moments -> same Philox draws -> same rollout -> same constraints
    oracle_ovs = _oracle_ovs(ov_cells, pasts, T)
    mom = orc.save_moments([ov.pred_positions for ov in oracle_ovs], T)
    ideal = orc.predict_ideal(mom, K, Tn, n_ideal, seed=(seed * 1_000_003 + 210))
    want = orc.minkowski_generator(oracle_ovs, Tn, T, ref, ideal_trajs=ideal, with_l4=False)
    _check_minkowski(out[0], want["records"])


def test_affine_generator(gpu):
    from ccmpc import ovehicle, planner
    T = 8
    ov_cells, ref, pasts = _scene(52, T=T)
    K = [len(c) for c in ov_cells]
    ovs = ovehicle.scene_from_positions(ov_cells, pasts, device=gpu)
    agent = planner.MidlevelAgent(prediction_horizon=T, device=gpu)
    out = agent.compute_obstacle_constraints_GMM_affine(
        Params(len(K), K, 300), ovs, None, None, None, orc.eps_ura_matrix(K), None, T, ref)
    want = orc.affine_generator(_oracle_ovs(ov_cells, pasts, T), T, T, ref, with_l4=False)
    assert len(out[0]) == len(want["records"])
    for c, r in zip(out[0], want["records"]):
        assert c.which == r["which"] and c.side == r["side"]
        assert c.rhs == pytest.approx(r["rhs"], rel=1e-11)
        assert c.margin == pytest.approx(r["margin"], rel=1e-10)
        # the OV's mean position is on the forbidden side of its own constraint
        assert not c.holds(np.array([r["mean"][0], r["mean"][1]]))


@pytest.mark.parametrize("N", [6000, 12000])
def test_make_ovehicles_matches_reference_bucketing(gpu, N):
    """Sampler output -> buckets: same membership, same order, same pmf / init_center as
    make_ovehicles + OVehicle.from_trajectron (v8ideal/__init__.py:469-505, ovehicle.py:24-117)."""
    from ccmpc import engine, ovehicle
    rng = np.random.default_rng(7)
    O, L, T = 3, 25, 8
    pmf = np.stack([np.exp(rng.normal(0, 1.6, L)) for _ in range(O)])
    pmf /= pmf.sum(1, keepdims=True)
    for o in range(O):                       # make sure every OV keeps >= 1 mode
        pmf[o, rng.integers(L)] += 0.3
        pmf[o] /= pmf[o].sum()
    init = np.stack([rng.uniform(20, 60, O), rng.uniform(20, 60, O),
                     rng.uniform(-np.pi, np.pi, O), rng.uniform(3, 10, O)], axis=1)
    gmm = np.zeros((O, L, T, 5), np.float32)
    gmm[..., 0] = rng.normal(0, 0.3, size=(O, L, 1))
    gmm[..., 1] = rng.normal(0, 1.5, size=(O, L, 1))
    gmm[..., 2:4] = np.log(0.1)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2, minpos[1] + init[o, 1]]]) for o in range(O)]
    z, sample_store = engine.sample_unicycle(init, pmf, gmm, N, T, seed=3, device=gpu)
    ovs = ovehicle.make_ovehicles(sample_store, z, pmf, minpos, pasts, device=gpu)
    # oracle bucketing on the very same sampler output
    pred = np.stack([sample_store.cell_positions(o).astype(np.float32) for o in range(O)])
    want = orc.make_ovehicles(pred, z.cpu().numpy(), pmf, minpos, pasts,
                              [np.array([4.5, 2.5])] * O, T)
    for o in range(O):
        assert ovs[o].n_states == want[o].n_states
        np.testing.assert_allclose(ovs[o].latent_pmf, want[o].latent_pmf, rtol=1e-15)
        np.testing.assert_allclose(ovs[o].init_center, want[o].init_center, rtol=1e-12)
        for k in range(want[o].n_states):
            np.testing.assert_array_equal(ovs[o].pred_positions[k], want[o].pred_positions[k])
            np.testing.assert_allclose(ovs[o].pred_yaws[k], want[o].pred_yaws[k], rtol=1e-12,
                                       atol=1e-13)


@pytest.mark.parametrize("method,scaled", [
    ("compute_obstacle_constraints_GMM_affine_scale_ideal", True),
    ("compute_obstacle_constraints_GMM_affine_robust", False)])
def test_affine_scale_ideal_two_frames(gpu, method, scaled):
    """compute_obstacle_constraints_GMM_affine_scale_ideal through the agent: frame 300 at
    T == ph, frame 310 at T < ph on the Philox ideal rollout of frame 300's moments with
    frame 300's meanNtangent loaded -- against the oracle chained the same way."""
    from ccmpc import ovehicle, planner
    T, n_ideal, seed = 8, 20_000, 6
    ov_cells, ref, pasts = _scene(61, O=2, N=2500, T=T)
    K = [len(c) for c in ov_cells]
    ovs = ovehicle.scene_from_positions(ov_cells, pasts, device=gpu)
    agent = planner.MidlevelAgent(prediction_horizon=T, n_ideal=n_ideal, seed=seed, device=gpu)
    eps = orc.eps_ura_matrix(K)
    x_init = np.array([ref[0][0] - 4.0, ref[0][1] - 0.5, 0.0, 5.0])
    p1 = Params(len(K), K, 300)
    p1.x_init = x_init
    out1 = getattr(agent, method)(
        p1, ovs, None, None, None, eps, None, T, ref)
    ref2 = ref + np.array([2.0, 0.25])
    p2 = Params(len(K), K, 310)
    p2.x_init = x_init
    out2 = getattr(agent, method)(
        p2, ovs, None, None, None, eps, None, T - 1, ref2)
    oracle_ovs = _oracle_ovs(ov_cells, pasts, T)
    w1 = orc.affine_scale_generator(oracle_ovs, T, T, ref, scaled=scaled)
    mom = orc.save_moments([ov.pred_positions for ov in oracle_ovs], T)
    ideal = orc.predict_ideal(mom, K, T - 1, n_ideal, seed=seed * 1_000_003 + 310)
    m1, t1, _, _, c1 = w1["meanNtangent"]
    w2 = orc.affine_scale_generator(oracle_ovs, T - 1, T, ref2, x_init=x_init,
                                    loaded=(m1, t1, c1), ideal_trajs=ideal, scaled=scaled)
    for out, want in ((out1, w1), (out2, w2)):
        assert len(out[0]) == len(want["records"])
        for c, r in zip(out[0], want["records"]):
            assert (c.ov, c.k, c.t) == (r["ov"], r["k"], r["t"])
            assert c.which == r["which"] and c.side == r["side"]
            assert c.rhs == pytest.approx(r["rhs"], rel=1e-9)
    # meanNtangent (the 9th element) carries the saved slopes / indices for the next frame
    assert out2[8][1][0][0][0] == pytest.approx(w2["meanNtangent"][1][0][0][0], rel=1e-9)


def test_data_save_npz_carries_mean_tangent_across_agents(gpu, tmp_path):
    """save_data / load_data (v8ideal/__init__.py:2547-2567, :2979-2993) through .npz files:
    a fresh agent that loads frame 300's moments and meanNtangent from disk generates frame
    310 exactly as the agent that produced them; without the file the T < ph step fails as
    the reference's does."""
    from ccmpc import ovehicle, planner
    T, n_ideal, seed = 8, 20_000, 4
    ov_cells, ref, pasts = _scene(62, O=2, N=2500, T=T)
    K = [len(c) for c in ov_cells]
    ovs = ovehicle.scene_from_positions(ov_cells, pasts, device=gpu)
    eps = orc.eps_ura_matrix(K)
    x_init = np.array([ref[0][0] - 4.0, ref[0][1] - 0.5, 0.0, 5.0])
    p1, p2 = Params(len(K), K, 300), Params(len(K), K, 310)
    p1.x_init = p2.x_init = x_init
    ref2 = ref + np.array([2.0, 0.25])
    a = planner.MidlevelAgent(prediction_horizon=T, n_ideal=n_ideal, seed=seed, device=gpu)
    out1 = a.compute_obstacle_constraints_GMM_affine_scale_ideal(p1, ovs, None, None, None, eps,
                                                                 None, T, ref)
    a.save_data(a.data_save(out1, p1), p1, a.ego_vehicle_id, directory=str(tmp_path))
    a.save_moments_npz(300, str(tmp_path / "m300.npz"))
    want = a.compute_obstacle_constraints_GMM_affine_scale_ideal(p2, ovs, None, None, None, eps,
                                                                 None, T - 1, ref2)
    b = planner.MidlevelAgent(prediction_horizon=T, n_ideal=n_ideal, seed=seed, device=gpu,
                              data_dir=str(tmp_path))
    with pytest.raises(KeyError):       # no moments / meanNtangent yet
        b.compute_obstacle_constraints_GMM_affine_scale_ideal(p2, ovs, None, None, None, eps,
                                                              None, T - 1, ref2)
    b.load_moments_npz(300, str(tmp_path / "m300.npz"))
    got = b.compute_obstacle_constraints_GMM_affine_scale_ideal(p2, ovs, None, None, None, eps,
                                                                None, T - 1, ref2)
    assert len(got[0]) == len(want[0])
    for c, r in zip(got[0], want[0]):
        assert (c.ov, c.k, c.t, c.which, c.side) == (r.ov, r.k, r.t, r.which, r.side)
        assert c.rhs == r.rhs and c.d == r.d
    d = np.load(tmp_path / f"agent{a.ego_vehicle_id}_frame300_cov.npz", allow_pickle=False)
    assert d["mnt_mean"].shape == (sum(K), T, 2) and d["mnt_const_idx"].dtype == np.int32
    assert bool(d["MeanCov"]) and bool(d["shrinking"])
    np.testing.assert_array_equal(d["x_init"], x_init)


@pytest.mark.parametrize("T_ctrl", [8, 6])
def test_v8_milp_rows_match_oracle(gpu, T_ctrl):
    """v8.MidlevelAgent.compute_obstacle_constraints (v8/__init__.py:692-724): the big-M rows
    over the device L4 polytopes against the oracle restatement, numerically (BigMRows) and
    as the reference's expression list evaluated at sample (X, Delta)."""
    from ccmpc import milp, ovehicle
    T = 8
    ov_cells, ref, pasts = _scene(63, O=3, N=2000, T=T)
    K = [len(c) for c in ov_cells]
    ovs = ovehicle.scene_from_positions(ov_cells, pasts, device=gpu)
    diag = milp.ego_diag(4.7, 1.9)
    agent = milp.MidlevelAgentV8(prediction_horizon=T, control_horizon=T_ctrl, diag=diag,
                                 device=gpu)
    p = Params(len(K), K, 0)
    rows, vertices, A_union, b_union = agent.compute_obstacle_constraints(
        p, ovs, None, None, None, None)
    want, holds = orc.milp_obstacle_rows(_oracle_ovs(ov_cells, pasts, T), T_ctrl, T, diag)
    assert len(rows) == 5 * len(want)
    for c, t, A, rhs in want:
        np.testing.assert_allclose(rows.A[c, t], A, rtol=1e-13, atol=1e-15)
        np.testing.assert_allclose(rows.rhs[c, t], rhs, rtol=1e-12)
    rng = np.random.default_rng(0)
    X = rng.normal(ref[0], 6.0, size=(T_ctrl, 2))
    Delta = rng.integers(0, 2, size=(sum(K), T_ctrl, 4)).astype(float)
    cons, *_ = agent.compute_obstacle_constraints(p, ovs, X, Delta, None, None)
    assert [bool(v) for v in cons] == holds(X, Delta)
    assert len(A_union) == T and np.allclose(A_union[0][0][0], rows.A[0, 0])


def test_make_ovehicles_and_l4_match_reference_functions(gpu, golden):
    """Pinned to the reference's own code (tests/golden/ovehicle_l4.npz, made by running
    OVehicle.from_trajectron, ovehicle.py:24-117, and midlevel/util.py:104-124 / :171-200 on
    the same input): device bucketing (membership, order, pmf, init_center), the device
    headings, and the device L4 polytopes A/b per kept mode and step."""
    from ccmpc import ovehicle
    g = golden("ovehicle_l4")
    T, O = int(g["T"]), g["pred"].shape[0]
    ovs = ovehicle.make_ovehicles(g["pred"], g["z"], g["latent_pmf"], g["minpos"],
                                  list(g["past"]), bboxes=np.tile(g["bbox"], (O, 1)),
                                  device=gpu)
    assert [ov.n_states for ov in ovs] == g["K"].tolist()
    c0 = 0
    for o, ov in enumerate(ovs):
        np.testing.assert_allclose(ov.latent_pmf, g["pmf_out"][o, :ov.n_states], rtol=1e-15)
        np.testing.assert_allclose(ov.init_center, g["init_center"][o, :ov.n_states],
                                   rtol=1e-12)
        for k in range(ov.n_states):
            n = g["counts"][c0 + k]
            off = int(np.sum(g["counts"][:c0 + k]))
            np.testing.assert_array_equal(ov.pred_positions[k], g["positions"][off:off + n])
            np.testing.assert_allclose(ov.pred_yaws[k], g["yaws"][off:off + n], rtol=1e-12,
                                       atol=1e-13)
        c0 += ov.n_states
    l4 = ovs[0].scene.l4()
    np.testing.assert_allclose(l4["A"].cpu().numpy(), g["A"], rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(l4["b"].cpu().numpy(), g["b"], rtol=1e-12)
    np.testing.assert_allclose(l4["yaw_mean"].cpu().numpy(), g["yaw_mean"], rtol=1e-12,
                               atol=1e-14)
