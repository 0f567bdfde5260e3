"""Pin the CPU oracle to the reference: every golden vector in tests/golden was produced by the
reference's own makeconstraint.py (see tests/golden/make_golden.py)."""
import numpy as np
import pytest

from oracle import ccmpc_oracle as orc

from _cycle_inputs import REFLOOP, ovehicles_from_fixture, refloop_inputs


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)


def test_mvoe_matches_reference(golden):
    g = golden("mvoe")
    for i in range(len(g["beta"])):
        beta, Q, _ = orc.compute_mvoe(g["S1"][i], g["S2"][i])
        assert beta == pytest.approx(g["beta"][i], rel=1e-12)
        assert rel(Q, g["Q"][i]) < 1e-12


def test_predict_moments_matches_reference(golden):
    g = golden("predict_moments")
    offs = g["offsets"]
    for i in range(len(offs) - 1):
        p = g["points"][:, offs[i]:offs[i + 1]]
        ci, cm, ct = orc.predict_moments([p[0], p[1], p[2], p[3]])
        assert rel(ci, g["cov_infer"][i]) < 1e-9   # Schur complement: cancellation-limited
        assert rel(cm, g["cov_mu"][i]) < 1e-12
        assert rel(ct, g["cov_t"][i]) < 1e-14


def test_tangent_matches_reference_including_ties(golden):
    g = golden("tangent")
    for i in range(len(g["m"])):
        n, d, which = orc.choose_closest_tangent(g["mu"][i], g["Sigma"][i], g["c"][i], g["m"][i],
                                                 g["a"][i])
        assert which == g["which"][i]
        np.testing.assert_array_equal(n, g["n"][i])
        assert d == pytest.approx(g["d"][i], rel=1e-15, abs=1e-12)
    # a == mu (the first 20 cases): the two distances differ only by the rounding of
    # proj +/- delta, and the reference's strict '<' resolves them both ways -- the oracle
    # reproduces every one of those knife-edge picks bit-for-bit above.
    assert 0 < np.sum(g["which"][:20]) < 20


def test_lower_bound_and_scale_match_reference(golden):
    g = golden("lower_bound")
    for i in range(len(g["eps"])):
        lb = orc.compute_lower_bound(g["cov_infer"][i], g["cov_mu"][i], g["cov_t"][i], g["eps"][i])
        sc = orc.compute_scale(g["cov_infer"][i], g["cov_mu"][i], g["cov_t"][i], g["gamma"][i])
        assert lb == pytest.approx(g["lower_bound"][i], rel=1e-12, abs=1e-15)
        assert sc == pytest.approx(g["scale"][i], rel=1e-12)


@pytest.mark.parametrize("name", ["cycle_o2_t8", "cycle_o1_t12"])
def test_minkowski_cycle_matches_reference(golden, name):
    g = golden(name)
    T = int(g["T"])
    ovs = ovehicles_from_fixture(g)
    out = orc.minkowski_generator(ovs, T, T, g["ref_traj"])
    recs = out["records"]
    assert len(recs) == len(g["rec_d"])
    cells = np.array([[r["ov"], r["k"], r["t"], r["tau"]] for r in recs])
    np.testing.assert_array_equal(cells, g["rec_cell"])           # record order
    np.testing.assert_array_equal([r["which"] for r in recs], g["rec_which"])
    np.testing.assert_array_equal([r["side"] for r in recs], g["rec_side"])
    for i, r in enumerate(recs):
        assert rel(r["Q"], g["rec_Q"][i]) < 1e-10
        assert rel(r["QR"], g["rec_QR"][i]) < 1e-10
        assert r["d"] == pytest.approx(g["rec_d"][i], rel=1e-12)
        assert r["lb"] == pytest.approx(g["rec_lb"][i], rel=1e-9, abs=1e-12)
    np.testing.assert_allclose(np.array(out["prob_lower_save"], float), g["prob_lower_save"],
                               rtol=1e-9)
    K = g["K"]
    A = np.array([[out["A_union"][t][k][o] for t in range(T)]
                  for o in range(len(K)) for k in range(K[o])])
    b = np.array([[out["b_union"][t][k][o] for t in range(T)]
                  for o in range(len(K)) for k in range(K[o])])
    np.testing.assert_allclose(A, g["A_union"], rtol=1e-14, atol=1e-15)
    np.testing.assert_allclose(b, g["b_union"], rtol=1e-13)


@pytest.mark.parametrize("name", ["cycle_o2_t8", "cycle_o1_t12"])
def test_affine_cycle_matches_reference(golden, name):
    g = golden(name)
    T = int(g["T"])
    out = orc.affine_generator(ovehicles_from_fixture(g), T, T, g["ref_traj"], with_l4=False)
    recs = out["records"]
    np.testing.assert_array_equal([r["which"] for r in recs], g["aff_which"])
    np.testing.assert_array_equal([r["side"] for r in recs], g["aff_side"])
    np.testing.assert_allclose([r["margin"] for r in recs], g["aff_margin"], rtol=1e-12)
    np.testing.assert_allclose([r["rhs"] for r in recs], g["aff_rhs"], rtol=1e-13)


@pytest.mark.parametrize("name", REFLOOP)
def test_generators_match_reference_loops(golden, name):
    """The oracle's restated generator glue against the reference's OWN loops
    (v8ideal/__init__.py:781-964 and :1378-1539 run by make_golden.py with a recording cp):
    constraint order, step and side exact; n, rhs, the state statistics, prob_lower_save and
    the saved moments (save_moments :2575-2618) to rounding -- including a T < ph step on
    injected ideal trajectories (the Tpred = T switch, :885-888)."""
    g = golden(name)
    K, T, ph, cells, yaws, ideal = refloop_inputs(g)
    ovs = [orc.OVehicle(ph, np.asarray(g["past"][o]).reshape(1, 2), np.ones(K[o]) / K[o],
                        cells[o], yaws[o], np.zeros((K[o], 2)), np.array([4.5, 2.5]))
           for o in range(len(K))]
    ideal_trajs = None
    if ideal is not None:
        it = iter(ideal)
        ideal_trajs = {o: {k: next(it) for k in range(K[o])} for o in range(len(K))}
    mk = orc.minkowski_generator(ovs, T, ph, g["ref_traj"], ideal_trajs=ideal_trajs,
                                 with_l4=False)
    recs = mk["records"]
    np.testing.assert_array_equal([r["t"] for r in recs], g["mk_t"])
    np.testing.assert_array_equal([r["side"] for r in recs], g["mk_side"])
    assert rel([r["n"] for r in recs], g["mk_n"]) < 1e-12
    np.testing.assert_allclose([r["d"] for r in recs], g["mk_rhs"], rtol=1e-12)
    assert bool(mk["OVconstraint"]) == bool(g["mk_ovconstraint"])
    C = sum(K)
    sm = np.array([[mk["ov_state_mean"][j][o][k] for j in range(3)]
                   for o in range(len(K)) for k in range(K[o])], float)
    sc = np.array([[mk["ov_state_cov"][j][o][k] for j in range(3)]
                   for o in range(len(K)) for k in range(K[o])], float)
    np.testing.assert_array_equal(sm, g["mk_state_mean"])
    np.testing.assert_array_equal(sc, g["mk_state_cov"])
    if T == ph:
        np.testing.assert_allclose(np.array(mk["prob_lower_save"], float),
                                   g["mk_prob_lower_save"], rtol=1e-9)
    mom = mk["moments"]
    for c, (o, k) in enumerate([(o, k) for o in range(len(K)) for k in range(K[o])]):
        for t in range(T):
            np.testing.assert_array_equal(mom["mean_p0p1"][o][k][t], g["mom_mean"][c, t])
            np.testing.assert_array_equal(mom["cov_p0p1"][o][k][t], g["mom_cov"][c, t])
            for tau in range(t):
                np.testing.assert_array_equal(mom["cross_cov"][o][k][t][tau],
                                              g["mom_xcov"][c, t, tau])
    assert len(recs) == C * T * (T - 1) // 2
    if "aff_t" in g.files:
        af = orc.affine_generator(ovs, T, ph, g["ref_traj"], with_l4=False)["records"]
        np.testing.assert_array_equal([r["t"] for r in af], g["aff_t"])
        np.testing.assert_array_equal([r["side"] for r in af], g["aff_side"])
        assert rel([r["n"] for r in af], g["aff_n"]) < 1e-13
        np.testing.assert_allclose([r["rhs"] for r in af], g["aff_rhs"], rtol=1e-12)


def test_predict_ideal_with_injected_draws(golden):
    g = golden("ideal_rollout")
    mom = dict(mean_p0p1=[list(g["mean"])], cov_p0p1=[list(g["cov"])],
               cross_cov=[[[list(g["xcov"][k][t]) for t in range(g["xcov"].shape[1])]
                           for k in range(2)]])
    ns, Tn = g["traj"].shape[1], g["traj"].shape[2]
    traj = orc.predict_ideal(mom, [2], Tn, ns, x0s=[list(g["x0"])],
                             Zs=[[list(g["Z"][k]) for k in range(2)]])
    for k in range(2):
        np.testing.assert_allclose(traj[0][k], g["traj"][k], rtol=1e-13)


def test_ideal_data_idx_fallback():
    """K grew since the moments were saved: extra modes reuse the last saved mode
    (v8ideal/__init__.py:2650-2656)."""
    rng = np.random.default_rng(0)
    T = 5
    cells = [[rng.normal(size=(200, T, 2)).cumsum(1)]]
    mom = orc.save_moments(cells, T)
    traj = orc.predict_ideal(mom, [3], T - 1, 16, seed=7)
    assert set(traj[0].keys()) == {0, 1, 2}
    # same source moments, different RNG cells -> same distribution, different draws
    assert not np.allclose(traj[0][1], traj[0][2])


def test_philox_known_answer():
    """Philox4x32-10 known-answer vector (Salmon et al., Random123 kat_vectors: counter 0,
    key 0)."""
    from oracle import philox
    w = philox.philox4x32(0, 0, 0, 0, 0)
    assert [int(x) for x in w] == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    w = philox.philox4x32(0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff,
                          0xffffffffffffffff)
    assert [int(x) for x in w] == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]


def _ideal_from_fixture(g):
    K = [int(k) for k in g["K"]]
    ideal, j = {}, 0
    for o, k_o in enumerate(K):
        ideal[o] = {}
        for k in range(k_o):
            ideal[o][k] = g["ideal"][j]
            j += 1
    return ideal


@pytest.mark.parametrize("scaled,pre", [(True, "s"), (False, "sr")])   # scale / _affine_robust
def test_affine_scale_generator_matches_reference(golden, scaled, pre):
    """compute_obstacle_constraints_GMM_affine_scale_ideal restated (v8ideal/__init__.py:
    2074-2456) vs the golden made with the reference's compute_scale / predict_moments /
    choose_closest_tangent: the T == ph step, then a T < ph step on injected ideal clouds that
    loads the first step's meanNtangent (mode matching, const_idx override)."""
    g = golden("affine_scale")
    T = int(g["T"])
    ovs = ovehicles_from_fixture(g)
    g1 = orc.affine_scale_generator(ovs, T, T, g["ref1"], scaled=scaled)
    mean1, tan1, _, _, ci1 = g1["meanNtangent"]
    g2 = orc.affine_scale_generator(ovs, T - 1, T, g["ref2"], x_init=g["x_init"],
                                    loaded=(mean1, tan1, ci1), ideal_trajs=_ideal_from_fixture(g),
                                    scaled=scaled)
    for i, out in ((1, g1), (2, g2)):
        recs = out["records"]
        np.testing.assert_array_equal([r["which"] for r in recs], g[f"{pre}{i}_which"])
        np.testing.assert_array_equal([r["side"] for r in recs], g[f"{pre}{i}_side"])
        for key, rtol in (("d", 1e-13), ("margin", 1e-12), ("rhs", 1e-13), ("scale", 1e-12),
                          ("m", 1e-13)):
            np.testing.assert_allclose([r[key] for r in recs], g[f"{pre}{i}_{key}"], rtol=rtol)
    assert set(g[f"{pre}2_which"]) <= {-1, 0, 1}
    if not scaled:
        assert np.all(g["sr1_scale"] == 1.0) and np.all(g["sr2_scale"] == 1.0)


def test_batched_scenes_allocate_risk_per_scene():
    """Several planning steps in one cycle keep eps_ura = 0.05 / O of their own scene
    (v8ideal/__init__.py:2920-2926): the batched risk table is the per-scene tables stacked."""
    import scipy.stats
    from ccmpc import risk
    scene_K = [[2, 1, 3], [1], [2, 2]]
    got = risk.scenes_cell_risk(scene_K, 8)
    want = []
    for K in scene_K:
        eps = orc.EPS_TOTAL / len(K) / 8
        for k in K:
            want += [[scipy.stats.chi2.ppf(1 - eps, 2), scipy.stats.chi2.ppf(orc.TARGET_P, 2),
                      scipy.stats.norm.ppf(1 - eps)]] * k
    np.testing.assert_allclose(got, np.array(want), rtol=1e-14)


# ---- reference-code pins of the restated glue (make_golden.py main_reference_glue) ----------
def test_make_ovehicles_matches_reference_from_trajectron(golden):
    """The oracle's make_ovehicles / from_trajectron restatement against the reference's own
    OVehicle.from_trajectron (ovehicle.py:24-117) run on the same sampler-shaped input: same
    kept modes, the same particles in the same order, pmf, init_center and yaws."""
    g = golden("ovehicle_l4")
    T = int(g["T"])
    O = g["pred"].shape[0]
    ovs = orc.make_ovehicles(g["pred"], g["z"], g["latent_pmf"], g["minpos"],
                             list(g["past"]), [g["bbox"]] * O, T)
    np.testing.assert_array_equal([ov.n_states for ov in ovs], g["K"])
    c0 = 0
    for o, ov in enumerate(ovs):
        np.testing.assert_array_equal(ov.latent_pmf, g["pmf_out"][o, :ov.n_states])
        np.testing.assert_array_equal(ov.init_center, g["init_center"][o, :ov.n_states])
        for k in range(ov.n_states):
            n = g["counts"][c0 + k]
            off = int(np.sum(g["counts"][:c0 + k]))
            np.testing.assert_array_equal(ov.pred_positions[k], g["positions"][off:off + n])
            np.testing.assert_array_equal(ov.pred_yaws[k], g["yaws"][off:off + n])
        c0 += ov.n_states


def test_l4_matches_reference_util(golden):
    """vertices_of_bboxes + compute_L4_outerapproximation restated vs midlevel/util.py's own
    get_vertices_from_centers / compute_L4_outerapproximation (:104-124, :171-200)."""
    g = golden("ovehicle_l4")
    T = int(g["T"])
    off = 0
    for c, n in enumerate(g["counts"]):
        ps, yw = g["positions"][off:off + n], g["yaws"][off:off + n]
        off += n
        for t in range(T):
            theta = np.mean(yw[:, t])
            assert theta == g["yaw_mean"][c, t]
            A, b = orc.compute_L4_outerapproximation(
                theta, orc.vertices_of_bboxes(ps[:, t], yw[:, t], g["bbox"]))
            np.testing.assert_array_equal(A, g["A"][c, t])
            np.testing.assert_allclose(b, g["b"][c, t], rtol=1e-15)


def ideal_ref_inputs(g):
    """ideal_ref.npz -> (moments dict of the oracle's save_moments format, x0s, Zs)."""
    import importlib.util
    import os
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "make_golden.py")
    spec = importlib.util.spec_from_file_location("make_golden", here)
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    K, T = g["mean_in"].shape[0], int(g["T"])
    mom = dict(mean_p0p1=[[g["mean_in"][k] for k in range(K)]],
               cov_p0p1=[[g["cov_in"][k] for k in range(K)]],
               cross_cov=[[g["xcov_in"][k] for k in range(K)]])
    return mom, [list(g["x0"])], [mg.ideal_noise(int(g["zseed"]), K, T, int(g["n"]))], mg


def test_predict_ideal_matches_reference_function(golden):
    """The oracle's predict_ideal with injected draws against the reference's own
    MidlevelAgent.predict_ideal (v8ideal/__init__.py:2620-2711, 1e6 samples as written)."""
    g = golden("ideal_ref")
    mom, x0s, Zs, _ = ideal_ref_inputs(g)
    K, T, n = g["mean_in"].shape[0], int(g["T"]), int(g["n"])
    traj = orc.predict_ideal(mom, [K], T, n, x0s=x0s, Zs=Zs)
    for k in range(K):
        np.testing.assert_allclose(traj[0][k][g["rows"]], g["traj_rows"][k], rtol=1e-13)
        np.testing.assert_allclose(traj[0][k].mean(axis=0), g["traj_mean"][k], rtol=1e-12)


def test_sampler_restatement_modes_agree():
    """The sampler restatement's upstream-shaped modes (injected z / eps, per-particle GMM
    parameters as p_y_xz emits them) reduce to the synthetic mode on the same draws.
    PARITY UNPINNED upstream (Trajectron++ absent)."""
    rng = np.random.default_rng(0)
    L, T, n = 5, 6, 400
    gmm = np.zeros((L, T, 5), np.float32)
    gmm[..., 0] = rng.normal(0, 0.2, (L, T))
    gmm[..., 1] = rng.normal(0, 1, (L, T))
    gmm[..., 2:4] = np.log(rng.uniform(0.05, 0.5, (L, T, 2)))
    gmm[..., 4] = rng.uniform(-0.9, 0.9, (L, T))
    init = np.array([10.0, -3.0, 0.4, 6.0])
    cdf = np.cumsum(np.full(L, 1.0 / L))
    z, pos = orc.sample_unicycle(init, cdf, gmm, n, T, 0.5, 17, ov=2)
    z2, pos2 = orc.sample_unicycle(init, None, gmm, n, T, 0.5, 17, ov=2, z=z)
    np.testing.assert_array_equal(pos2, pos)
    eps = rng.standard_normal((n, T, 2)).astype(np.float32)
    _, a = orc.sample_unicycle(init, None, gmm, n, T, 0.5, 0, z=z, eps=eps)
    _, b = orc.sample_unicycle(init, None, gmm[z], n, T, 0.5, 0, z=z, eps=eps, per_particle=True)
    np.testing.assert_array_equal(a, b)
    # |rho| = 1 stays finite through GMM2D's clamp of 1 - rho^2
    pp = gmm[z].copy()
    pp[..., 4] = 1.0
    _, c = orc.sample_unicycle(init, None, pp, n, T, 0.5, 0, z=z, eps=eps, per_particle=True)
    assert np.all(np.isfinite(c))
