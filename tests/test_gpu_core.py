"""GPU parity of the core kernels against the oracle and the reference's golden fixtures.

Tolerances: the BASELINE.json bar is 1e-5 relative (Frobenius) on ellipsoid shapes Q and
centres, bit-exact on integer outputs (which tangent, side, record order).  The kernels compute
in float64 and typically agree to ~1e-12; tighter checks below are regressions guards.
"""
import numpy as np
import pytest
import torch

from oracle import ccmpc_oracle as orc

from _cycle_inputs import cells_from_fixture, ovehicles_from_fixture

pytestmark = pytest.mark.gpu

BASELINE_TOL = 1e-5


def fro_rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def ccmpc():
    import ccmpc.engine as eng
    return eng


def oracle_cell_moments(cell):
    """np.mean / np.cov (ddof=1) of one (N, T, 2) cloud, rows (x_0, y_0, x_1, ...)."""
    N, T, _ = cell.shape
    X = cell.transpose(1, 2, 0).reshape(2 * T, N)
    return X.mean(axis=1), np.cov(X)


@pytest.mark.parametrize("T,counts", [
    (8, [300, 180, 420]),
    (1, [2, 3, 17]),
    (3, [5, 15, 16, 17, 63, 64, 65]),
    (12, [256, 97, 1000]),
    (9, [4, 2, 255, 256, 257]),          # 4-row-block (Scheme4) path from here to T = 12
    (10, [20000, 31, 4096]),             # > 64 items: two combine-tree levels
    (11, [700, 5, 1300]),
    (20, [33, 700]),
    (40, [129, 2051]),
])
def test_moments_f64_match_numpy(gpu, T, counts):
    eng = ccmpc()
    rng = np.random.default_rng(T * 1000 + len(counts))
    cells = [190 + np.cumsum(rng.normal(0, 0.5, size=(n, T, 2)), axis=1) for n in counts]
    store = eng.ParticleStore.from_cells(cells, device=gpu)
    mean, cov = eng.moments(store)
    mean, cov = mean.cpu().numpy(), cov.cpu().numpy()
    for j, c in enumerate(cells):
        m_ref, c_ref = oracle_cell_moments(c)
        np.testing.assert_allclose(mean[j].reshape(-1), m_ref, rtol=1e-13)
        assert fro_rel(cov[j], c_ref) < 1e-11
        np.testing.assert_array_equal(cov[j], cov[j].T)


@pytest.mark.parametrize("T", [8, 11])
def test_moments_f32_relative_store(gpu, T):
    """Trajectron++ hands float32 scene-relative positions; the reference adds minpos in
    float64 (v8ideal/__init__.py:486).  The F32 store keeps them relative + per-cell origin."""
    eng = ccmpc()
    rng = np.random.default_rng(5)
    minpos = np.array([123.25, -211.5])
    rel = [np.cumsum(rng.normal(0, 0.7, size=(n, T, 2)), axis=1).astype(np.float32) + 60
           for n in (511, 64, 3)]
    store = eng.ParticleStore(T, [r.shape[0] for r in rel], dtype=torch.float32, device=gpu,
                              origin=np.tile(minpos, (3, 1)))
    host = np.zeros((2 * T, store.ld), np.float32)
    for j, r in enumerate(rel):
        host[:, store.offsets[j]:store.offsets[j] + r.shape[0]] = r.transpose(1, 2, 0).reshape(
            2 * T, -1)
    store.pos.copy_(torch.from_numpy(host))
    mean, cov = eng.moments(store)
    for j, r in enumerate(rel):
        m_ref, c_ref = oracle_cell_moments(r + minpos)          # float32 + float64 -> float64
        np.testing.assert_allclose(mean[j].cpu().numpy().reshape(-1), m_ref, rtol=1e-13)
        assert fro_rel(cov[j].cpu().numpy(), c_ref) < 1e-11


@pytest.mark.parametrize("name", ["cycle_o2_t8", "cycle_o1_t12"])
def test_minkowski_records_match_reference_golden(gpu, golden, name):
    from ccmpc import risk
    eng = ccmpc()
    g = golden(name)
    T = int(g["T"])
    K = [int(k) for k in g["K"]]
    store = eng.ParticleStore.from_cells(cells_from_fixture(g), device=gpu)
    mean, cov = eng.moments(store)
    cr = torch.as_tensor(risk.cell_risk(risk.eps_ura(K), K, T), device=gpu)
    ref = torch.as_tensor(np.asarray(g["ref_traj"], float).reshape(1, T, 2), device=gpu)
    rec, pl = eng.minkowski(mean, cov, ref, cr)
    h = eng.halfspaces(rec).reshape(-1)
    assert len(h) == len(g["rec_d"])
    assert np.all(h["status"] == 0)
    # record order: (ov, k, t, tau) flattened as cell-major, pair p = t(t-1)/2 + tau
    t_tau = np.stack((h["t_tau"] >> 16, h["t_tau"] & 0xFFFF), axis=1)
    np.testing.assert_array_equal(t_tau, g["rec_cell"][:, 2:4])
    np.testing.assert_array_equal(h["which"], g["rec_which"])
    np.testing.assert_array_equal(h["side"], g["rec_side"])
    for i in range(len(h)):
        Q = np.array([[h["q00"][i], h["q01"][i]], [h["q01"][i], h["q11"][i]]])
        QR = np.array([[h["r00"][i], h["r01"][i]], [h["r01"][i], h["r11"][i]]])
        assert fro_rel(Q, g["rec_Q"][i]) < BASELINE_TOL
        assert fro_rel(QR, g["rec_QR"][i]) < BASELINE_TOL
        assert fro_rel(Q, g["rec_Q"][i]) < 1e-9          # regression guard
        c = np.array([h["mean0"][i], h["mean1"][i]])
        assert fro_rel(c, g["rec_mean"][i]) < 1e-13
        assert h["d"][i] == pytest.approx(g["rec_d"][i], rel=1e-11)
        assert h["lower_bound"][i] == pytest.approx(g["rec_lb"][i], rel=1e-8, abs=1e-12)
    # the reference keeps prob_lower_save of the LAST cell (v8ideal/__init__.py:947)
    np.testing.assert_allclose(pl.cpu().numpy()[-1], g["prob_lower_save"], rtol=1e-8)


@pytest.mark.parametrize("name", ["cycle_o2_t8", "cycle_o1_t12"])
def test_affine_records_match_reference_golden(gpu, golden, name):
    from ccmpc import risk
    eng = ccmpc()
    g = golden(name)
    T = int(g["T"])
    K = [int(k) for k in g["K"]]
    store = eng.ParticleStore.from_cells(cells_from_fixture(g), device=gpu)
    mean, cov = eng.moments(store)
    gam = torch.as_tensor(risk.cell_gamma(risk.eps_ura(K), K, T), device=gpu)
    ref = torch.as_tensor(np.asarray(g["ref_traj"], float).reshape(1, T, 2), device=gpu)
    h = eng.affine_records(eng.affine(mean, cov, ref, gam)).reshape(-1)
    assert np.all(h["status"] == 0)
    np.testing.assert_array_equal(h["which"], g["aff_which"])
    np.testing.assert_array_equal(h["side"], g["aff_side"])
    np.testing.assert_allclose(h["margin"], g["aff_margin"], rtol=1e-10)
    np.testing.assert_allclose(h["rhs"], g["aff_rhs"], rtol=1e-12)


def test_minkowski_random_cells_match_oracle(gpu):
    """Fresh seeded clouds (not the fixture): every record vs the oracle restatement."""
    from ccmpc import risk
    eng = ccmpc()
    rng = np.random.default_rng(11)
    T = 8
    ovs_cells = [[190 + np.cumsum(rng.normal(0, 0.6, size=(n, T, 2)), axis=1) for n in ns]
                 for ns in ((900, 700), (1200,), (64, 333, 2000))]
    K = [len(c) for c in ovs_cells]
    ovs = []
    for cells in ovs_cells:
        past = cells[0][:1, 0] - np.array([[3.0, 0.5]])
        ovs.append(orc.OVehicle(T, past, np.ones(len(cells)) / len(cells), cells,
                                [orc._step_yaws(c, past[-1], T) for c in cells],
                                np.zeros((len(cells), 2)), np.array([4.5, 2.5])))
    ego = np.array([170.0, 10.0])
    ref_traj = np.array([ego + [4.0 * (t + 1), 0.5 * (t + 1)] for t in range(T)])
    want = orc.minkowski_generator(ovs, T, T, ref_traj, with_l4=False)["records"]
    store = eng.ParticleStore.from_cells([c for cs in ovs_cells for c in cs], device=gpu)
    mean, cov = eng.moments(store)
    cr = torch.as_tensor(risk.cell_risk(risk.eps_ura(K), K, T), device=gpu)
    rec, _ = eng.minkowski(mean, cov, torch.as_tensor(ref_traj[None], device=gpu), cr)
    h = eng.halfspaces(rec).reshape(-1)
    assert len(h) == len(want)
    np.testing.assert_array_equal(h["which"], [r["which"] for r in want])
    np.testing.assert_array_equal(h["side"], [r["side"] for r in want])
    for i, r in enumerate(want):
        QR = np.array([[h["r00"][i], h["r01"][i]], [h["r01"][i], h["r11"][i]]])
        assert fro_rel(QR, r["QR"]) < 1e-9
        assert h["d"][i] == pytest.approx(r["d"], rel=1e-11)


def test_ideal_rollout_injected_draws_match_golden(gpu, golden):
    eng = ccmpc()
    g = golden("ideal_rollout")
    T_src = g["mean"].shape[1]
    Tn, ns = g["traj"].shape[2], g["traj"].shape[1]
    cov = np.zeros((2, 2 * T_src, 2 * T_src))
    for k in range(2):
        for t in range(T_src):
            cov[k, 2 * t:2 * t + 2, 2 * t:2 * t + 2] = g["cov"][k][t]
            for tau in range(t):
                cov[k, 2 * t:2 * t + 2, 2 * tau:2 * tau + 2] = g["xcov"][k][t][tau]
                cov[k, 2 * tau:2 * tau + 2, 2 * t:2 * t + 2] = g["xcov"][k][t][tau].T
    dev = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=gpu)
    Z = np.ascontiguousarray(np.asarray(g["Z"]).transpose(0, 1, 3, 2))      # [c][t][2][n]
    store, status = eng.ideal_rollout(dev(g["mean"]), dev(cov), dev([0, 1], torch.int32), Tn, ns,
                                      x0=dev(g["x0"]), Z=dev(Z))
    assert status.cpu().numpy().tolist() == [0, 0]
    for k in range(2):
        np.testing.assert_allclose(store.cell_positions(k), g["traj"][k], rtol=1e-12)


def _source_moments(gpu, T_src=8, seed=3):
    eng = ccmpc()
    rng = np.random.default_rng(seed)
    cells = [190 + np.cumsum(rng.normal(0, 0.4, size=(n, T_src, 2)), axis=1) for n in (3000, 800)]
    store = eng.ParticleStore.from_cells(cells, device=gpu)
    mean, cov = eng.moments(store)
    return cells, mean, cov


def test_ideal_rollout_philox_matches_oracle(gpu):
    eng = ccmpc()
    cells, mean, cov = _source_moments(gpu)
    T_src = mean.shape[1]
    Tn, ns, seed = T_src - 1, 1000, 1234
    src = torch.tensor([0, 1, 1], dtype=torch.int32, device=gpu)   # data_idx fallback
    store, status = eng.ideal_rollout(mean, cov, src, Tn, ns, seed=seed)
    assert status.cpu().numpy().tolist() == [0, 0, 0]
    mom = orc.save_moments([cells], T_src)
    want = orc.predict_ideal(mom, [3], Tn, ns, seed=seed)
    for k in range(3):
        np.testing.assert_allclose(store.cell_positions(k), want[0][k], rtol=1e-9, atol=1e-9)


def test_ideal_moments_fused_equals_materialised(gpu):
    eng = ccmpc()
    _, mean, cov = _source_moments(gpu)
    Tn = mean.shape[1] - 1
    src = torch.tensor([0, 1], dtype=torch.int32, device=gpu)
    for ns in (4099, 100_000):
        store, st = eng.ideal_rollout(mean, cov, src, Tn, ns, seed=77)
        m_a, c_a = eng.moments(store)
        m_b, c_b, st_b = eng.ideal_moments(mean, cov, src, Tn, ns, seed=77)
        assert st_b.cpu().numpy().tolist() == [0, 0]
        np.testing.assert_allclose(m_b.cpu().numpy(), m_a.cpu().numpy(), rtol=1e-12)
        assert fro_rel(c_b.cpu().numpy(), c_a.cpu().numpy()) < 1e-10


@pytest.mark.parametrize("T_src", [2, 9, 10, 17, 40])   # T = 1, 8 | 9, 16 | 17, 39
def test_ideal_moments_fused_equals_materialised_across_row_blocks(gpu, T_src):
    """Every row-block instance's edges (the fused kernel's plan table holds 8 RB steps), three
    cells from two sources, sample counts that leave ragged waves and a ragged last item."""
    eng = ccmpc()
    _, mean, cov = _source_moments(gpu, T_src=T_src)
    Tn = T_src - 1
    src = torch.tensor([1, 0, 1], dtype=torch.int32, device=gpu)
    for ns in (777, 70_001):
        store, st = eng.ideal_rollout(mean, cov, src, Tn, ns, seed=31)
        m_a, c_a = eng.moments(store)
        m_b, c_b, st_b = eng.ideal_moments(mean, cov, src, Tn, ns, seed=31)
        assert st.cpu().numpy().tolist() == [0, 0, 0] and st_b.cpu().numpy().tolist() == [0, 0, 0]
        np.testing.assert_allclose(m_b.cpu().numpy(), m_a.cpu().numpy(), rtol=1e-12)
        assert fro_rel(c_b.cpu().numpy(), c_a.cpu().numpy()) < 1e-10


def test_ideal_moments_full_size_properties(gpu):
    """BASELINE size (1e6 samples per cell): the sample moments of the rollout reproduce the
    conditional-Gaussian model it samples (mean_{t+1} + A (x0-mean_t) ...) to sampling error,
    and two launches are bitwise identical."""
    eng = ccmpc()
    _, mean, cov = _source_moments(gpu)
    Tn, ns = mean.shape[1] - 1, 1_000_000
    src = torch.tensor([0, 1], dtype=torch.int32, device=gpu)
    m1, c1, st = eng.ideal_moments(mean, cov, src, Tn, ns, seed=9)
    m2, c2, _ = eng.ideal_moments(mean, cov, src, Tn, ns, seed=9)
    assert torch.equal(m1, m2) and torch.equal(c1, c2)
    assert st.cpu().numpy().tolist() == [0, 0]
    # the sample moments reproduce the Gaussian the rollout propagates analytically
    # (v8ideal/__init__.py:2671-2700): slot t holds x_{t+1} = mu_{t+1} + A_t (x_t - mu_t) + L_t z,
    # so m_t = mu_{t+1} + A_t (m_{t-1} - mu_t), C_t = A_t C_{t-1} A_t^T + L_t L_t^T, C_{-1} = 0,
    # m_{-1} = x0 (the one shared draw); the lag-1 cross block is A_t C_{t-1}.
    c1, m1 = c1.cpu().numpy(), m1.cpu().numpy()
    mu, src_cov = mean.cpu().numpy(), cov.cpu().numpy()
    for k in range(2):
        blk = lambda M, i, j: M[2 * i:2 * i + 2, 2 * j:2 * j + 2]
        x0 = orc.ideal_x0(mu[k, 0], blk(src_cov[k], 0, 0), k, 9)
        m_prev, C_prev = x0, np.zeros((2, 2))
        for t in range(Tn):
            S_t, X = blk(src_cov[k], t, t), blk(src_cov[k], t + 1, t)
            A = X @ np.linalg.inv(S_t)
            LLt = blk(src_cov[k], t + 1, t + 1) - A @ X.T
            m = mu[k, t + 1] + A @ (m_prev - mu[k, t])
            C = A @ C_prev @ A.T + LLt
            got_C = blk(c1[k], t, t)
            # 1e6 samples: ~5 sigma of the sampling error of a mean / a covariance entry
            sd = np.sqrt(np.diag(C))
            assert np.all(np.abs(m1[k, t] - m) <= 5 * sd / np.sqrt(ns)), (k, t)
            assert np.all(np.abs(got_C - C) <= 5 * np.outer(sd, sd) * np.sqrt(2.0 / ns)), (k, t)
            if t > 0:
                got_X = blk(c1[k], t, t - 1)
                sdp = np.sqrt(np.diag(C_prev))
                assert np.all(np.abs(got_X - A @ C_prev) <=
                              5 * np.outer(sd, sdp) * np.sqrt(2.0 / ns)), (k, t)
            m_prev, C_prev = m, C


def test_moments_deterministic(gpu):
    eng = ccmpc()
    rng = np.random.default_rng(2)
    cells = [190 + rng.normal(size=(n, 8, 2)) for n in (50_000, 7, 12345)]
    store = eng.ParticleStore.from_cells(cells, device=gpu)
    a = eng.moments(store)
    b = eng.moments(store)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("scaled,pre", [(True, "s"), (False, "sr")])   # scale / _affine_robust
def test_affine_scale_records_match_reference_golden(gpu, golden, scaled, pre):
    """ccmpc_affine_scale (v8ideal/__init__.py:2074-2456) vs the reference-driven golden: the
    T == ph step from the particle cells, then the T < ph step from the ideal clouds with the
    slopes / tangent indices of the first step's meanNtangent matched per mode on the host."""
    from ccmpc import planner, risk
    eng = ccmpc()
    g = golden("affine_scale")
    T = int(g["T"])
    K = [int(k) for k in g["K"]]
    cr = torch.as_tensor(risk.cell_risk(risk.eps_ura(K), K, T), device=gpu)

    def check(h, i):
        h = h.reshape(-1)
        assert np.all(h["status"] == 0)
        np.testing.assert_array_equal(h["which"], g[f"{pre}{i}_which"])
        np.testing.assert_array_equal(h["side"], g[f"{pre}{i}_side"])
        np.testing.assert_allclose(h["s00"], g[f"{pre}{i}_scale"], rtol=1e-10)
        np.testing.assert_allclose(h["margin"], g[f"{pre}{i}_margin"], rtol=1e-10)
        np.testing.assert_allclose(h["rhs"], g[f"{pre}{i}_rhs"], rtol=1e-12)
        np.testing.assert_allclose(h["d"], g[f"{pre}{i}_d"], rtol=1e-12)

    store = eng.ParticleStore.from_cells(cells_from_fixture(g), device=gpu)
    mean, cov = eng.moments(store)
    ref1 = torch.as_tensor(g["ref1"][None], device=gpu)
    check(eng.affine_records(eng.affine_scale(mean, cov, ref1, cr, scaled=scaled)), 1)

    Tn = T - 1
    store2 = eng.ParticleStore.from_cells(list(g["ideal"]), device=gpu)
    mean2, cov2 = eng.moments(store2)
    m2 = mean2.cpu().numpy()
    tangent = np.zeros((sum(K), Tn))
    const = np.zeros((sum(K), Tn), np.int32)
    c0 = 0
    for o, k_o in enumerate(K):
        # the first step's saved means are the particle means either way (scale only changes
        # the spread); slopes and indices are the variant's own
        mean_l = [[g["load_mean"][c0 + j][t] for t in range(T)] for j in range(k_o)]
        picks = planner._match_modes(mean_l, g["x_init"], [m2[c0 + k] for k in range(k_o)],
                                     k_o, 10_000)
        for k, idx in enumerate(picks):
            tangent[c0 + k] = g[f"{pre}1_m"][(c0 + idx) * T:(c0 + idx + 1) * T][1:]
            const[c0 + k] = g[f"{pre}1_which"][(c0 + idx) * T:(c0 + idx + 1) * T][1:]
        c0 += k_o
    ref2 = torch.as_tensor(g["ref2"][None, :Tn], device=gpu)
    check(eng.affine_records(eng.affine_scale(mean2, cov2, ref2, cr, tangent, const,
                                              scaled=scaled)), 2)


def test_ideal_rollout_matches_reference_predict_ideal(gpu, golden):
    """Pinned to the reference's own MidlevelAgent.predict_ideal (v8ideal/__init__.py:
    2620-2711) run at its 1e6 samples with injected x0 and normals (tests/golden/ideal_ref.npz):
    the device rollout fed the same draws reproduces the kept sample rows, and the moment
    kernel over the device's 1e6-sample store reproduces the reference output's mean and
    covariance."""
    import importlib.util
    import os
    eng = ccmpc()
    g = golden("ideal_ref")
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "make_golden.py")
    spec = importlib.util.spec_from_file_location("make_golden", here)
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    K, T, n = g["mean_in"].shape[0], int(g["T"]), int(g["n"])
    T_src = g["mean_in"].shape[1]
    cov = np.zeros((K, 2 * T_src, 2 * T_src))
    for k in range(K):
        for t in range(T_src):
            cov[k, 2 * t:2 * t + 2, 2 * t:2 * t + 2] = g["cov_in"][k][t]
            for tau in range(t):
                cov[k, 2 * t:2 * t + 2, 2 * tau:2 * tau + 2] = g["xcov_in"][k][t][tau]
                cov[k, 2 * tau:2 * tau + 2, 2 * t:2 * t + 2] = g["xcov_in"][k][t][tau].T
    noise = mg.ideal_noise(int(g["zseed"]), K, T, n)
    Z = torch.empty((K, T, 2, n), dtype=torch.float64, device=gpu)
    for k in range(K):
        for t in range(T):
            Z[k, t] = torch.as_tensor(noise[k][t].T.copy(), device=gpu)
    del noise
    dev = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=gpu)
    store, status = eng.ideal_rollout(dev(g["mean_in"]), dev(cov), dev(list(range(K)), torch.int32),
                                      T, n, x0=dev(g["x0"]), Z=Z)
    assert status.cpu().numpy().tolist() == [0] * K
    mean, cv = eng.moments(store)
    rows = torch.as_tensor(g["rows"], device=gpu)
    for k in range(K):
        o = store.offsets[k]
        got = store.pos[:, o:o + n].index_select(1, rows).cpu().numpy()
        got = got.reshape(T, 2, -1).transpose(2, 0, 1)
        np.testing.assert_allclose(got, g["traj_rows"][k], rtol=1e-12)
        np.testing.assert_allclose(mean[k].cpu().numpy(), g["traj_mean"][k], rtol=1e-12)
        np.testing.assert_allclose(cv[k].cpu().numpy(), g["traj_cov"][k], rtol=1e-9,
                                   atol=1e-12 * np.abs(g["traj_cov"][k]).max())
