"""The half-space tail's device arithmetic on the reference's own component goldens, and the
reference's failure modes through the real cycle kernels.

Part 1 feeds the golden vectors that tests/golden/make_golden.py recorded from the reference's
makeconstraint.py (compute_mvoe, choose_closest_tangent incl. 20 exact ties under strict '<',
compute_lower_bound / compute_scale, predict_moments) to ccmpc_selftest, which runs the same
__device__ functions the fused cycle runs per record (constraints.hpp).

Part 2 builds inputs on which the reference raises -- a singular tau block or MVOE solve, an
infinite tangent slope (ref_y == mean_y), N_k < 2, a non-PD conditional covariance in
predict_ideal, no real tangent -- and checks the record status the kernels write, that the
oracle (numpy/scipy like the reference) raises there, and the exception the drop-in planner
raises for that status (ccmpc._lib.record_error).
"""
import warnings

import numpy as np
import pytest
import torch

from oracle import ccmpc_oracle as orc

pytestmark = pytest.mark.gpu


def _selftest(kind, rows, out_width, tol=1e-8, maxiter=1000):
    from ccmpc import _lib, engine
    x = torch.as_tensor(np.ascontiguousarray(rows, np.float64), device="cuda")
    n = x.shape[0]
    y = torch.full((n, out_width), np.nan, dtype=torch.float64, device="cuda")
    _lib.check(_lib.load().ccmpc_selftest(kind, n, engine._p(x), engine._p(y), tol, maxiter,
                                          engine._stream()), "ccmpc_selftest")
    return y.cpu().numpy()


def _m(a):
    return np.asarray(a, np.float64).reshape(-1, 4)


def _rel(a, b):
    return np.linalg.norm(np.asarray(a) - b) / max(np.linalg.norm(b), 1e-300)


# ---- part 1: component goldens ---------------------------------------------------------------
def test_mvoe_golden_on_device(gpu, golden):
    """All 160 SPD pairs of mvoe.npz, incl. the near-degenerate S2 ~ 1e-21 and the (Q, R^2 I)
    shape: Q within 1e-9 relative Frobenius (bar 1e-5), beta within 1e-8 (the reformulated
    fixed point may stop one step earlier or later at the tol = 1e-8 threshold)."""
    from ccmpc import _lib
    g = golden("mvoe")
    y = _selftest(_lib.SELFTEST_MVOE, np.hstack((_m(g["S1"]), _m(g["S2"]))), 6)
    assert np.all(y[:, 5] == 1.0)
    worst_q = max(_rel(y[i, 1:5].reshape(2, 2), g["Q"][i]) for i in range(len(g["beta"])))
    worst_b = np.max(np.abs(y[:, 0] - g["beta"]) / np.abs(g["beta"]))
    assert worst_q < 1e-9, worst_q
    assert worst_b < 1e-8, worst_b


def test_tangent_golden_on_device_including_ties(gpu, golden):
    """All 200 cases of tangent.npz.  The first 20 put the reference point on the mean: the two
    candidate distances differ only by the rounding of proj +/- delta and the reference's strict
    '<' resolves them both ways; `which` must agree bit for bit on every case."""
    from ccmpc import _lib
    g = golden("tangent")
    rows = np.hstack((g["mu"], _m(g["Sigma"]), g["c"][:, None], g["m"][:, None], g["a"]))
    y = _selftest(_lib.SELFTEST_TANGENT, rows, 5)
    assert np.all(y[:, 4] == 0)
    np.testing.assert_array_equal(y[:, 3].astype(int), g["which"])
    np.testing.assert_array_equal(y[:, 0:2], g["n"])
    np.testing.assert_allclose(y[:, 2], g["d"], rtol=1e-15, atol=1e-12)
    assert 0 < np.sum(y[:20, 3]) < 20        # the ties really go both ways


def test_lower_bound_and_scale_golden_on_device(gpu, golden):
    from ccmpc import _lib
    g = golden("lower_bound")
    chi_p = orc.scipy.stats.chi2.ppf(orc.TARGET_P, df=2)
    rows = np.hstack((_m(g["cov_infer"]), _m(g["cov_mu"]), _m(g["cov_t"]), g["gamma"][:, None],
                      np.full((len(g["eps"]), 1), chi_p)))
    y = _selftest(_lib.SELFTEST_BOUND, rows, 2)
    np.testing.assert_allclose(y[:, 0], g["lower_bound"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(y[:, 1], g["scale"], rtol=1e-12)


def test_predict_moments_golden_through_the_moment_kernel(gpu, golden):
    """predict_moments.npz (ragged N from 5 to 2048): each case's (p_t, p_tau) clouds become a
    T = 2 cell of a device particle store (slot 0 = tau, slot 1 = t), the moments kernel makes
    its 4x4 covariance and the device pair_moments splits it -- against the reference's
    np.cov-based outputs."""
    from ccmpc import _lib, engine
    g = golden("predict_moments")
    offs = g["offsets"]
    cells = []
    for i in range(len(offs) - 1):
        p = g["points"][:, offs[i]:offs[i + 1]]
        cells.append(np.stack((p[2:4].T, p[0:2].T), axis=1))       # (N, 2 steps, xy)
    store = engine.ParticleStore.from_cells(cells, device=gpu)
    _, cov = engine.moments(store)
    rows = np.hstack((cov.cpu().numpy().reshape(-1, 16), np.ones((len(cells), 2))))
    y = _selftest(_lib.SELFTEST_PAIR, rows, 14)
    for i in range(len(cells)):
        assert _rel(y[i, 0:4].reshape(2, 2), g["cov_infer"][i]) < 1e-8   # Schur complement
        assert _rel(y[i, 4:8].reshape(2, 2), g["cov_mu"][i]) < 1e-11
        assert _rel(y[i, 8:12].reshape(2, 2), g["cov_t"][i]) < 1e-12


def test_no_real_tangent_status(gpu):
    """n^T Sigma n <= 0: the reference returns (None, None, None, None)
    (makeconstraint.py:163-165, 193-194); the device reports CCMPC_REC_NO_TANGENT."""
    from ccmpc import _lib
    sig = [[-1.0, 0.0, 0.0, -2.0], [0.0, 0.0, 0.0, 0.0], [1.0, 0.0, 0.0, 1.0]]
    rows = np.array([[5.0, 1.0, *s, 1.0, 0.7, 9.0, -3.0] for s in sig])
    y = _selftest(_lib.SELFTEST_TANGENT, rows, 5)
    np.testing.assert_array_equal(y[:, 4], [_lib.REC_NO_TANGENT, _lib.REC_NO_TANGENT, 0])
    for s in sig[:2]:
        assert orc.choose_closest_tangent(np.array([5.0, 1.0]), np.array(s).reshape(2, 2), 1.0,
                                          0.7, np.array([9.0, -3.0]))[0] is None
    with pytest.raises(ValueError):      # v8ideal/__init__.py:925 unpacks it into 3 names
        raise _lib.record_error(_lib.REC_NO_TANGENT, "t")


# ---- part 2: failure modes through the cycle -------------------------------------------------
class Params:
    def __init__(self, O, K, frame):
        self.O, self.K, self.frame = O, np.asarray(K), frame


def _dyadic_cell(rng, n, T, base=(64.0, -32.0)):
    """A cloud whose every coordinate is a multiple of 1/64 near `base`, so sums and the mean
    (n a power of two) are exact in both the kernel's shifted Gram sums and np.mean."""
    steps = np.arange(1, T + 1)[None, :, None] * np.array([2.0, 0.5])
    noise = rng.integers(-256, 257, size=(n, T, 2)) / 64.0
    drift = np.cumsum(rng.integers(-8, 9, size=(n, T, 2)) / 64.0, axis=1)
    return np.asarray(base)[None, None, :] + steps + noise + drift


def _run_cycle(cells, ref, gpu):
    from ccmpc import cycle, engine
    store = engine.ParticleStore.from_cells(cells, device=gpu)
    cyc = cycle.MinkowskiCycle(store, [len(cells)], ref)
    cyc.run()
    return cyc.records()


def _oracle_raises(cells, ref, T):
    ovs = [orc.OVehicle(T, cells[0][:1, 0] - 1.0, np.ones(len(cells)) / len(cells), cells,
                        [orc._step_yaws(c, cells[0][0, 0] - 1.0, T) for c in cells],
                        np.zeros((len(cells), 2)), np.array([4.5, 2.5]))]
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        try:
            orc.minkowski_generator(ovs, T, T, ref, with_l4=False)
        except Exception as e:              # noqa: BLE001 - the type is what is compared
            return e
    return None


def _planner_raises(cells, ref, T, gpu):
    from ccmpc import ovehicle, planner
    ovs = ovehicle.scene_from_positions([cells], [cells[0][0, 0] - 1.0], device=gpu)
    agent = planner.MidlevelAgent(prediction_horizon=T, device=gpu)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        try:
            agent.compute_obstacle_constraints_GMM_Minkowski_idealprediction(
                Params(1, [len(cells)], 10), ovs, None, None, None,
                orc.eps_ura_matrix([len(cells)]), None, T, ref)
        except Exception as e:              # noqa: BLE001
            return e
    return None


def test_singular_tau_block(gpu):
    """Every particle of the cell shares its y at step s: cov_tau at s is singular
    (np.linalg.inv raises, makeconstraint.py:63) and so is cov_infer at t = s (scipy solve
    raises, :21).  Records with t == s or tau == s carry CCMPC_REC_SINGULAR, the rest are OK;
    the oracle and the planner both raise LinAlgError."""
    from ccmpc import _lib
    T, s = 5, 2
    rng = np.random.default_rng(7)
    cell = _dyadic_cell(rng, 512, T)
    cell[:, s, 1] = cell[0, s, 1]
    ref = np.array([[cell[:, t, 0].mean() - 9.0, cell[:, t, 1].mean() + 4.0] for t in range(T)])
    h = _run_cycle([cell], ref, gpu).reshape(-1)
    t_, tau_ = h["t_tau"] >> 16, h["t_tau"] & 0xFFFF
    bad = (t_ == s) | (tau_ == s)
    assert np.all(h["status"][bad] == _lib.REC_SINGULAR)
    assert np.all(h["status"][~bad] == 0)
    assert isinstance(_oracle_raises([cell], ref, T), np.linalg.LinAlgError)
    assert isinstance(_planner_raises([cell], ref, T, gpu), np.linalg.LinAlgError)


def test_infinite_slope_when_ref_y_equals_mean_y(gpu):
    """ref_traj[t][1] == mean_y(t) exactly: m = -(dx) / 0 (v8ideal/__init__.py:923) is
    infinite.  The reference's candidate distances are NaN and it indexes its candidate list
    with None (TypeError); the records of that t carry CCMPC_REC_NONFINITE."""
    from ccmpc import _lib
    T, s = 5, 3
    rng = np.random.default_rng(11)
    cell = _dyadic_cell(rng, 1024, T)
    ref = np.array([[cell[:, t, 0].mean() - 9.0, cell[:, t, 1].mean() + 4.0] for t in range(T)])
    ref[s, 1] = cell[:, s, 1].mean()             # exact: dyadic values, n = 2^10
    h = _run_cycle([cell], ref, gpu).reshape(-1)
    t_ = h["t_tau"] >> 16
    assert np.all(h["status"][t_ == s] == _lib.REC_NONFINITE)
    assert np.all(h["status"][t_ != s] == 0)
    e = _oracle_raises([cell], ref, T)
    assert isinstance(e, (TypeError, ValueError)), e
    pe = _planner_raises([cell], ref, T, gpu)
    assert isinstance(pe, _lib.NonFiniteRecordError) and isinstance(pe, type(e)), pe


def test_single_particle_cell(gpu):
    """N_k = 1: np.cov(ddof=1) is NaN, scipy.linalg.solve rejects it (ValueError); every record
    of the cell is CCMPC_REC_NONFINITE and the cell's neighbour is untouched."""
    from ccmpc import _lib
    T = 4
    rng = np.random.default_rng(3)
    good = _dyadic_cell(rng, 256, T)
    one = good[:1] + 0.5
    ref = np.array([[good[:, t, 0].mean() - 9.0, good[:, t, 1].mean() + 4.0] for t in range(T)])
    h = _run_cycle([good, one], ref, gpu)
    assert np.all(h[0]["status"] == 0)
    assert np.all(h[1]["status"] == _lib.REC_NONFINITE)
    e = _oracle_raises([good, one], ref, T)
    assert isinstance(e, ValueError), e
    assert isinstance(_planner_raises([good, one], ref, T, gpu), ValueError)


def test_not_pd_conditional_covariance_in_predict_ideal(gpu):
    """Saved moments whose consecutive-step conditional covariance cov_{t+1} - A C^T is not PD:
    np.linalg.cholesky raises in the reference (v8ideal/__init__.py:2693); the rollout kernels
    report CCMPC_REC_NOT_PD for that cell only."""
    from ccmpc import _lib, engine
    T = 4
    rng = np.random.default_rng(5)
    cells = [_dyadic_cell(rng, 512, T), _dyadic_cell(rng, 512, T)]
    store = engine.ParticleStore.from_cells(cells, device=gpu)
    mean, cov = engine.moments(store)
    bad = cov.clone()
    # cell 1: Cov(x_2, x_1) = 2 L_2 L_1^T, so cov_2 - C cov_1^-1 C^T = -3 cov_2
    c = bad[1]
    c[4:6, 2:4] = 2.0 * torch.linalg.cholesky(c[4:6, 4:6]) @ torch.linalg.cholesky(c[2:4, 2:4]).T
    c[2:4, 4:6] = c[4:6, 2:4].T
    src = torch.tensor([0, 1], dtype=torch.int32, device=gpu)
    _, status = engine.ideal_rollout(mean, bad, src, T - 1, 64, seed=1)
    assert status.cpu().numpy().tolist() == [0, _lib.REC_NOT_PD]
    _, _, st2 = engine.ideal_moments(mean, bad, src, T - 1, 4096, seed=1)
    assert st2.cpu().numpy().tolist() == [0, _lib.REC_NOT_PD]
    m, cv = mean.cpu().numpy(), bad.cpu().numpy()
    mom = dict(mean_p0p1=[[m[k] for k in range(2)]],
               cov_p0p1=[[[cv[k][2 * t:2 * t + 2, 2 * t:2 * t + 2] for t in range(T)]
                          for k in range(2)]],
               cross_cov=[[[[cv[k][2 * t:2 * t + 2, 2 * u:2 * u + 2] for u in range(T)]
                            for t in range(T)] for k in range(2)]])
    with pytest.raises(np.linalg.LinAlgError):
        orc.predict_ideal(mom, [2], T - 1, 16, seed=1)
    with pytest.raises(np.linalg.LinAlgError):
        raise _lib.record_error(_lib.REC_NOT_PD, "predict_ideal")
