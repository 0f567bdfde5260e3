"""GPU parity at every point of BASELINE.json configs[2] (C3): one OV, ph = 8,
np in {1e3, 5e3, 2e4, 1e5} -- the exact scenes `bench.py`'s roofline_sweep times
(synthetic.scene(seed + 1000, O=1, N, T=8) with the bench's default seed), in the plain
(non-balanced) store, so the np = 1e5 point runs the same launch the sweep times: a cell of
~200 work items of 512 particles climbing the two-level combine tree with the fused half-space
tail.

Every record against the oracle's Minkowski generator (v8ideal/__init__.py:881-947,
golden-pinned to makeconstraint.py): record order, `which` and `side` exact, Q / QR / centre
within 1e-9 relative Frobenius (BASELINE bar 1e-5), lower bounds and prob_lower_save; the
moments against numpy's ddof=1 covariance; the fused launch bitwise equal to the two-call path
and to a graph replay.
"""
import numpy as np
import pytest
import torch

from oracle import ccmpc_oracle as orc

pytestmark = pytest.mark.gpu

BENCH_SEED = 20251015          # bench.py's --seed default
C3_POINTS = (1000, 5000, 20000, 100000)


def _fro_rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.mark.parametrize("N", C3_POINTS)
def test_c3_sweep_point_oracle_parity(gpu, N):
    from ccmpc import cycle, engine, synthetic
    T = 8
    ovs, ref, pasts = synthetic.scene(BENCH_SEED + 1000, O=1, N=N, T=T)
    K = [len(o) for o in ovs]
    cells = [c for o in ovs for c in o]
    store = engine.ParticleStore.from_cells(cells, device=gpu)
    assert store.n_bound <= 2 ** 18           # the plain (non-balanced) launch the sweep times
    cyc = cycle.MinkowskiCycle(store, K, ref)
    cyc.run()
    rec0, mean0, cov0, pl0 = (cyc.rec.clone(), cyc.mean.clone(), cyc.cov.clone(),
                              cyc.prob_lower.clone())
    # fused == unfused, bit for bit
    cyc.rec.zero_()
    cyc.run_unfused()
    assert torch.equal(rec0, cyc.rec) and torch.equal(cov0, cyc.cov)
    assert torch.equal(mean0, cyc.mean) and torch.equal(pl0, cyc.prob_lower)
    # a graph replay leaves the same bits (the workspace's counters returned to zero)
    cyc.rec.zero_()
    cyc.capture()
    cyc.replay()
    torch.cuda.synchronize(gpu)
    assert torch.equal(rec0, cyc.rec)

    # moments vs numpy (np.cov ddof=1 of the 2T trajectory vector)
    cov = cov0.cpu().numpy()
    for c, traj in enumerate(cells):
        X = traj.reshape(len(traj), 2 * T)
        np.testing.assert_allclose(cov[c], np.cov(X, rowvar=False), rtol=1e-10, atol=1e-12)

    # every record vs the oracle's generator on the same clouds
    past = np.asarray(pasts[0], float).reshape(1, 2)
    oov = orc.OVehicle(T, past, np.ones(K[0]) / K[0], ovs[0],
                       [orc._step_yaws(c, past[-1], T) for c in ovs[0]],
                       np.zeros((K[0], 2)), np.array([4.5, 2.5]))
    want = orc.minkowski_generator([oov], T, T, ref, with_l4=False)
    h = cyc.records().reshape(-1)
    recs = want["records"]
    assert len(h) == len(recs) == sum(K) * T * (T - 1) // 2
    assert np.all(h["status"] == 0)
    np.testing.assert_array_equal(np.stack((h["t_tau"] >> 16, h["t_tau"] & 0xFFFF), 1),
                                  [(r["t"], r["tau"]) for r in recs])
    np.testing.assert_array_equal(h["which"], [r["which"] for r in recs])
    np.testing.assert_array_equal(h["side"], [r["side"] for r in recs])
    wq = wqr = wc = 0.0
    for i, r in enumerate(recs):
        Q = np.array([[h["q00"][i], h["q01"][i]], [h["q01"][i], h["q11"][i]]])
        QR = np.array([[h["r00"][i], h["r01"][i]], [h["r01"][i], h["r11"][i]]])
        wq = max(wq, _fro_rel(Q, r["Q"]))
        wqr = max(wqr, _fro_rel(QR, r["QR"]))
        wc = max(wc, _fro_rel(np.array([h["mean0"][i], h["mean1"][i]]), r["mean"]))
        assert h["lower_bound"][i] == pytest.approx(r["lb"], rel=1e-7, abs=1e-12)
    assert wq <= 1e-9 and wqr <= 1e-9 and wc <= 1e-9, (wq, wqr, wc)
    np.testing.assert_allclose(pl0.cpu().numpy()[-1], want["prob_lower_save"], rtol=1e-7,
                               atol=1e-12)
