"""GPU parity at the shapes of BASELINE.json configs[3] (C4) and configs[4] (C5).

C4: a batch of 64 independent scenes x 4 OVs at ph = 12 in ONE ccmpc_minkowski_cycle launch.
Every scene is its own planning step (the reference plans one scene per agent,
v8ideal/__init__.py:2934-2976) with its own reference trajectory and its own risk allocation
(eps_ura = 0.05 / O, :2920-2926), so each scene's records are compared with the oracle's
Minkowski generator (v8ideal/__init__.py:781-964, golden-pinned to makeconstraint.py) run on
that scene alone.

C5: ph = 40, 8 OVs: all T(T-1)/2 = 780 coinciding (t, tau) MVOE half-spaces per cell.

Bar (BASELINE.json): Q and QR within 1e-5 relative Frobenius, centre within 1e-5 relative;
record order, `which` and `side` bit-exact.  Reduced particle counts keep the oracle to
seconds; the full-size runs check status, determinism and a few scenes against the oracle.
"""
import numpy as np
import pytest
import torch

from oracle import ccmpc_oracle as orc

pytestmark = pytest.mark.gpu

BASELINE_TOL = 1e-5


def _fro_rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def _oracle_ovs(ov_cells, pasts, T):
    out = []
    for cells, p in zip(ov_cells, pasts):
        past = np.asarray(p, float).reshape(1, 2)
        out.append(orc.OVehicle(T, past, np.ones(len(cells)) / len(cells), cells,
                                [orc._step_yaws(c, past[-1], T) for c in cells],
                                np.zeros((len(cells), 2)), np.array([4.5, 2.5])))
    return out


def _batch(seeds, O, N, T):
    from ccmpc import synthetic
    scenes = [synthetic.scene(s, O=O, N=N, T=T) for s in seeds]
    cells = [c for ovs, _, _ in scenes for o in ovs for c in o]
    scene_K = [[len(o) for o in ovs] for ovs, _, _ in scenes]
    refs = np.array([ref for _, ref, _ in scenes])
    return scenes, cells, scene_K, refs


def _check_scene(h, pl, want, tol_guard=1e-9):
    """Records of one scene (its cells' blocks, flattened in (ov, k, t, tau) order) vs the
    oracle's generator output for that scene."""
    recs = want["records"]
    h = h.reshape(-1)
    assert len(h) == len(recs)
    assert np.all(h["status"] == 0)
    t_tau = np.stack((h["t_tau"] >> 16, h["t_tau"] & 0xFFFF), axis=1)
    np.testing.assert_array_equal(t_tau, [(r["t"], r["tau"]) for r in recs])
    np.testing.assert_array_equal(h["which"], [r["which"] for r in recs])
    np.testing.assert_array_equal(h["side"], [r["side"] for r in recs])
    worst_q = worst_qr = worst_c = 0.0
    for i, r in enumerate(recs):
        Q = np.array([[h["q00"][i], h["q01"][i]], [h["q01"][i], h["q11"][i]]])
        QR = np.array([[h["r00"][i], h["r01"][i]], [h["r01"][i], h["r11"][i]]])
        worst_q = max(worst_q, _fro_rel(Q, r["Q"]))
        worst_qr = max(worst_qr, _fro_rel(QR, r["QR"]))
        worst_c = max(worst_c, _fro_rel(np.array([h["mean0"][i], h["mean1"][i]]), r["mean"]))
        assert h["lower_bound"][i] == pytest.approx(r["lb"], rel=1e-7, abs=1e-12)
    assert worst_q < BASELINE_TOL and worst_qr < BASELINE_TOL and worst_c < BASELINE_TOL
    assert worst_q < tol_guard and worst_qr < tol_guard, (worst_q, worst_qr)   # regression
    # the reference keeps prob_lower_save of the LAST cell of the scene (:947)
    np.testing.assert_allclose(pl[-1], want["prob_lower_save"], rtol=1e-7, atol=1e-12)
    return worst_q, worst_qr


def _scene_slices(scene_K):
    out, c0 = [], 0
    for K in scene_K:
        out.append(slice(c0, c0 + sum(K)))
        c0 += sum(K)
    return out


def test_c4_batch_64_scenes_per_scene_oracle_parity(gpu):
    """configs[3] shape at N = 1000 per OV: 64 scenes x 4 OVs, T = 12, one launch; every
    scene's records against the oracle run on that scene with that scene's ref_traj."""
    from ccmpc import cycle, engine
    T, O, N = 12, 4, 1000
    seeds = list(range(4000, 4064))
    scenes, cells, scene_K, refs = _batch(seeds, O, N, T)
    store = engine.ParticleStore.from_cells(cells, device=gpu)
    cyc = cycle.MinkowskiCycle(store, [k for K in scene_K for k in K], refs, scene_K=scene_K)
    assert cyc.cell_ref is not None
    cyc.run()
    h = cyc.records()
    pl = cyc.prob_lower.cpu().numpy()
    for s, sl in enumerate(_scene_slices(scene_K)):
        ovs, ref, pasts = scenes[s]
        want = orc.minkowski_generator(_oracle_ovs(ovs, pasts, T), T, T, ref, with_l4=False)
        _check_scene(h[sl], pl[sl], want)
    # sensitivity: every cell reading scene 0's reference must change other scenes' records
    wrong = cycle.MinkowskiCycle(store, [k for K in scene_K for k in K], refs,
                                 cell_ref=np.zeros(store.n_cells, np.int64), scene_K=scene_K)
    wrong.run()
    hw = wrong.records()
    sl1 = _scene_slices(scene_K)[1]
    assert not np.array_equal(hw[sl1]["d"], h[sl1]["d"])
    sl0 = _scene_slices(scene_K)[0]
    assert np.array_equal(hw[sl0].view(np.uint8), h[sl0].view(np.uint8))


def test_c4_batch_equals_per_scene_cycles(gpu):
    """A scene's records do not depend on the batch it rides in: the batched launch equals one
    cycle per scene, bit for bit (fixed reduction order, per-scene risk and reference)."""
    from ccmpc import cycle, engine
    T, O, N = 12, 4, 700
    seeds = list(range(4100, 4108))
    scenes, cells, scene_K, refs = _batch(seeds, O, N, T)
    store = engine.ParticleStore.from_cells(cells, device=gpu)
    cyc = cycle.MinkowskiCycle(store, [k for K in scene_K for k in K], refs, scene_K=scene_K)
    cyc.run()
    h = cyc.records()
    for s, sl in enumerate(_scene_slices(scene_K)):
        ovs, ref, _ = scenes[s]
        one = engine.ParticleStore.from_cells([c for o in ovs for c in o], device=gpu)
        c1 = cycle.MinkowskiCycle(one, scene_K[s], ref)
        c1.run()
        h1 = c1.records()
        assert np.array_equal(h1.view(np.uint8), h[sl].view(np.uint8)), s


def test_c4_full_size_batch(gpu):
    """configs[3] at full size on one GPU: 64 scenes x 4 OVs x 20000 particles, T = 12 (the
    balanced-mode launch).  Every record OK, replays bitwise identical, the fused launch equal
    to the two-call path, and four scenes (first, two inner, last) against the oracle."""
    from ccmpc import cycle, engine
    T, O, N = 12, 4, 20000
    seeds = list(range(4200, 4264))
    scenes, cells, scene_K, refs = _batch(seeds, O, N, T)
    store = engine.ParticleStore.from_cells(cells, device=gpu)
    assert store.n_bound > 2 ** 18
    cyc = cycle.MinkowskiCycle(store, [k for K in scene_K for k in K], refs, scene_K=scene_K)
    cyc.run()
    first = (cyc.mean.clone(), cyc.cov.clone(), cyc.rec.clone(), cyc.prob_lower.clone())
    for _ in range(2):
        cyc.rec.zero_()
        cyc.run()
        assert torch.equal(first[2], cyc.rec) and torch.equal(first[0], cyc.mean)
    cyc.run_unfused()
    assert torch.equal(first[1], cyc.cov) and torch.equal(first[2], cyc.rec)
    assert torch.equal(first[3], cyc.prob_lower)
    h = cyc.records()
    assert np.all(h["status"] == 0)
    pl = cyc.prob_lower.cpu().numpy()
    slices = _scene_slices(scene_K)
    for s in (0, 21, 42, 63):
        ovs, ref, pasts = scenes[s]
        want = orc.minkowski_generator(_oracle_ovs(ovs, pasts, T), T, T, ref, with_l4=False)
        _check_scene(h[slices[s]], pl[slices[s]], want)


def test_c5_t40_eight_ovs_oracle_parity(gpu):
    """configs[4] shape at N = 2000 per OV: T = 40, 8 OVs, all 780 (t, tau) half-spaces of
    every cell against the oracle."""
    from ccmpc import cycle, engine, synthetic
    T, O, N = 40, 8, 2000
    ovs, ref, pasts = synthetic.scene(5000, O=O, N=N, T=T)
    K = [len(o) for o in ovs]
    store = engine.ParticleStore.from_cells([c for o in ovs for c in o], device=gpu)
    cyc = cycle.MinkowskiCycle(store, K, ref)
    cyc.run()
    assert cyc.records().shape[1] == 780
    want = orc.minkowski_generator(_oracle_ovs(ovs, pasts, T), T, T, ref, with_l4=False)
    _check_scene(cyc.records(), cyc.prob_lower.cpu().numpy(), want, tol_guard=1e-6)


def test_c5_full_size(gpu):
    """configs[4] at full size: T = 40, 8 OVs x 50000 particles.  Every record OK, replays
    bitwise identical, fused == two calls; the first OV's clouds as a one-OV step against the
    oracle, and the batch's moments of those cells equal to that step's."""
    from ccmpc import cycle, engine, synthetic
    T, O, N = 40, 8, 50000
    ovs, ref, pasts = synthetic.scene(5001, O=O, N=N, T=T)
    K = [len(o) for o in ovs]
    store = engine.ParticleStore.from_cells([c for o in ovs for c in o], device=gpu)
    cyc = cycle.MinkowskiCycle(store, K, ref)
    cyc.run()
    rec0 = cyc.rec.clone()
    cyc.rec.zero_()
    cyc.run()
    assert torch.equal(rec0, cyc.rec)
    cyc.run_unfused()
    assert torch.equal(rec0, cyc.rec)
    h = cyc.records()
    assert np.all(h["status"] == 0)
    # OV 0 as a one-OV planning step (eps_ura = 0.05 / 1) against the oracle on that OV
    want = orc.minkowski_generator(_oracle_ovs(ovs[:1], pasts[:1], T), T, T, ref,
                                   with_l4=False)
    one = engine.ParticleStore.from_cells(ovs[0], device=gpu)
    c1 = cycle.MinkowskiCycle(one, [K[0]], ref)
    c1.run()
    _check_scene(c1.records(), c1.prob_lower.cpu().numpy(), want, tol_guard=1e-6)
    # and the batched cells of OV 0 carry the same moments as the one-OV cycle
    torch.testing.assert_close(cyc.mean[:K[0]], c1.mean, rtol=1e-14, atol=0)
    torch.testing.assert_close(cyc.cov[:K[0]], c1.cov, rtol=1e-12, atol=1e-14)
