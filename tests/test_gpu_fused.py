"""GPU tests of the one-launch cycles, the L4 / heading kernel and the GMM sampler."""
import numpy as np
import pytest
import torch

from oracle import ccmpc_oracle as orc

from _cycle_inputs import cells_from_fixture, ovehicles_from_fixture

pytestmark = pytest.mark.gpu


def eng():
    import ccmpc.engine as e
    return e


@pytest.mark.parametrize("name", ["cycle_o2_t8", "cycle_o1_t12"])  # 16-row tiles / 4-row blocks
def test_fused_cycle_bitwise_equals_two_calls(gpu, golden, name):
    from ccmpc import cycle
    g = golden(name)
    T = int(g["T"])
    store = eng().ParticleStore.from_cells(cells_from_fixture(g), device=gpu)
    cyc = cycle.MinkowskiCycle(store, [int(k) for k in g["K"]], g["ref_traj"])
    cyc.run_unfused()
    a = (cyc.mean.clone(), cyc.cov.clone(), cyc.rec.clone(), cyc.prob_lower.clone())
    for _ in range(3):                     # counters must come back to zero every launch
        cyc.rec.zero_()
        cyc.run()
    assert torch.equal(a[0], cyc.mean) and torch.equal(a[1], cyc.cov)
    assert torch.equal(a[2], cyc.rec) and torch.equal(a[3], cyc.prob_lower)
    h = cyc.records().reshape(-1)
    np.testing.assert_array_equal(h["which"], g["rec_which"])
    assert len(h) == T * (T - 1) // 2 * store.n_cells


@pytest.mark.parametrize("T", [16, 20])
def test_fused_tail_both_lower_bound_paths(gpu, T):
    """The fused tail's two lower-bound layouts against the unfused rows launch, bit for bit:
    T = 16 (120 pairs on a 256-thread workgroup: one lower-bound wave, two pairs on most lanes,
    the per-t minimum from that wave's own LDS writes, no workgroup barrier) and T = 20 (190
    pairs on 512 threads: every thread takes whole pairs, then the barrier and the minimum)."""
    from ccmpc import cycle, synthetic
    ovs, ref, _ = synthetic.scene(5, O=3, N=4000, T=T)
    store = eng().ParticleStore.from_cells([c for o in ovs for c in o], device=gpu)
    cyc = cycle.MinkowskiCycle(store, [len(o) for o in ovs], ref)
    cyc.run_unfused()
    a = (cyc.mean.clone(), cyc.cov.clone(), cyc.rec.clone(), cyc.prob_lower.clone())
    cyc.rec.zero_()
    cyc.prob_lower.zero_()
    cyc.run()
    assert torch.equal(a[0], cyc.mean) and torch.equal(a[1], cyc.cov)
    assert torch.equal(a[2], cyc.rec) and torch.equal(a[3], cyc.prob_lower)
    assert np.all(cyc.records()["status"] == 0)
    pl = cyc.prob_lower.cpu().numpy()
    assert np.all(pl[:, 0] == 1.0) and np.all((pl >= 0.0) & (pl <= 1.0))


def test_graph_replay_is_stable(gpu):
    from ccmpc import cycle, synthetic
    ovs, ref, _ = synthetic.scene(3, O=4, N=5000, T=8)
    store = eng().ParticleStore.from_cells([c for o in ovs for c in o], device=gpu)
    cyc = cycle.MinkowskiCycle(store, [len(o) for o in ovs], ref)
    cyc.run()
    first = cyc.rec.clone()
    cyc.capture()
    for _ in range(200):
        cyc.replay()
    torch.cuda.synchronize()
    assert torch.equal(first, cyc.rec)
    assert np.all(cyc.records()["status"] == 0)


def test_bound_launch_equals_run(gpu):
    """The pre-bound one-call path bench.py times is the same launch as the engine path."""
    from ccmpc import cycle, synthetic
    ovs, ref, _ = synthetic.scene(4, O=4, N=5000, T=8)
    store = eng().ParticleStore.from_cells([c for o in ovs for c in o], device=gpu)
    a = cycle.MinkowskiCycle(store, [len(o) for o in ovs], ref)
    a.run()
    b = cycle.MinkowskiCycle(store, [len(o) for o in ovs], ref).bind()
    for _ in range(100):
        b.launch()
    torch.cuda.synchronize()
    assert torch.equal(a.rec, b.rec) and torch.equal(a.cov, b.cov)
    assert torch.equal(a.prob_lower, b.prob_lower)


def test_workspace_reused_across_shapes(gpu):
    """One zero-initialised workspace serves calls of different cell counts back to back."""
    e = eng()
    ws = e.Workspace(gpu)
    rng = np.random.default_rng(8)
    for counts in ([5000, 3], [17], [100, 200, 300, 400], [70000]):
        cells = [100 + np.cumsum(rng.normal(size=(n, 8, 2)), axis=1) for n in counts]
        store = e.ParticleStore.from_cells(cells, device=gpu)
        m, c = e.moments(store, workspace=ws)
        for j, cl in enumerate(cells):
            X = cl.transpose(1, 2, 0).reshape(16, -1)
            np.testing.assert_allclose(c[j].cpu().numpy(), np.cov(X), rtol=1e-9, atol=1e-12)


def test_workspace_shared_by_calls_of_different_shapes(gpu):
    """Regression: a moments call on a small store and a 1e6-sample fused rollout (two tree
    levels) alternating on ONE workspace, as the planner's shrinking steps do.  The counter
    region depends on the buffer size only, so neither call's slabs land on the other's
    counters; results equal fresh-workspace calls bit for bit."""
    from ccmpc import risk
    e = eng()
    rng = np.random.default_rng(12)
    cells = [190 + np.cumsum(rng.normal(0, 0.4, size=(n, 8, 2)), axis=1) for n in (900, 1500)]
    store = e.ParticleStore.from_cells(cells, device=gpu)
    src = torch.tensor([0, 1], dtype=torch.int32, device=gpu)
    cr = torch.as_tensor(risk.cell_risk(risk.eps_ura([2]), [2], 8), device=gpu)
    shared = e.Workspace(gpu)
    m, c = e.moments(store, workspace=shared)
    for Tn in (7, 6, 5):
        ref = torch.as_tensor((np.array([170.0, 5.0]) + np.arange(1, Tn + 1)[:, None] * [4.0, 0.5])
                              [None], device=gpu)
        e.moments(store, workspace=shared)                        # small call in between
        got = e.ideal_minkowski_cycle(m, c, src, Tn, 1_000_000, ref, cr, seed=Tn,
                                      workspace=shared)
        want = e.ideal_minkowski_cycle(m, c, src, Tn, 1_000_000, ref, cr, seed=Tn,
                                       workspace=e.Workspace(gpu))
        for a, b in zip(got, want):
            assert torch.equal(a, b)
        assert np.all(e.halfspaces(got[3])["status"] == 0)
        m, c = got[0], got[1]


def test_empty_and_singleton_cells_give_nan_like_numpy(gpu):
    e = eng()
    store = e.ParticleStore(4, [0, 1, 6], device=gpu)
    store.pos.normal_()
    m, c = e.moments(store)
    assert torch.isnan(c[0]).all() and torch.isnan(m[0]).all()   # np.cov of nothing
    assert not torch.isfinite(c[1]).any()                         # ddof=1 with one sample
    assert torch.isfinite(c[2]).all()


@pytest.mark.parametrize("T_src", [8, 9, 17, 40])   # T = 7 / 8 | 16 | 39: the row-block edges
def test_ideal_cycle_equals_ideal_moments_plus_minkowski(gpu, T_src):
    """The fused cycle's half-space tables are sized per row-block instance (T <= 8 RB,
    CCMPC_IDEAL_LDS_SHRINK): the cycle equals ideal_moments + minkowski bit for bit at each
    instance's largest T."""
    from ccmpc import risk
    e = eng()
    rng = np.random.default_rng(4)
    cells = [190 + np.cumsum(rng.normal(0, 0.4, size=(n, T_src, 2)), axis=1) for n in (900, 1500)]
    store = e.ParticleStore.from_cells(cells, device=gpu)
    mean, cov = e.moments(store)
    Tn, ns = T_src - 1, 50_000
    src = torch.tensor([0, 1], dtype=torch.int32, device=gpu)
    K = [2]
    cr = torch.as_tensor(risk.cell_risk(risk.eps_ura(K), K, T_src), device=gpu)
    ref = torch.as_tensor((np.array([170.0, 5.0]) + np.arange(1, Tn + 1)[:, None] * [4.0, 0.5])
                          [None], device=gpu)
    m1, c1, st1 = e.ideal_moments(mean, cov, src, Tn, ns, seed=5)
    r1, pl1 = e.minkowski(m1, c1, ref, cr)
    m2, c2, st2, r2, pl2 = e.ideal_minkowski_cycle(mean, cov, src, Tn, ns, ref, cr, seed=5)
    assert torch.equal(m1, m2) and torch.equal(c1, c2)
    assert torch.equal(r1, r2) and torch.equal(pl1, pl2)
    assert st2.cpu().tolist() == [0, 0]


@pytest.mark.parametrize("name", ["cycle_o2_t8", "cycle_o1_t12"])
def test_l4_matches_reference_golden(gpu, golden, name):
    e = eng()
    g = golden(name)
    T = int(g["T"])
    K = [int(k) for k in g["K"]]
    store = e.ParticleStore.from_cells(cells_from_fixture(g), device=gpu)
    past = np.concatenate([[g["past"][o]] * K[o] for o in range(len(K))])
    bbox = np.tile([4.5, 2.5], (store.n_cells, 1))
    out = e.l4(store, past, bbox, with_yaw=True, with_vertices=True)
    np.testing.assert_allclose(out["A"].cpu().numpy(), g["A_union"], rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(out["b"].cpu().numpy(), g["b_union"], rtol=1e-12)
    # yaw statistics of ovStateMean/Cov_tau_1 (v8ideal/__init__.py:872, :875)
    np.testing.assert_allclose(out["yaw_mean"].cpu().numpy()[:, 0], g["state_mean"][:, 2],
                               rtol=1e-12)
    np.testing.assert_allclose(out["yaw0_var"].cpu().numpy(), g["state_cov"][:, 2], rtol=1e-9)
    # per-particle yaws and vertices against the oracle restatement
    ovs = ovehicles_from_fixture(g)
    yaw = out["yaw"].cpu().numpy()
    vert = out["vertices"].cpu().numpy()
    j = 0
    for ov in ovs:
        for k in range(ov.n_states):
            o, n = store.offsets[j], store.counts[j]
            np.testing.assert_allclose(yaw[:, o:o + n].T, ov.pred_yaws[k], rtol=1e-13, atol=1e-14)
            t = T - 1
            want = orc.vertices_of_bboxes(ov.pred_positions[k][:, t], ov.pred_yaws[k][:, t],
                                          ov.bbox)
            got = vert[8 * t:8 * t + 8, o:o + n].T.reshape(n, 4, 2)
            np.testing.assert_allclose(got, want, rtol=1e-13)
            j += 1


def _sampler_inputs(O=3, L=25, T=8, seed=0):
    rng = np.random.default_rng(seed)
    init = np.stack([rng.uniform(20, 60, O), rng.uniform(20, 60, O),
                     rng.uniform(-np.pi, np.pi, O), rng.uniform(3, 10, O)], axis=1)
    pmf = np.stack([np.exp(rng.normal(0, 2.0, L)) for _ in range(O)])
    pmf /= pmf.sum(1, keepdims=True)
    gmm = np.zeros((O, L, T, 5), np.float32)
    gmm[..., 0] = rng.normal(0, 0.15, size=(O, L, 1))
    gmm[..., 1] = rng.normal(0, 1.0, size=(O, L, 1))
    gmm[..., 2] = rng.uniform(np.log(0.05), np.log(0.5), size=(O, L, T))
    gmm[..., 3] = rng.uniform(np.log(0.05), np.log(0.5), size=(O, L, T))
    gmm[..., 4] = rng.uniform(-0.5, 0.5, size=(O, L, T))
    gmm[:, 0, :, 0] = 0.0                      # one mode drives straight (|dphi| small branch)
    gmm[:, 0, :, 2] = np.log(1e-4)
    return init, pmf, gmm


def test_sampler_matches_restatement(gpu):
    """PARITY UNPINNED upstream (Trajectron++ absent): GPU sampler vs the repo's float32
    restatement of DiscreteLatent.sample_p + GMM2D.rsample + Unicycle.integrate_samples."""
    e = eng()
    O, L, T, N, seed = 3, 25, 8, 20_000, 99
    init, pmf, gmm = _sampler_inputs(O, L, T)
    z, store = e.sample_unicycle(init, pmf, gmm, N, T, dt=0.5, seed=seed, device=gpu)
    zc = z.cpu().numpy()
    for o in range(O):
        cdf = np.cumsum(pmf[o])
        zo, pos = orc.sample_unicycle(init[o], cdf, gmm[o], N, T, 0.5, seed, ov=o)
        np.testing.assert_array_equal(zc[o], zo)
        got = store.cell_positions(o)
        # float32 IEEE ops + float64-rounded transcendentals on both sides: bit-for-bit
        mism = np.mean(got != pos)
        assert mism < 1e-4, mism
        np.testing.assert_allclose(got, pos, rtol=0, atol=1e-3)
    # sharded launch: OVs 1..2 alone with ov_base=1 draw exactly what the batched call drew
    z2, store2 = e.sample_unicycle(init[1:], pmf[1:], gmm[1:], N, T, dt=0.5, seed=seed,
                                   device=gpu, ov_base=1)
    np.testing.assert_array_equal(z2.cpu().numpy(), zc[1:])
    for o in range(2):
        np.testing.assert_array_equal(store2.cell_positions(o), store.cell_positions(o + 1))
    # empirical latent frequencies follow p(z|x)
    freq = np.bincount(zc[0], minlength=L) / N
    assert np.max(np.abs(freq - pmf[0])) < 5 * np.sqrt(pmf[0].max() / N) + 1e-3


def _torch_draws(pmf, N, T, seed):
    """z and eps as the upstream boundary draws them in torch (latent.sample_p -> one-hot ->
    argmax, prediction.py:81-83/:103; randn inside GMM2D.rsample)."""
    g = torch.Generator().manual_seed(seed)
    O = pmf.shape[0]
    z = torch.multinomial(torch.as_tensor(pmf), N, replacement=True, generator=g).to(torch.int32)
    eps = torch.randn((O, N, T, 2), generator=g, dtype=torch.float32)
    return z.numpy(), eps.numpy()


def _assert_cloud(got, want):
    # float32 IEEE ops + float64-rounded transcendentals on both sides
    assert np.mean(got != want) < 1e-4
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-3)


def test_sampler_injected_latents_and_noise(gpu):
    """Upstream-shaped boundary, per-latent parameters: torch-drawn z and eps injected
    (ccmpc_sample_unicycle_ex).  PARITY UNPINNED upstream (Trajectron++ absent): vs the
    restatement fed the same draws."""
    e = eng()
    O, L, T, N = 3, 25, 8, 6000
    init, pmf, gmm = _sampler_inputs(O, L, T, seed=4)
    z, eps = _torch_draws(pmf, N, T, seed=11)
    zg, store = e.sample_unicycle(init, pmf, gmm, N, T, dt=0.5, device=gpu, z=z, eps=eps)
    np.testing.assert_array_equal(zg.cpu().numpy(), z)
    for o in range(O):
        _, want = orc.sample_unicycle(init[o], None, gmm[o], N, T, 0.5, 0, ov=o, z=z[o],
                                      eps=eps[o])
        _assert_cloud(store.cell_positions(o), want)
    # z injected, eps from Philox: the same eps stream as the synthetic mode
    zg2, store2 = e.sample_unicycle(init, None, gmm, N, T, dt=0.5, seed=5, device=gpu, z=z)
    for o in range(O):
        _, want = orc.sample_unicycle(init[o], None, gmm[o], N, T, 0.5, 5, ov=o, z=z[o])
        _assert_cloud(store2.cell_positions(o), want)


def test_sampler_per_particle_parameters(gpu):
    """p_y_xz's decoder is autoregressive: every sample has its own GMM parameters per step
    (O, N, T, 5).  GPU vs restatement on the same draws; and the per-particle path fed the
    per-latent table gathered by z reproduces the per-latent path bit for bit."""
    e = eng()
    O, L, T, N = 2, 6, 12, 5000
    init, pmf, gmm = _sampler_inputs(O, L, T, seed=8)
    z, eps = _torch_draws(pmf, N, T, seed=3)
    rng = np.random.default_rng(1)
    pp = np.stack([gmm[o][z[o]] for o in range(O)])                     # (O, N, T, 5)
    jitter = pp.copy()
    jitter[..., 0] += rng.normal(0, 0.05, jitter[..., 0].shape).astype(np.float32)
    jitter[..., 4] = np.clip(jitter[..., 4] + rng.normal(0, 0.3, jitter[..., 4].shape),
                             -1, 1).astype(np.float32)                   # |rho| = 1: the clamp
    _, s_pp = e.sample_unicycle(init, None, jitter, N, T, device=gpu, z=z, eps=eps,
                                per_particle=True)
    for o in range(O):
        _, want = orc.sample_unicycle(init[o], None, jitter[o], N, T, 0.5, 0, ov=o, z=z[o],
                                      eps=eps[o], per_particle=True)
        got = s_pp.cell_positions(o)
        assert np.all(np.isfinite(got))
        _assert_cloud(got, want)
    _, s_gather = e.sample_unicycle(init, None, pp, N, T, device=gpu, z=z, eps=eps,
                                    per_particle=True)
    _, s_lat = e.sample_unicycle(init, pmf, gmm, N, T, device=gpu, z=z, eps=eps)
    for o in range(O):
        np.testing.assert_array_equal(s_gather.cell_positions(o), s_lat.cell_positions(o))
    # device tensors are accepted as they come out of torch
    _, s_dev = e.sample_unicycle(init, None, torch.as_tensor(jitter, device=gpu), N, T,
                                 device=gpu, z=torch.as_tensor(z, device=gpu),
                                 eps=torch.as_tensor(eps, device=gpu), per_particle=True)
    np.testing.assert_array_equal(s_dev.cell_positions(1), s_pp.cell_positions(1))


def test_sampler_rejects_bad_injections(gpu):
    e = eng()
    O, L, T, N = 1, 4, 3, 100
    init, pmf, gmm = _sampler_inputs(O, L, T)
    z = np.zeros((O, N), np.int32)
    z[0, 7] = L
    with pytest.raises(ValueError):
        e.sample_unicycle(init, pmf, gmm, N, T, device=gpu, z=z)
    with pytest.raises(ValueError):
        e.sample_unicycle(init, pmf, np.zeros((O, N, T, 5), np.float32), N, T, device=gpu,
                          per_particle=True)
    lib = e._lib.load()
    rc = lib.ccmpc_sample_unicycle_ex(None, None, L, None, 1, None, None, 1, N, T, 0.5, 0, None,
                                      0, None, None, N, None)
    assert rc == -1                     # CCMPC_ERR_INVALID: per-particle parameters need z_in


@pytest.mark.parametrize("dtype,T,N", [(torch.float64, 8, 3000), (torch.float32, 12, 40000)])
def test_l4_split_equals_one_workgroup_form(gpu, dtype, T, N):
    """ccmpc_l4_split (each (cell, t) over several workgroups, chunk-ordered sums) against
    ccmpc_l4 (one workgroup per (cell, t)): same headings, same corners; the mean heading's sum
    order differs, so A / b / yaw statistics agree to rounding; repeated calls are bitwise
    stable (deterministic chunk order, counters back to zero)."""
    from ccmpc import engine, synthetic
    ovs, _, pasts = synthetic.scene(91, O=3, N=N, T=T)
    cells = [c for o in ovs for c in o]
    origin = np.array([c[:, 0].mean(0) for c in cells]) if dtype == torch.float32 else None
    store = engine.ParticleStore.from_cells(cells, device=gpu, dtype=dtype, origin=origin)
    past = np.repeat(pasts, [len(o) for o in ovs], axis=0)
    bbox = np.tile([4.5, 2.5], (store.n_cells, 1))
    one = engine.l4(store, past, bbox, with_yaw=True, with_vertices=True, split=False)
    ws = engine.Workspace(gpu)
    a = engine.l4(store, past, bbox, with_yaw=True, with_vertices=True, split=True, workspace=ws)
    b = engine.l4(store, past, bbox, with_yaw=True, with_vertices=True, split=True, workspace=ws)
    cols = torch.as_tensor(np.concatenate([np.arange(o, o + n) for o, n in
                                           zip(store.offsets, store.counts)]), device=gpu)
    for x in (one, a, b):       # the per-particle outputs, at the particles' slots only
        x["yaw"], x["vertices"] = x["yaw"][:, cols], x["vertices"][:, cols]
    for k in ("A", "b", "yaw_mean", "yaw0_var", "yaw", "vertices"):
        assert torch.equal(a[k], b[k]), k
    torch.testing.assert_close(a["yaw"], one["yaw"], rtol=0, atol=0)
    torch.testing.assert_close(a["yaw_mean"], one["yaw_mean"], rtol=1e-12, atol=1e-13)
    torch.testing.assert_close(a["yaw0_var"], one["yaw0_var"], rtol=1e-10, atol=1e-14)
    torch.testing.assert_close(a["A"], one["A"], rtol=1e-12, atol=1e-13)
    torch.testing.assert_close(a["b"], one["b"], rtol=1e-12, atol=1e-10)
    torch.testing.assert_close(a["vertices"], one["vertices"], rtol=1e-13, atol=1e-12)
