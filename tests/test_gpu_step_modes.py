"""GPU tests of the graph-captured planning step beyond the synthetic C2 shape:

* the per-particle mode at Trajectron++'s own boundary (prediction.py:81-86): every sample's
  GMM parameters, the one-hot z's argmax (:103) and GMM2D.rsample's noise handed over as DEVICE
  tensors -- the graph step must equal the eager drop-in calls on the same tensors;
* the reference's real particle count: `n_predictions = 100_000` at the "np5000" label
  (tests/Hz20/params.py:372-383), where the graph takes its non-fused branch (sampler, then
  ccmpc_bucket) -- equal to the eager calls and to the oracle;
* the host-side guards: a bounded graph cache, stale-frame reads refused, and a kept mode that
  drew no particle failing as the reference fails (ovehicle.py:72).
"""
import numpy as np
import pytest
import torch

from oracle import ccmpc_oracle as orc

pytestmark = pytest.mark.gpu

PH = 8


def _ref(frame):
    ego = np.array([165.0 + 0.2 * frame, -72.0])
    return np.array([ego + [4.0 * (t + 1), 0.5 * (t + 1)] for t in range(PH)])


def _scene_inputs(O, seed=4242):
    from ccmpc import episode
    init, pmf, gmm = episode.synthetic_gmm(O, T=PH, seed=seed)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]])
             for o in range(O)]
    K = [int(np.count_nonzero(pmf[o] > 0.1)) for o in range(O)]
    eps = np.full((O, max(K)), 0.05 / O)
    return init, pmf, gmm, minpos, pasts, K, eps


def _pp_draws(pmf, gmm, N, seed, gpu, with_eps=True):
    """Trajectron-shaped device tensors: z ~ p(z|x) (torch.multinomial, the one-hot sample's
    argmax), per-sample parameters = the latent's row + a per-sample perturbation (an
    autoregressive decoder's outputs differ per sample), standard-normal noise."""
    g = torch.Generator(device=gpu).manual_seed(seed)
    O, L = pmf.shape
    probs = torch.as_tensor(pmf, device=gpu)
    z = torch.multinomial(probs, N, replacement=True, generator=g).to(torch.int32)
    base = torch.as_tensor(gmm, device=gpu)                           # (O, L, T, 5)
    pp = torch.stack([base[o][z[o].long()] for o in range(O)])        # (O, N, T, 5)
    pp = pp + 0.02 * torch.randn(pp.shape, device=gpu, generator=g)
    pp[..., 4].clamp_(-0.9, 0.9)
    eps = torch.randn((O, N, PH, 2), device=gpu, generator=g) if with_eps else None
    return pp.float().contiguous(), z, eps


def _eager(agent, init, pmf, gmm, N, seed, minpos, pasts, params, eps_ura, ref, gpu, z=None,
           eps=None, pp=False):
    from ccmpc import engine, ovehicle
    zz, store = engine.sample_unicycle(init, pmf, gmm, N, PH, seed=seed, device=gpu, z=z,
                                       eps=eps, per_particle=pp)
    ovs = ovehicle.make_ovehicles(store, zz, pmf, minpos, pasts, device=gpu)
    out = agent.compute_obstacle_constraints_GMM_Minkowski_idealprediction(
        params, ovs, None, None, None, eps_ura, None, PH, ref)
    return ovs, out


def _same(out_g, out_e, ovs_g, ovs_e, K, T=PH):
    """Graph step == eager drop-in calls, bit for bit (records, L4, statistics, clouds)."""
    cons_g, cons_e = out_g[0], out_e[0]
    assert len(cons_g) == len(cons_e) == sum(K) * T * (T - 1) // 2
    for a, b in zip(cons_g, cons_e):
        assert (a.ov, a.k, a.t, a.tau, a.side, a.which) == (b.ov, b.k, b.t, b.tau, b.side,
                                                            b.which)
        assert a.d == b.d and np.array_equal(a.n, b.n)
    O = len(K)
    for t in range(PH):
        for o in range(O):
            for k in range(K[o]):
                np.testing.assert_array_equal(out_g[2][t][k][o], out_e[2][t][k][o])
                np.testing.assert_array_equal(out_g[3][t][k][o], out_e[3][t][k][o])
    for i in range(3):
        for o in range(O):
            for k in range(K[o]):
                assert out_g[6][i][o][k] == out_e[6][i][o][k]
                assert out_g[7][i][o][k] == out_e[7][i][o][k]
    for og, oe in zip(ovs_g, ovs_e):
        np.testing.assert_array_equal(og.latent_pmf, oe.latent_pmf)
        np.testing.assert_array_equal(og.init_center, oe.init_center)
        for pg, pe in zip(og.pred_positions, oe.pred_positions):
            np.testing.assert_array_equal(pg, pe)


def _oracle_check(ovs, out, pasts, ref, K, tol=1e-9):
    oovs = [orc.OVehicle(PH, pasts[o], ov.latent_pmf, ov.pred_positions,
                         [orc._step_yaws(c, pasts[o][-1], PH) for c in ov.pred_positions],
                         ov.init_center, ov.bbox) for o, ov in enumerate(ovs)]
    want = orc.minkowski_generator(oovs, PH, PH, ref)
    assert len(out[0]) == len(want["records"])
    for c, r in zip(out[0], want["records"]):
        assert (c.ov, c.k, c.t, c.tau, c.which, c.side) == (r["ov"], r["k"], r["t"], r["tau"],
                                                            r["which"], r["side"])
        assert abs(c.d - r["d"]) <= tol * max(1.0, abs(r["d"]))
    for t in range(PH):
        for o in range(len(K)):
            for k in range(K[o]):
                np.testing.assert_allclose(out[2][t][k][o], want["A_union"][t][k][o],
                                           rtol=1e-12, atol=1e-12)
                np.testing.assert_allclose(out[3][t][k][o], want["b_union"][t][k][o],
                                           rtol=1e-9)


@pytest.mark.parametrize("with_eps", [True, False])
def test_per_particle_graph_step_equals_eager(gpu, with_eps):
    """C2 shape (4 OVs x 5000, fused sampler + bucketing launches) in the per-particle mode:
    two frames through ONE graph, every output equal to the eager calls on the same device
    tensors, and frame 0 against the oracle."""
    from ccmpc import episode, planner
    O, N = 4, 5000
    init, pmf, gmm, minpos, pasts, K, eps_ura = _scene_inputs(O)
    ag = planner.MidlevelAgent(prediction_horizon=PH, device=gpu)
    ae = planner.MidlevelAgent(prediction_horizon=PH, device=gpu)
    for frame, seed in ((0, 21), (10, 22)):
        pp, z, eps = _pp_draws(pmf, gmm, N, seed, gpu, with_eps)
        params = episode.Params(O, K, frame)
        sampler = dict(init_state=init, latent_pmf=pmf, gmm=pp, z=z, eps=eps, N=N, seed=seed,
                       per_particle=True)
        ovs_g, out_g = ag.predict_and_constrain(params, sampler, eps_ura, PH, _ref(frame),
                                                minpos, pasts)
        ovs_e, out_e = _eager(ae, init, pmf, pp, N, seed, minpos, pasts, params, eps_ura,
                              _ref(frame), gpu, z=z, eps=eps, pp=True)
        _same(out_g, out_e, ovs_g, ovs_e, K)
        np.testing.assert_array_equal(ag.last_records.view(np.uint8),
                                      ae.last_records.view(np.uint8))
        if frame == 0:
            _oracle_check(ovs_g, out_g, pasts, _ref(frame), K)
    assert len(ag._graphs) == 1
    g = next(iter(ag._graphs.values()))
    assert g.per_particle and g.fused and g.eps_in == with_eps


def test_per_particle_particle_minor_input_is_used_in_place(gpu):
    """An upstream that writes the graph's own buffers (pp_gmm in the sampler's (O, T, 5, N)
    layout) is not copied, and gives the same step as the (O, N, T, 5) form."""
    from ccmpc import step
    O, N = 2, 3000
    init, pmf, gmm, minpos, pasts, K, eps_ura = _scene_inputs(O, seed=77)
    pp, z, eps = _pp_draws(pmf, gmm, N, 5, gpu)
    outs = []
    for minor in (False, True):
        g = step.MinkowskiStepGraph(O, N, PH, pmf.shape[1], K, device=gpu, per_particle=True,
                                    eps_in=True)
        cr = np.tile([[10.0, 18.4, 2.5]], (sum(K), 1))
        g.set_inputs(1, init, pmf, None, minpos, _ref(0), cr, np.zeros((O, 2)),
                     np.tile([4.5, 2.5], (O, 1)))
        if minor:
            g.pp_gmm.copy_(pp.permute(0, 2, 3, 1))
            ptr = g.pp_gmm.data_ptr()
            g.set_device_inputs(g.pp_gmm, z, eps.permute(0, 2, 3, 1))
            assert g.pp_gmm.data_ptr() == ptr
        else:
            g.set_device_inputs(pp, z, eps)
        g.replay()
        outs.append(g.out.snapshot()["rec"].copy())
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("N", [100_000, 300_000])
def test_reference_particle_count_graph_step(gpu, N):
    """C1's real particle count (100 000 per OV, params.py:377): the graph's one-pass placement
    (ccmpc_sample_bucket: natives straight into their cells, rare particles keyed then copied),
    two frames through one graph equal to the eager calls (sampler -> ccmpc_bucket), and frame 0
    against the oracle (records, L4); above 262 144 particles the graph's sampler ->
    ccmpc_bucket branch."""
    from ccmpc import episode, planner
    O = 1
    init, pmf, gmm, minpos, pasts, K, eps_ura = _scene_inputs(O, seed=20251015)
    ag = planner.MidlevelAgent(prediction_horizon=PH, device=gpu)
    ae = planner.MidlevelAgent(prediction_horizon=PH, device=gpu)
    for frame, seed in ((0, 31), (10, 32)):
        params = episode.Params(O, K, frame)
        sampler = dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=seed)
        ovs_g, out_g = ag.predict_and_constrain(params, sampler, eps_ura, PH, _ref(frame),
                                                minpos, pasts)
        ovs_e, out_e = _eager(ae, init, pmf, gmm, N, seed, minpos, pasts, params, eps_ura,
                              _ref(frame), gpu)
        _same(out_g, out_e, ovs_g, ovs_e, K)
        if frame == 0:
            if N == 100_000:
                _oracle_check(ovs_g, out_g, pasts, _ref(frame), K)
    g = next(iter(ag._graphs.values()))
    assert g.fused == (N <= 262_144)
    assert sum(len(p) for p in ovs_g[0].pred_positions) == N


def test_reference_particle_count_per_particle(gpu):
    """The same count in the per-particle mode (4 OVs x 20 000: the large clouds' placement --
    the actions kernel on device-side z / parameters / noise, then the placement) against the
    eager calls."""
    from ccmpc import episode, planner
    O, N = 4, 20_000
    init, pmf, gmm, minpos, pasts, K, eps_ura = _scene_inputs(O, seed=99)
    pp, z, eps = _pp_draws(pmf, gmm, N, 41, gpu)
    ag = planner.MidlevelAgent(prediction_horizon=PH, device=gpu)
    ae = planner.MidlevelAgent(prediction_horizon=PH, device=gpu)
    params = episode.Params(O, K, 0)
    sampler = dict(init_state=init, latent_pmf=pmf, gmm=pp, z=z, eps=eps, N=N, seed=0,
                   per_particle=True)
    ovs_g, out_g = ag.predict_and_constrain(params, sampler, eps_ura, PH, _ref(0), minpos,
                                            pasts)
    ovs_e, out_e = _eager(ae, init, pmf, pp, N, 0, minpos, pasts, params, eps_ura, _ref(0),
                          gpu, z=z, eps=eps, pp=True)
    _same(out_g, out_e, ovs_g, ovs_e, K)
    assert next(iter(ag._graphs.values())).fused


def test_stale_frame_reads_raise(gpu):
    """Frame 0's OVehicles are views of the graph's store: read before the next same-shape
    step they are frame 0's data; after it, reading them raises instead of returning frame
    1's particles.  The 9-tuple's arrays are host copies and stay frame 0's."""
    from ccmpc import episode, planner
    O, N = 2, 2000
    init, pmf, gmm, minpos, pasts, K, eps_ura = _scene_inputs(O, seed=5)
    agent = planner.MidlevelAgent(prediction_horizon=PH, device=gpu)
    params = episode.Params(O, K, 0)
    s0 = dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=1)
    ovs0, out0 = agent.predict_and_constrain(params, s0, eps_ura, PH, _ref(0), minpos, pasts)
    pos0 = [np.copy(p) for p in ovs0[0].pred_positions]       # read while live: cached copy
    b0 = np.copy(out0[3][3][0][0])
    d0 = out0[0][5].d
    s1 = dict(s0, seed=2)
    ovs1, out1 = agent.predict_and_constrain(episode.Params(O, K, 10), s1, eps_ura, PH,
                                             _ref(10), minpos, pasts)
    assert not np.array_equal(out1[3][3][0][0], b0)
    np.testing.assert_array_equal(out0[3][3][0][0], b0)    # host copies survive the replay
    assert out0[0][5].d == d0
    for p, q in zip(ovs0[0].pred_positions, pos0):          # already read: still frame 0's
        np.testing.assert_array_equal(p, q)
    with pytest.raises(RuntimeError, match="stale"):
        ovs0[1].pred_positions                                # never read: refused
    with pytest.raises(RuntimeError, match="stale"):
        out0[1][2][0][0]                                      # vertices of frame 0
    ovs1[1].pred_positions                                    # the live frame reads fine


def test_graph_cache_is_bounded(gpu):
    """Kept-mode splits that change from frame to frame each need a graph; the cache keeps
    the `max_graphs` most recently used."""
    from ccmpc import episode, planner
    O, N, L = 2, 1000, 25
    init, _, gmm, minpos, pasts, _, _ = _scene_inputs(O, seed=6)
    agent = planner.MidlevelAgent(prediction_horizon=PH, device=gpu, max_graphs=2)
    splits = [(1, 1), (2, 1), (1, 2), (2, 2), (1, 1)]
    for f, Ks in enumerate(splits):
        pmf = np.zeros((O, L))
        for o, k in enumerate(Ks):
            pmf[o, :k] = 0.9 / k
            pmf[o, k:] = 0.1 / (L - k)
        eps_ura = np.full((O, max(Ks)), 0.05 / O)
        s = dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=f)
        ovs, out = agent.predict_and_constrain(episode.Params(O, list(Ks), 10 * f), s, eps_ura,
                                               PH, _ref(0), minpos, pasts)
        assert [ov.n_states for ov in ovs] == list(Ks)
        assert len(agent._graphs) <= 2
    assert list(agent._graphs.values())[-1].K == [1, 1]


def test_kept_mode_without_draws_fails_like_the_reference(gpu):
    """A latent with p(z|x) > 0.1 that no sample drew: the reference's from_trajectron fails
    on the empty prediction array (ovehicle.py:72, IndexError); the oracle restatement fails the
    same way, and so do the eager drop-in calls and the graph step."""
    from ccmpc import engine, episode, ovehicle, planner
    O, N, L = 1, 600, 25
    init, _, gmm, minpos, pasts, _, _ = _scene_inputs(O, seed=8)
    pmf = np.full((O, L), 0.3 / (L - 2))
    pmf[0, 0], pmf[0, 1] = 0.58, 0.12                          # both kept
    z = torch.zeros((O, N), dtype=torch.int32, device=gpu)
    z[0, ::3] = 5                                              # rare latent; latent 1 never
    zs, store = engine.sample_unicycle(init, pmf, gmm, N, PH, seed=3, device=gpu, z=z)
    pred = store.cell_positions(0).astype(np.float32)[None]      # scene-relative (origin 0)
    with pytest.raises(IndexError):
        orc.make_ovehicles(pred, zs.cpu().numpy(), pmf, minpos, pasts,
                           [np.array([4.5, 2.5])], PH)
    with pytest.raises(IndexError):
        ovehicle.make_ovehicles(store, zs, pmf, minpos, pasts, device=gpu)
    agent = planner.MidlevelAgent(prediction_horizon=PH, device=gpu)
    pp = torch.as_tensor(gmm, device=gpu)[0][z[0].long()][None].contiguous()
    s = dict(init_state=init, latent_pmf=pmf, gmm=pp, z=z, eps=None, N=N, seed=3,
             per_particle=True)
    with pytest.raises(IndexError):
        agent.predict_and_constrain(episode.Params(O, [2], 0), s, np.full((1, 2), 0.05), PH,
                                    _ref(0), minpos, pasts)


@pytest.mark.parametrize("as_tensors", [False, True], ids=["host_arrays", "device_tensors"])
def test_predictions_source_at_the_reference_particle_count(gpu, as_tensors):
    """generate_vehicle_latents' 5-tuple at C1's 100 000 particles per OV (with an ego node in
    row 0, as the reference's batch has it): the step graph built with source='predictions'
    (ccmpc_bucket_predictions -> cycle) gives the records, moments and
    per-cell counts of the sampler route's graph on the same particles, frame after frame, and
    of the shrinking (ideal) and receding (affine) kinds."""
    from ccmpc import engine, episode, planner
    O, N = 1, 100_000
    init, pmf, gmm, minpos, pasts, K, eps_ura = _scene_inputs(O, seed=20251015)
    a = planner.MidlevelAgent(prediction_horizon=PH, n_ideal=50_000, device=gpu)
    b = planner.MidlevelAgent(prediction_horizon=PH, n_ideal=50_000, device=gpu)
    for frame, T, kind in ((0, PH, "minkowski"), (10, PH - 1, "minkowski"), (20, PH, "affine"),
                           (30, PH, "minkowski")):
        seed = 700 + frame
        sampler = dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=seed)
        z, store = engine.sample_unicycle(init, pmf, gmm, N, PH, seed=seed, device=gpu)
        pred = store.pos[:, :N].reshape(PH, 2, N).permute(2, 0, 1)[None]      # (1, N, T, 2)
        ego = torch.zeros_like(pred)
        P = torch.cat([ego, pred]).contiguous()
        Z = torch.cat([torch.zeros_like(z), z]).to(torch.int64).contiguous()
        if not as_tensors:
            P, Z = P.cpu().numpy(), Z.cpu().numpy()
        lp = np.concatenate([pmf[:1], pmf])
        psrc = dict(source="predictions", predictions=P, z=Z, rows=[1], latent_pmf=lp[1:],
                    N=N)
        params = episode.Params(O, K, frame)
        fn_a = a.predict_and_constrain_affine if kind == "affine" else a.predict_and_constrain
        fn_b = b.predict_and_constrain_affine if kind == "affine" else b.predict_and_constrain
        _, out_a = fn_a(params, sampler, eps_ura, T, _ref(frame), minpos, pasts)
        rec_a = np.array(a.last_records).tobytes()
        _, out_b = fn_b(params, psrc, eps_ura, T, _ref(frame), minpos, pasts)
        assert np.array(b.last_records).tobytes() == rec_a, (frame, kind)
        np.testing.assert_array_equal(np.asarray(out_a[6][0][0]), np.asarray(out_b[6][0][0]))
    g = [g for k, g in b._graphs.items() if "predictions" in k]
    assert g and all(x.source == "predictions" and x.fused for x in g)   # one placement pass


def test_device_predictions_read_in_place_or_copied(gpu):
    """A pred_device graph reads the predictor's tensors in place when the OVs are one run of
    nodes in the kernels' layout (float32 predictions, int64 z: their addresses travel in the
    input pack, ccmpc_bucket_predictions_indirect), and copies them into its own buffers
    otherwise (rows out of order, int32 z); both give the host-array route's records."""
    import torch
    from ccmpc import engine, episode, planner
    O, N = 2, 3000
    init, pmf, gmm, minpos, pasts, K, eps_ura = _scene_inputs(O, seed=77)
    z, store = engine.sample_unicycle(init, pmf, gmm, N, PH, seed=5, device=gpu)
    pred = torch.zeros((4, N, PH, 2), dtype=torch.float32, device=gpu)
    Z = torch.zeros((4, N), dtype=torch.int64, device=gpu)
    for o, r in enumerate((1, 2)):                  # nodes 1 and 2: a run
        off = store.offsets[o]
        pred[r] = store.pos[:, off:off + N].reshape(PH, 2, N).permute(2, 0, 1)
        Z[r] = z[o].to(torch.int64)
    perm = [3, 0]                                   # the same OVs at nodes 3 and 0: no run
    pred2, Z2 = pred.clone(), Z.clone()
    pred2[3], pred2[0], Z2[3], Z2[0] = pred[1], pred[2], Z[1], Z[2]
    params = episode.Params(O, K, 0)
    recs = []
    for P, ZZ, rows in ((pred.cpu().numpy(), Z.cpu().numpy(), [1, 2]), (pred, Z, [1, 2]),
                        (pred2, Z2.to(torch.int32), perm)):
        ag = planner.MidlevelAgent(prediction_horizon=PH, device=gpu)
        s = dict(source="predictions", predictions=P, z=ZZ, rows=rows, latent_pmf=pmf, N=N)
        for _ in range(3):                          # eager, capture, replay
            ag.predict_and_constrain(params, s, eps_ura, PH, _ref(0), minpos, pasts)
        recs.append(np.array(ag.last_records).tobytes())
        g = next(iter(ag._graphs.values()))
        if torch.is_tensor(P):
            in_place = rows == [1, 2]
            assert (g._held is not None) == in_place
    assert recs[0] == recs[1] == recs[2]
