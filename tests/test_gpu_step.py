"""GPU tests of the graph-captured planning step (ccmpc.step.MinkowskiStepGraph behind
MidlevelAgent.predict_and_constrain): one replay = sampler -> bucketing -> Minkowski cycle -> L4
with packed input/output copies.  It must give exactly what the eager drop-in calls give
(do_prediction + make_ovehicles + the Minkowski generator, v8ideal/__init__.py:414-505,
:781-964), step after step, and its records must meet the oracle."""
import numpy as np
import pytest

from oracle import ccmpc_oracle as orc

pytestmark = pytest.mark.gpu

O, N, PH = 4, 3000, 8


def _inputs():
    from ccmpc import episode
    init, pmf, gmm = episode.synthetic_gmm(O, T=PH, seed=4242)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]])
             for o in range(O)]
    K = [int(np.count_nonzero(pmf[o] > 0.1)) for o in range(O)]
    eps = np.full((O, max(K)), 0.05 / O)
    return init, pmf, gmm, minpos, pasts, K, eps


def _ref(frame):
    ego = np.array([165.0 + 0.2 * frame, -72.0])
    return np.array([ego + [4.0 * (t + 1), 0.5 * (t + 1)] for t in range(PH)])


def _eager(agent, init, pmf, gmm, seed, minpos, pasts, params, eps, T, ref, gpu):
    from ccmpc import engine, ovehicle
    z, store = engine.sample_unicycle(init, pmf, gmm, N, PH, seed=seed, device=gpu)
    ovs = ovehicle.make_ovehicles(store, z, pmf, minpos, pasts, device=gpu)
    out = agent.compute_obstacle_constraints_GMM_Minkowski_idealprediction(
        params, ovs, None, None, None, eps, None, T, ref)
    return ovs, out


def _same(out_g, out_e, ovs_g, ovs_e, K, T):
    cons_g, cons_e = out_g[0], out_e[0]
    assert len(cons_g) == len(cons_e) == sum(K) * T * (T - 1) // 2
    for a, b in zip(cons_g, cons_e):
        assert (a.ov, a.k, a.t, a.tau, a.side, a.which) == (b.ov, b.k, b.t, b.tau, b.side,
                                                            b.which)
        assert a.d == b.d and np.array_equal(a.n, b.n)
    for t in range(PH):
        for o in range(O):
            for k in range(max(K)):
                ag, ae = out_g[2][t][k][o], out_e[2][t][k][o]
                assert (ag is None) == (ae is None)
                if ag is not None:
                    np.testing.assert_array_equal(ag, ae)
                    np.testing.assert_array_equal(out_g[3][t][k][o], out_e[3][t][k][o])
    assert out_g[4] == out_e[4]
    for i in range(3):
        for o in range(O):
            for k in range(K[o]):
                assert out_g[6][i][o][k] == out_e[6][i][o][k]
                assert out_g[7][i][o][k] == out_e[7][i][o][k]
    for og, oe in zip(ovs_g, ovs_e):
        assert og.n_states == oe.n_states
        np.testing.assert_array_equal(og.latent_pmf, oe.latent_pmf)
        np.testing.assert_array_equal(og.init_center, oe.init_center)
        for pg, pe in zip(og.pred_positions, oe.pred_positions):
            np.testing.assert_array_equal(pg, pe)


@pytest.mark.parametrize("packed", [1, 2])
def test_graph_step_equals_eager_drop_in_calls(gpu, packed, monkeypatch):
    """packed = 2: the sampler route's input copy inside the placement's first launch
    (ccmpc_sample_bucket_packed, CCMPC_STEP_PACKED=2) -- the same bits."""
    from ccmpc import episode, planner, step
    monkeypatch.setattr(step, "_STEP_PACKED", packed)
    init, pmf, gmm, minpos, pasts, K, eps = _inputs()
    ag = planner.MidlevelAgent(prediction_horizon=PH, n_ideal=200_000, device=gpu)
    ae = planner.MidlevelAgent(prediction_horizon=PH, n_ideal=200_000, device=gpu)
    # two full-horizon frames through ONE captured graph (fresh Philox draws per replay), then
    # a shrinking frame on the graph step's saved moments
    for frame, seed in ((0, 11), (100, 12), (110, 13)):
        T = PH if frame != 110 else PH - 1
        params = episode.Params(O, K, frame)
        sampler = dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=seed)
        ovs_g, out_g = ag.predict_and_constrain(params, sampler, eps, T, _ref(frame), minpos,
                                                pasts)
        ovs_e, out_e = _eager(ae, init, pmf, gmm, seed, minpos, pasts, params, eps, T,
                              _ref(frame), gpu)
        _same(out_g, out_e, ovs_g, ovs_e, K, T)
        np.testing.assert_array_equal(ag.last_records.view(np.uint8),
                                      ae.last_records.view(np.uint8))
        if T == PH:
            assert ag.prob_lower_save == ae.prob_lower_save
    assert sorted(g.kind for g in ag._graphs.values()) == ["ideal", "minkowski"]


def test_graph_step_records_meet_the_oracle(gpu):
    from ccmpc import episode, planner
    init, pmf, gmm, minpos, pasts, K, eps = _inputs()
    agent = planner.MidlevelAgent(prediction_horizon=PH, device=gpu)
    params = episode.Params(O, K, 0)
    sampler = dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=5)
    ovs, out = agent.predict_and_constrain(params, sampler, eps, PH, _ref(0), minpos, pasts)
    oovs = [orc.OVehicle(PH, pasts[o], ov.latent_pmf, ov.pred_positions,
                         [orc._step_yaws(c, pasts[o][-1], PH) for c in ov.pred_positions],
                         ov.init_center, ov.bbox) for o, ov in enumerate(ovs)]
    want = orc.minkowski_generator(oovs, PH, PH, _ref(0))
    cons = out[0]
    assert len(cons) == len(want["records"])
    for c, r in zip(cons, want["records"]):
        assert (c.ov, c.k, c.t, c.tau, c.which) == (r["ov"], r["k"], r["t"], r["tau"],
                                                    r["which"])
        assert c.side == r["side"]
        assert abs(c.d - r["d"]) <= 1e-9 * max(1.0, abs(r["d"]))
    for t in range(PH):
        for o in range(O):
            for k in range(K[o]):
                np.testing.assert_allclose(out[2][t][k][o], want["A_union"][t][k][o],
                                           rtol=1e-12, atol=1e-12)
                np.testing.assert_allclose(out[3][t][k][o], want["b_union"][t][k][o],
                                           rtol=1e-9)


def test_graph_step_refuses_a_different_mode_split(gpu):
    from ccmpc import step
    init, pmf, gmm, minpos, pasts, K, eps = _inputs()
    g = step.MinkowskiStepGraph(O, N, PH, pmf.shape[1], [k + 1 for k in K], device=gpu)
    with pytest.raises(ValueError):
        g.set_inputs(1, init, pmf, gmm, minpos, _ref(0), np.zeros((sum(K) + O, 3)),
                     np.zeros((sum(K) + O, 2)), np.zeros((sum(K) + O, 2)))


def test_graph_replay_equals_its_first_eager_launch(gpu):
    """A step graph's first launch runs its calls eagerly (StepGraph.capture_at), the second is
    the captured graph: with the same inputs (same frame, seed and saved moments) both give the
    same bytes, for every step kind -- full-horizon Minkowski, shrinking (ideal rollout) and
    receding affine."""
    from ccmpc import episode, planner
    init, pmf, gmm, minpos, pasts, K, eps = _inputs()
    ag = planner.MidlevelAgent(prediction_horizon=PH, n_ideal=200_000, device=gpu)
    for frame, T, affine in ((0, PH, False), (10, PH - 1, False), (20, PH, True)):
        params = episode.Params(O, K, frame)
        sampler = dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=77 + frame)
        fn = ag.predict_and_constrain_affine if affine else ag.predict_and_constrain
        got = []
        for _ in range(2):
            ovs, out = fn(params, sampler, eps, T, _ref(frame), minpos, pasts)
            g = list(ag._graphs.values())[-1]           # this frame's graph (most recent)
            L4 = list(g.l4_outputs(g.generation).values())
            got.append((np.array(ag.last_records).view(np.uint8), L4,
                        [np.array(p) for ov in ovs for p in ov.pred_positions]))
        (r0, l0, p0), (r1, l1, p1) = got
        np.testing.assert_array_equal(r0, r1)
        for a, b in zip(l0 + p0, l1 + p1):
            np.testing.assert_array_equal(a, b)
    assert len(ag._graphs) == 3
    assert all(g.graphs is not None and g.generation == 2 for g in ag._graphs.values())


def test_first_replay_is_not_signalled_by_the_capture_warmup(gpu, monkeypatch):
    """capture() runs the whole step eagerly once (warm-up), signal included, with the
    generation of the launch that captures.  The signal word must be stepped back after it, so
    wait() returns only once the REPLAY has signalled (otherwise the host read the
    output pack while the replay's copy-out rewrote it).  The replay is held back here: the word
    must still be one generation behind; replaying then satisfies the poll."""
    import torch
    from ccmpc import episode, planner, step
    init, pmf, gmm, minpos, pasts, K, eps = _inputs()
    ag = planner.MidlevelAgent(prediction_horizon=PH, device=gpu)
    params = episode.Params(O, K, 0)
    sampler = dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=5)
    ag.predict_and_constrain(params, sampler, eps, PH, _ref(0), minpos, pasts)   # eager
    g = list(ag._graphs.values())[-1]
    assert g.graphs is None and g.generation == 1
    held = []
    monkeypatch.setattr(step.HipGraph, "replay", lambda self, stream=None: held.append(self))
    g.launch()                                            # generation 2: capture, replay held
    torch.cuda.synchronize(gpu)
    assert g.graphs is not None and len(held) == 1
    assert int(g._flags[0]) == 1, int(g._flags[0])        # the warm-up's signal was taken back
    monkeypatch.undo()
    held[0].replay(torch.cuda.current_stream(gpu).cuda_stream)
    g.wait()
    assert int(g._flags[0]) == 2


def test_capture_warmup_signals_neither_the_step_nor_its_attached_qp(gpu, monkeypatch):
    """The same with the planning frame's QP attached (attach_qp): the warm-up also
    runs the QP's copy-out + signal with the QP's current generation, so its word must lag by
    one too until the held replay runs -- else PlanningQPStep.wait() returned on the warm-up's
    signal and read the answer pack while the replay rewrote it."""
    import torch
    from ccmpc import mpc, step
    init, pmf, gmm, minpos, pasts, K, eps = _inputs()
    C = sum(K)
    g = step.StepGraph(O, N, PH, pmf.shape[1], K, device=gpu)
    qs = mpc.PlanningQPStep(C, PH, PH, device=gpu)
    xbar = torch.empty((1, 4 * PH), dtype=torch.float64, device=gpu)
    gamma = torch.empty((1, 4 * PH, 2 * PH), dtype=torch.float64, device=gpu)
    g.attach_qp(qs, xbar, gamma, True)
    past = np.stack([p[-1] for p in pasts])
    risk = np.tile([[5.99, 0.95, 0.5]], (C, 1))
    x0, goal = np.array([165.0, -72.0, 0.0, 6.0]), np.array([200.0, -70.0])

    def frame(f):
        g.set_inputs(10 + f, init, pmf, gmm, minpos, _ref(f), risk, past,
                     np.tile([[4.5, 2.5]], (O, 1)))
        return qs.prepare(x0, goal, _ref(f))
    q1 = frame(1)
    g.launch()                                            # generation 1: eager
    g.wait()
    r1 = qs.wait(q1)
    held = []
    monkeypatch.setattr(step.HipGraph, "replay", lambda self, stream=None: held.append(self))
    q2 = frame(2)
    g.launch()                                            # generation 2: capture, replay held
    torch.cuda.synchronize(gpu)
    assert g.graphs is not None and len(held) == 1
    assert int(g._flags[0]) == 1, int(g._flags[0])
    assert int(qs._flags[0]) == q2 - 1, (int(qs._flags[0]), q2)
    monkeypatch.undo()
    held[0].replay(torch.cuda.current_stream(gpu).cuda_stream)
    g.wait()
    r2 = qs.wait(q2)
    assert int(g._flags[0]) == 2 and int(qs._flags[0]) == q2
    assert r1["status"] >= 0 and r2["status"] >= 0


def test_pack_record_view_is_the_byte_field(gpu):
    """Pack(record_views=...): a snapshot's record field covers the byte field's bytes with the
    record dtype (what predict_and_constrain hands to HalfSpaceList), in the snapshot's own
    copy; a byte field whose last axis is not one record is refused."""
    import torch
    from ccmpc import engine, step
    hd = engine._lib.HALFSPACE_DTYPE
    p = step.Pack([("a", (3,), torch.float64), ("rec", (2, 5, hd.itemsize), torch.uint8)], gpu,
                  record_views={"records": ("rec", hd)})
    p.h("rec")[...] = np.random.default_rng(1).integers(0, 256, p.h("rec").shape, dtype=np.uint8)
    o = p.snapshot()
    assert o["records"].dtype == hd and o["records"].shape == (2, 5)
    np.testing.assert_array_equal(o["records"].view(np.uint8).reshape(2, 5, -1), o["rec"])
    np.testing.assert_array_equal(o["rec"], p.h("rec"))
    assert not np.shares_memory(o["records"], p.h("rec"))
    assert set(o) == {"a", "rec", "records"}
    with pytest.raises(ValueError, match="not one"):
        step.Pack([("rec", (2, 100), torch.uint8)], gpu, record_views={"r": ("rec", hd)})
