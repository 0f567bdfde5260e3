"""One episode's planning schedule through the drop-in surface, against the
oracle chained the same way: frame 0 on sampler particles, frames 10..70 on predict_ideal
rollouts of the previous frame's moments (same Philox draws), then receding affine steps."""
import numpy as np
import pytest

from oracle import ccmpc_oracle as orc

pytestmark = pytest.mark.gpu


def _oracle_ovs(ovs, T):
    out = []
    for ov in ovs:
        cells = [np.asarray(p, float) for p in ov.pred_positions]
        past = np.asarray(ov.past, float).reshape(-1, 2)
        out.append(orc.OVehicle(T, past, np.asarray(ov.latent_pmf), cells,
                                [orc._step_yaws(c, past[-1], T) for c in cells],
                                np.zeros((len(cells), 2)), np.array([4.5, 2.5])))
    return out


def test_episode_schedule_matches_oracle_chain(gpu):
    from ccmpc import episode
    n_ideal, seed = 20_000, 3
    rep = episode.EpisodeReplay(O=2, N=3000, ph=8, n_ideal=n_ideal, receding_steps=2,
                                seed=seed, device=gpu)
    mom = None
    for frame, T, kind in rep.schedule():
        ovs, out = rep.step(frame, T, kind)
        K = [ov.n_states for ov in ovs]
        cons = out[0]
        if kind == "affine":
            assert len(cons) == sum(K) * T
            assert all(c.side in (-1, 1) for c in cons)
            continue
        oracle_ovs = _oracle_ovs(ovs, rep.ph)
        ref = rep.ref_traj(frame)
        if T == rep.ph:
            want = orc.minkowski_generator(oracle_ovs, T, rep.ph, ref, with_l4=False)
            mom = orc.save_moments([ov.pred_positions for ov in oracle_ovs], T)
        else:
            ideal = orc.predict_ideal(mom, K, T, n_ideal, seed=seed * 1_000_003 + frame)
            want = orc.minkowski_generator(oracle_ovs, T, rep.ph, ref, ideal_trajs=ideal,
                                           with_l4=False)
            mom = orc.save_moments([[ideal[o][k] for k in range(K[o])]
                                    for o in range(len(K))], T)
        recs = want["records"]
        assert len(cons) == len(recs) == sum(K) * T * (T - 1) // 2, (frame, T)
        for c, r in zip(cons, recs):
            assert (c.ov, c.k, c.t, c.tau) == (r["ov"], r["k"], r["t"], r["tau"])
            assert c.which == r["which"] and c.side == r["side"], (frame, T, c)
            assert c.d == pytest.approx(r["d"], rel=1e-8)


def test_episode_at_reference_scale(gpu):
    """C1 at the reference's own scale: one OV, n_predictions = 100 000 particles per frame
    (tests/Hz20/params.py:372-383, the "np5000" label) and 1e6-sample predict_ideal rollouts
    (v8ideal/__init__.py:2640) on every shrinking step.  Frames 0 and 10 are chained against
    the oracle (frame 0 on the sampler's particles; frame 10 on the oracle's own 1e6-sample
    rollout of frame 0's moments with the same Philox draws); the rest of the schedule (T = 6..1,
    then two receding affine steps) is checked by properties: every record OK, the reference's
    record counts, each record's centre equal to the saved moments' mean at its t, and the
    lower bounds probabilities."""
    from ccmpc import episode
    n_ideal, seed = 1_000_000, 11
    rep = episode.EpisodeReplay(O=1, N=100_000, ph=8, n_ideal=n_ideal, receding_steps=2,
                                seed=seed, device=gpu)
    mom = None
    for frame, T, kind in rep.schedule():
        ovs, out = rep.step(frame, T, kind)
        K = [ov.n_states for ov in ovs]
        assert sum(sum(p.shape[0] for p in ov.pred_positions) for ov in ovs) == 100_000
        cons = out[0]
        if kind == "affine":
            assert len(cons) == sum(K) * T and all(c.side in (-1, 1) for c in cons)
            continue
        P = T * (T - 1) // 2
        assert len(cons) == sum(K) * P, (frame, T)
        h = rep.agent.last_records.reshape(sum(K), -1)[:, :P]
        assert np.all(h["status"] == 0)
        mean = rep.agent._moments[frame][0]
        mean = mean.cpu().numpy() if hasattr(mean, "cpu") else np.asarray(mean)
        for c in range(sum(K)):
            t_of = h[c]["t_tau"] >> 16
            np.testing.assert_array_equal(h[c]["mean0"], mean[c, t_of, 0])
            np.testing.assert_array_equal(h[c]["mean1"], mean[c, t_of, 1])
            assert np.all((h[c]["lower_bound"] >= 0) & (h[c]["lower_bound"] <= 1))
        if frame > 10:
            continue
        ref = rep.ref_traj(frame)
        oracle_ovs = _oracle_ovs(ovs, rep.ph)
        if T == rep.ph:
            want = orc.minkowski_generator(oracle_ovs, T, rep.ph, ref, with_l4=False)
            mom = orc.save_moments([ov.pred_positions for ov in oracle_ovs], T)
        else:
            ideal = orc.predict_ideal(mom, K, T, n_ideal, seed=seed * 1_000_003 + frame)
            want = orc.minkowski_generator(oracle_ovs, T, rep.ph, ref, ideal_trajs=ideal,
                                           with_l4=False)
            del ideal
        recs = want["records"]
        assert len(recs) == len(cons)
        for c, r in zip(cons, recs):
            assert (c.ov, c.k, c.t, c.tau) == (r["ov"], r["k"], r["t"], r["tau"])
            assert c.which == r["which"] and c.side == r["side"], (frame, T, c)
            assert c.d == pytest.approx(r["d"], rel=1e-8)


def test_compute_prediction_controls_drives_the_schedule(gpu):
    """MidlevelAgent.compute_prediction_controls -- the CARLA-free __compute_prediction_controls
    (v8ideal/__init__.py:3163-3210): sampler -> make_ovehicles -> the generator the schedule
    selects -> QP -> U_prev -- driven frame by frame like the reference harness loop, equal to
    EpisodeReplay's separate calls (eager generator + solve_planning_qp) step for step."""
    from ccmpc import episode, planner
    seed = 3
    rep = episode.EpisodeReplay(O=2, N=3000, ph=8, n_ideal=20_000, receding_steps=2, seed=seed,
                                device=gpu)
    agent = planner.MidlevelAgent(prediction_horizon=8, n_ideal=20_000, seed=seed, device=gpu)
    n_cmp = 0
    for frame, T, kind in rep.schedule():
        ovs, out = rep.step(frame, T, kind)
        want = rep.plan(frame, T)
        sampler = dict(init_state=rep.init, latent_pmf=rep.pmf, gmm=rep.gmm, N=rep.N,
                       seed=rep.seed * 7919 + frame)
        ref = rep.ref_traj(frame)
        try:
            speeds, angles, timeout = agent.compute_prediction_controls(
                frame, T, kind == "minkowski", sampler, rep.minpos, rep.pasts,
                rep.x_init(frame), ref[-1] + [4.0, 0.5], ref)
        except planner.InSimulationException:
            assert want is None, (frame, T)
            break                                   # the reference's episode ends here
        assert want is not None and timeout is False
        np.testing.assert_array_equal(speeds, want["X_star"][:, 3])
        np.testing.assert_array_equal(angles, -want["X_star"][:, 2])
        g_cons, e_cons = agent.last_generator_output[1][0], out[0]
        assert len(g_cons) == len(e_cons)
        assert all(a.rhs == b.rhs and a.side == b.side for a, b in zip(g_cons, e_cons))
        n_cmp += 1
    assert n_cmp >= 3


def test_planning_frame_qp_inside_the_graph_and_the_pool(gpu):
    """compute_prediction_controls captures the frame's QP inside the step graph (after the
    record path, before L4) reading the agent's LTV buffers: a destroyed agent's graphs and LTV
    buffers go to the pool together, and the next agent replays those graphs -- same answers
    as the first agent and as the eager QP on the same records."""
    from ccmpc import episode, planner
    seed = 5
    rep = episode.EpisodeReplay(O=2, N=3000, ph=8, n_ideal=20_000, receding_steps=1, seed=seed,
                                device=gpu)
    sched = [s for s in rep.schedule() if s[2] != "ideal"][:3]

    def run(agent):
        out = []
        for frame, T, kind in sched:
            sampler = dict(init_state=rep.init, latent_pmf=rep.pmf, gmm=rep.gmm, N=rep.N,
                           seed=rep.seed * 7919 + frame)
            ref = rep.ref_traj(frame)
            goal = ref[-1] + [4.0, 0.5]
            agent.compute_prediction_controls(frame, T, kind == "minkowski", sampler,
                                              rep.minpos, rep.pasts, rep.x_init(frame), goal, ref)
            u = agent.last_ctrl["u"].copy()
            # the eager QP on the same records and LTV model
            up = np.concatenate(agent._u_prev[:-1]) if T < 8 else None
            again = agent.solve_planning_qp(rep.x_init(frame), goal, ref, T, u_prev=up,
                                            lon=agent.ego_lon)["u"]
            np.testing.assert_array_equal(u, again)
            out.append(u)
        return out

    a = planner.MidlevelAgent(prediction_horizon=8, n_ideal=20_000, seed=seed, device=gpu)
    ua = run(a)
    qp_graphs = {id(g) for k, g in a._graphs.items() if "qp" in k}
    assert qp_graphs and all(a._graphs[k].qp is not None for k in a._graphs if "qp" in k)
    a.destroy()
    b = planner.MidlevelAgent(prediction_horizon=8, n_ideal=20_000, seed=seed, device=gpu)
    ub = run(b)
    assert {id(g) for k, g in b._graphs.items() if "qp" in k} == qp_graphs
    for x, y in zip(ua, ub):
        np.testing.assert_array_equal(x, y)
    b.destroy()


def test_episode_timing_log(gpu):
    from ccmpc import episode
    rep = episode.EpisodeReplay(O=1, N=5000, ph=8, n_ideal=100_000, receding_steps=2,
                                device=gpu)
    log = rep.run()
    assert [s["T"] for s in log] == [8, 7, 6, 5, 4, 3, 2, 1, 8, 8]
    assert all(s["ms"] > 0 for s in log)
    assert log[-1]["generator"] == "affine"
    # the default scene is one the reference could run: every planning step's QP solves
    # (the old lane started the C1 schedule with an infeasible QP)
    assert [s["qp"] for s in log] == ["solved"] * len(log)
    # the default step-graph cache holds the whole schedule: a second episode replays the
    # first one's graphs (an LRU smaller than the schedule would recapture on every step)
    first = {id(g) for g in rep.agent._graphs.values()}
    assert len(first) == 9
    rep.run()
    assert {id(g) for g in rep.agent._graphs.values()} == first


def test_episode_planning_qp_matches_oracle_chain(gpu):
    """The caller's QP at every planning step of the schedule (do_highlevel_control
    :2850-3110): the first step's LTV model, sliced with the executed controls U_prev at
    Tsh < ph (:2858-2891, :3186), on the generator's device records; against the oracle's QP on
    the oracle's records (same particles, same Philox draws)."""
    from ccmpc import episode, mpc
    from oracle import mpc_oracle as mo
    n_ideal, seed = 20_000, 3
    rep = episode.EpisodeReplay(O=2, N=3000, ph=8, n_ideal=n_ideal, receding_steps=2,
                                seed=seed, device=gpu)
    prm = mpc.MPCParams.reference_defaults().as_dict()
    mom, model, n_solved = None, None, 0
    for frame, T, kind in rep.schedule():
        ovs, out = rep.step(frame, T, kind)
        K = [ov.n_states for ov in ovs]
        oracle_ovs = _oracle_ovs(ovs, rep.ph)
        ref = rep.ref_traj(frame)
        if kind == "affine":
            want_rec = orc.affine_generator(oracle_ovs, T, rep.ph, ref, with_l4=False)["records"]
        elif T == rep.ph:
            want_rec = orc.minkowski_generator(oracle_ovs, T, rep.ph, ref, with_l4=False)["records"]
            mom = orc.save_moments([ov.pred_positions for ov in oracle_ovs], T)
        else:
            ideal = orc.predict_ideal(mom, K, T, n_ideal, seed=seed * 1_000_003 + frame)
            want_rec = orc.minkowski_generator(oracle_ovs, T, rep.ph, ref, ideal_trajs=ideal,
                                               with_l4=False)["records"]
            mom = orc.save_moments([[ideal[o][k] for k in range(K[o])]
                                    for o in range(len(K))], T)
        if T == rep.ph:
            xb, _, G, _, _ = mo.VehicleModel(rep.ph, 0.5, 1.85, 3.7).get_optimization_ltv(
                rep.x_init(frame), np.zeros(2))
            model = (xb, G)
        u_prev = np.concatenate(rep.u_prev) if (T < rep.ph and rep.u_prev) else None
        got = rep.plan(frame, T)
        want = mo.solve_step(model[1], model[0], T, rep.ph, ref[-1] + [4.0, 0.5], ref[:T],
                             want_rec, "affine" if kind == "affine" else "halfspace", prm,
                             u_prev=u_prev)
        if not want["feasible"]:
            assert got is None, (frame, T)
            break                       # the reference's episode ends here
        assert got is not None, (frame, T)
        tol = 1e-6 * (1 + np.abs(want["u"]).max())
        assert np.abs(got["u"] - want["u"]).max() <= tol, (frame, T)
        np.testing.assert_allclose(got["X_star"], want["X"], rtol=0,
                                   atol=1e-6 * (1 + np.abs(want["X"]).max()))
        n_solved += 1
    assert n_solved >= 3
