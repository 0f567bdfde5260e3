"""The reference harness's episode loop (tests/Hz20/__init__.py:183-359, MonteCarloScenario)
driving the library through MidlevelAgent's reference constructor and run_step(frame,
offline_index, T, shrinking), with CARLA and Trajectron++ replaced by ccmpc.standins.

Checked per planning step:
  * gating: plans exactly at first_frame + record_interval * (n_burn_interval + j), with the
    harness's T schedule 8, 7, ..., 1 (shrinking, Minkowski), then 8 (receding, affine);
  * warm start: each step's x_init is the previous step's X_star[0] (make_local_params
    :526-532), the first one the simulator's flipped state;
  * the same step through the lower-level entry point compute_prediction_controls on a fresh
    agent (EpisodeReplay's path) gives bit-identical records, speeds and angles;
  * the Minkowski steps' records against the oracle chain (frame 0 on the sampler's particles,
    later frames on the oracle's predict_ideal rollout of the previous moments, same Philox
    draws), and the QP against the oracle QP on the oracle's records.
"""
import numpy as np
import torch
import pytest

from oracle import ccmpc_oracle as orc

pytestmark = pytest.mark.gpu

N_IDEAL = 20_000


def _oracle_ovs(ovs, T):
    out = []
    for ov in ovs:
        cells = [np.asarray(p, float) for p in ov.pred_positions]
        past = np.asarray(ov.past, float).reshape(-1, 2)
        out.append(orc.OVehicle(T, past, np.asarray(ov.latent_pmf), cells,
                                [orc._step_yaws(c, past[-1], T) for c in cells],
                                np.zeros((len(cells), 2)), np.asarray(ov.bbox, float)))
    return out


def _scenario(gpu, per_particle, run_interval=10, n_ov=2, N=3000):
    from ccmpc import harness, standins

    def make_world():
        world, ego, ids, mr = standins.town03_scene(n_ov=n_ov, ego_xy=(60.0, 81.76),
                                                    ego_speed=8.0, ov_gap=20.0, ov_speed=8.0,
                                                    ov_lateral=40.0)
        return world, ego, ids, mr

    route = make_world()[3].route_points
    ref_route = route[::2]                         # 4 m spacing: 8 m/s x 0.5 s per step
    stg = standins.SyntheticTrajectron(L=25, ph=8, seed=5, per_particle=per_particle,
                                       device=gpu)
    sp = harness.ScenarioParameters(n_burn_interval=4, run_interval=run_interval)
    cp = harness.CtrlParameters(n_predictions=N, prediction_horizon=8, control_horizon=8)
    return harness.MonteCarloScenario(
        sp, cp, make_world, stg,
        agent_kwargs=dict(n_ideal=N_IDEAL, reference_trajectory=ref_route, device=gpu))


@pytest.mark.parametrize("per_particle", [False, True], ids=["per_latent", "per_particle"])
def test_harness_episode_through_run_step(gpu, per_particle):
    from ccmpc import planner
    scen = _scenario(gpu, per_particle)
    stats = scen.episode(0)
    assert not stats.infeasibility, stats
    steps = scen.steps
    first = scen.agent._first_frame
    # gating (:3244-3254) and the harness's T schedule (:330-359)
    assert [s["frame"] - first for s in steps] == [10 * (4 + j) for j in range(len(steps))]
    want_T = [8, 7, 6, 5, 4, 3, 2, 1] + [8] * (len(steps) - 8)
    assert [s["T"] for s in steps] == want_T[:len(steps)]
    assert len(steps) == 10 and stats.steps == 100
    assert [s["shrinking"] for s in steps] == [True] * 8 + [False] * 2
    # warm start: x_init(j+1) = X_star(j)[0]
    for a, b in zip(steps, steps[1:]):
        np.testing.assert_array_equal(b["x_init"], a["X_star"][0])
    # the same inputs through compute_prediction_controls on a fresh agent
    ref_agent = planner.MidlevelAgent(prediction_horizon=8, n_ideal=N_IDEAL, device=gpu)
    for s in steps:
        sp, an, to = ref_agent.compute_prediction_controls(
            s["frame"], s["T"], s["shrinking"], s["sampler"], s["minpos"], s["pasts"],
            s["x_init"], s["goal"], s["ref"], s["bboxes"])
        assert to is False
        np.testing.assert_array_equal(sp, s["speeds"])
        np.testing.assert_array_equal(an, s["angles"])
        assert ref_agent.last_records.tobytes() == s["records"].tobytes(), s["frame"]


def test_next_episode_takes_the_destroyed_agents_graphs(gpu):
    """The harness builds a fresh agent per episode and destroys the last (tests/Hz20/
    __init__.py:383-399): the next agent takes the released step graphs from the pool (its
    steps replay them, captured) and plans the same episode to the same bytes."""
    from ccmpc import step
    scen = _scenario(gpu, False, run_interval=10, n_ov=1, N=2000)
    step._POOL.clear()
    scen.episode(0)
    first_ids = {id(g) for lst in step._POOL.values() for g in lst}
    first = [(s["records"].tobytes(), s["speeds"].tobytes(), s["angles"].tobytes())
             for s in scen.steps]
    assert len(first_ids) >= 9          # T = 8 .. 1 and the receding affine shape at least
    scen.episode(0)                     # same seeds: the same episode again
    again = [(s["records"].tobytes(), s["speeds"].tobytes(), s["angles"].tobytes())
             for s in scen.steps]
    assert again == first
    assert {id(g) for lst in step._POOL.values() for g in lst} == first_ids
    assert all(g.graphs is not None for lst in step._POOL.values() for g in lst
               if g.generation >= 2)


def test_harness_steps_match_oracle_chain(gpu):
    """Minkowski records of the harness's shrinking steps against the oracle chain, and the
    planning QP against the oracle QP on the oracle's records."""
    from ccmpc import mpc, planner
    from oracle import mpc_oracle as mo
    scen = _scenario(gpu, per_particle=False, run_interval=6)
    stats = scen.episode(0)
    assert not stats.infeasibility
    agent = planner.MidlevelAgent(prediction_horizon=8, n_ideal=N_IDEAL, device=gpu)
    prm = mpc.MPCParams.reference_defaults().as_dict()
    mom, model, n_qp = None, None, 0
    u_prev = []
    for s in scen.steps:
        T, frame = s["T"], s["frame"]
        agent.compute_prediction_controls(frame, T, s["shrinking"], s["sampler"], s["minpos"],
                                          s["pasts"], s["x_init"], s["goal"], s["ref"],
                                          s["bboxes"])
        ovs, out = agent.last_generator_output
        K = [ov.n_states for ov in ovs]
        oracle_ovs = _oracle_ovs(ovs, 8)
        ref = s["ref"]
        if T == 8:
            want = orc.minkowski_generator(oracle_ovs, T, 8, ref, with_l4=False)
            mom = orc.save_moments([ov.pred_positions for ov in oracle_ovs], T)
        else:
            ideal = orc.predict_ideal(mom, K, T, N_IDEAL, seed=frame)
            want = orc.minkowski_generator(oracle_ovs, T, 8, ref, ideal_trajs=ideal,
                                           with_l4=False)
            mom = orc.save_moments([[ideal[o][k] for k in range(K[o])]
                                    for o in range(len(K))], T)
        recs = want["records"]
        cons = out[0]
        assert len(cons) == len(recs) == sum(K) * T * (T - 1) // 2
        for c, r in zip(cons, recs):
            assert (c.ov, c.k, c.t, c.tau) == (r["ov"], r["k"], r["t"], r["tau"])
            assert c.which == r["which"] and c.side == r["side"], (frame, T, c)
            assert c.d == pytest.approx(r["d"], rel=1e-8)
        if T == 8:
            xb, _, G, _, _ = mo.VehicleModel(8, 0.5, 1.85, 3.7).get_optimization_ltv(
                s["x_init"], np.zeros(2))
            model, u_prev = (xb, G), []
        up = np.concatenate(u_prev) if (T < 8 and u_prev) else None
        w = mo.solve_step(model[1], model[0], T, 8, s["goal"], ref[:T], recs, "halfspace",
                          prm, u_prev=up)
        assert w["feasible"], (frame, T)
        tol = 1e-6 * (1 + np.abs(w["u"]).max())
        assert np.abs(s["u"] - w["u"]).max() <= tol, (frame, T)
        u_prev.append(s["u"][:2])
        n_qp += 1
    assert n_qp == 6


def test_run_step_raises_where_the_qp_fails(gpu):
    """An OV parked on the route: the chance constraints leave no feasible plan, run_step
    raises InSimulationException (:3099-3110, :3176-3177) and the harness records
    infeasibility (:389-390)."""
    from ccmpc import harness, standins
    stg = standins.SyntheticTrajectron(L=25, ph=8, seed=1, device=gpu)

    def make_world():
        world, ego, ids, mr = standins.town03_scene(n_ov=1, ego_xy=(60.0, 81.76),
                                                    ego_speed=8.0, ov_gap=22.0, ov_speed=0.0)
        return world, ego, ids, mr
    route = make_world()[3].route_points
    scen = harness.MonteCarloScenario(
        harness.ScenarioParameters(run_interval=10),
        harness.CtrlParameters(n_predictions=2000), make_world, stg,
        agent_kwargs=dict(n_ideal=N_IDEAL, reference_trajectory=route[::2], device=gpu))
    stats = scen.episode(0)
    assert stats.infeasibility and not stats.success


def test_filter_pmf_reaches_every_stage(gpu):
    """sampler['filter_pmf'] != 0.1 sizes K, the step graph and the bucketing alike (Minkowski
    at T == ph through the graph, T < ph eager, the receding affine step)."""
    from ccmpc import episode, planner
    rep = episode.EpisodeReplay(O=2, N=3000, ph=8, n_ideal=N_IDEAL, seed=4, device=gpu)
    agent = planner.MidlevelAgent(prediction_horizon=8, n_ideal=N_IDEAL, seed=4, device=gpu)
    fp = 0.04
    K = (rep.pmf > fp).sum(1)
    assert (K != (rep.pmf > 0.1).sum(1)).any()       # the threshold matters for these inputs
    for frame, T, shrinking in ((0, 8, True), (10, 7, True), (20, 8, False)):
        sampler = dict(init_state=rep.init, latent_pmf=rep.pmf, gmm=rep.gmm, N=rep.N,
                       seed=frame + 1, filter_pmf=fp)
        ref = rep.ref_traj(frame)
        try:
            agent.compute_prediction_controls(frame, T, shrinking, sampler, rep.minpos,
                                              rep.pasts, rep.x_init(frame),
                                              ref[-1] + [4.0, 0.5], ref)
        except planner.InSimulationException:
            pass                                     # the QP may fail; the records are set
        except ValueError as e:                      # T < ph after a failed T == ph QP: no
            assert "needs u_prev" in str(e)          # executed controls; records still set
        ovs, out = agent.last_generator_output
        assert [ov.n_states for ov in ovs] == K.tolist()
        per_cell = T * (T - 1) // 2 if shrinking else T
        assert len(out[0]) == K.sum() * per_cell


def _latents_route(gpu, per_particle, device_tensors=False, run_interval=10,
                   keep_on_device=False):
    """The same scenario with an eval_stg shaped like a real Trajectron++ model (no
    sample_boundary): do_prediction calls generate_vehicle_latents and the step graph takes
    its predictions + z (source='predictions')."""
    import torch
    from ccmpc import standins
    scen = _scenario(gpu, per_particle, run_interval=run_interval)
    scen.eval_stg = standins.TrajectronModel(scen.eval_stg)
    gvl = standins.generate_vehicle_latents
    if device_tensors:          # a predictor that leaves its outputs on the GPU
        def gvl(*a, **k):
            z, pred, nodes, pdict, lp = standins.generate_vehicle_latents(*a, **k)
            return (torch.as_tensor(z, device=gpu), torch.as_tensor(pred, device=gpu), nodes,
                    pdict, lp)
    scen.agent_kwargs["generate_vehicle_latents"] = gvl
    if keep_on_device:          # the opt-in: generate_vehicle_latents(..., keep_on_device=True)
        scen.agent_kwargs["keep_predictions_on_device"] = True
    return scen


@pytest.mark.parametrize("per_particle,device_tensors,keep", [
    (False, False, False), (True, False, False), (False, True, False), (False, False, True),
    (True, False, True)],
    ids=["per_latent", "per_particle", "device_tensors", "keep_on_device",
         "keep_on_device_per_particle"])
def test_reference_predictor_output_drives_run_step(gpu, per_particle, device_tensors, keep):
    """an eval_stg without sample_boundary takes the reference's route --
    generate_vehicle_latents (prediction.py:19-105) -> the 5-tuple -> make_ovehicles on
    predictions + z (v8ideal/__init__.py:469-505) -> generator -> QP, no sampler in the step
    graph.  With a stand-in predictor whose particles are the sampler's own draws, every planning
    step's records, speeds and angles are the sample_boundary route's bytes."""
    from ccmpc import step
    a = _scenario(gpu, per_particle)
    a.episode(0)
    b = _latents_route(gpu, per_particle, device_tensors, keep_on_device=keep)
    b.episode(0)
    assert len(a.steps) == len(b.steps) == 10
    for sa, sb in zip(a.steps, b.steps):
        assert sb["sampler"]["source"] == "predictions"
        assert sa["frame"] == sb["frame"] and sa["T"] == sb["T"]
        assert sa["records"].tobytes() == sb["records"].tobytes(), sa["frame"]
        assert sa["speeds"].tobytes() == sb["speeds"].tobytes()
        assert sa["angles"].tobytes() == sb["angles"].tobytes()
    keys = [k for k in step._POOL if k[1][9] == "predictions"]
    assert keys, "the predictions-source graphs were not used"
    if keep or device_tensors:      # the device route: pred_device graphs, no host pack
        assert any(k[1][10] for k in keys)
        assert torch.is_tensor(b.steps[0]["sampler"]["predictions"])


def test_make_ovehicles_on_the_reference_5_tuple(gpu):
    """The agent's make_ovehicles(result) on do_prediction's 5-tuple: bucketed clouds equal the
    oracle's restatement of :469-505 + from_trajectron on the same predictions + z, and past /
    ground truth come from prediction_output_to_trajectories (+ minpos)."""
    from ccmpc import planner, standins
    scen = _latents_route(gpu, False)
    world, ego, ids, mr = scen.make_world()
    agent = planner.MidlevelAgent(ego, mr, ids, scen.eval_stg,
                                  scene_builder_cls=standins.ReplaySceneBuilder,
                                  scene_config=standins.OnlineConfig(10), prediction_horizon=8,
                                  n_predictions=3000, device=gpu, **{
                                      k: v for k, v in scen.agent_kwargs.items()
                                      if k != "device"})
    frame = world.tick()
    for _ in range(31):
        agent.run_step(frame)                       # burn-in frames only: no planning yet
        frame = world.tick()
    res = agent.do_prediction(agent._first_frame + 30)
    assert set(res) >= {"scene", "timestep", "nodes", "predictions", "z", "latent_probs",
                        "past_dict", "ground_truth_dict"}
    assert res["z"].dtype == np.int64 and res["predictions"].dtype == np.float32
    ovs = agent.make_ovehicles(res)
    minpos = np.array([res["scene"].x_min, res["scene"].y_min])
    rows = [i for i, n in enumerate(res["nodes"]) if n.id != "ego"]
    assert len(ovs) == len(rows)
    ts = res["timestep"]
    pasts = [res["past_dict"][ts][res["nodes"][r]] + minpos for r in rows]
    want = orc.make_ovehicles(res["predictions"][rows], res["z"][rows],
                              np.asarray(res["latent_probs"], float)[rows], minpos, pasts,
                              [np.array([4.5, 2.5])] * len(rows), 8)
    for ov, w, r, past in zip(ovs, want, rows, pasts):
        got = ov.pred_positions
        assert len(got) == len(w.pred_positions)
        for g, x in zip(got, w.pred_positions):
            np.testing.assert_array_equal(g, x)
        np.testing.assert_array_equal(ov.latent_pmf, w.latent_pmf)
        np.testing.assert_array_equal(ov.past, past)
        assert ov.node is res["nodes"][r]
        np.testing.assert_array_equal(ov.ground_truth, res["ground_truth_dict"][ts][
            res["nodes"][r]] + minpos)


@pytest.mark.parametrize("junction", [True, False], ids=["junction_road", "open_road"])
def test_harness_episode_with_road_boundaries(gpu, junction):
    """road_boundary_constraints=True through run_step (v8ideal/__init__.py:2906-2916): every
    planning step is the road MILP over the stand-in map's polytopes (one per step, chosen by
    the branch and bound), each plan inside the polytopes it chose.  On a junction road
    (S_big = 0) the wide lane does not bind and the plans equal the road-free episode's; on an
    open road the affine receding steps' '>=' rows carry S_big = M_big (as the reference writes
    them), which no plan can meet, so those steps fail as the reference's solve would."""
    from ccmpc import harness, standins

    def make_world():
        world, ego, ids, mr = standins.town03_scene(n_ov=1, ego_xy=(60.0, 81.76),
                                                    ego_speed=8.0, ov_gap=20.0, ov_speed=8.0,
                                                    ov_lateral=40.0)
        r = mr.route_points
        disc = [(float(r[0, 0]), float(r[0, 1]), 1e4)] if junction else []
        return world, ego, ids, standins.StubMapReader(r, lane_width=6.0, junctions=disc)

    runs = {}
    for road in (False, True):
        route = make_world()[3].route_points
        stg = standins.SyntheticTrajectron(L=25, ph=8, seed=5, device=gpu)
        scen = harness.MonteCarloScenario(
            harness.ScenarioParameters(n_burn_interval=4, run_interval=10),
            harness.CtrlParameters(n_predictions=2000, prediction_horizon=8, control_horizon=8),
            make_world, stg, agent_kwargs=dict(n_ideal=N_IDEAL, reference_trajectory=route[::2],
                                               road_boundary_constraints=road, device=gpu))
        runs[road] = (scen.episode(0), scen.steps)
    (st0, steps0), (st1, steps1) = runs[False], runs[True]
    assert not st0.infeasibility
    for s in steps1:
        assert s["polytopes"] is not None and len(s["polytopes"]) == s["T"]
        for t, i in enumerate(s["polytopes"]):
            A, b = s["segments"].polytopes[i]
            assert np.all(A @ s["X_star"][t, :2] <= b + 1e-6)
    if junction:
        assert not st1.infeasibility and len(steps1) == len(steps0)
        for a, b in zip(steps0, steps1):
            tol = 1e-6 * (1.0 + np.abs(a["u"]).max())
            assert np.abs(a["u"] - b["u"]).max() <= tol, a["frame"]
    else:
        shrink = [s for s in steps1 if s["shrinking"]]
        assert len(shrink) == 8                        # the Minkowski steps plan
        assert st1.infeasibility                       # the first affine step cannot
