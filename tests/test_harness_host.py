"""Host logic of the harness-facing surface, no GPU: MidlevelAgent's reference constructor
(v8ideal/__init__.py:202-235), run_step's frame gating (:3226-3284) and the Monte-Carlo
episode loop (tests/Hz20/__init__.py:243-359) with the planning step replaced by a recorder;
load_refT's index rule (:2768-2787) and the route goal (road.py:663-666)."""
import numpy as np
import pytest
import torch


@pytest.fixture
def host_agent_cls(monkeypatch):
    """MidlevelAgent whose device checks accept the CPU and whose planning step records its
    arguments and returns a fixed plan (the device chain is tested under -m gpu)."""
    from ccmpc import engine, planner
    monkeypatch.setattr(engine, "require_device", lambda d: torch.device("cpu"))

    class Recorder(planner.MidlevelAgent):
        def _MidlevelAgent__compute_prediction_controls(self, frame, Tsh, shrinking):
            self.calls.append((frame, Tsh, shrinking, self.offline_index))
            x = self.make_local_params(frame, Tsh)
            self._X_warm = np.array([x + np.array([4.0, 0.0, 0.0, 0.0])])
            return np.full(Tsh, 8.0), np.zeros(Tsh), False

    return Recorder


def _make(host_agent_cls, **kw):
    from ccmpc import standins
    world, ego, ids, mr = standins.town03_scene(n_ov=2, ego_xy=(60.0, 81.76), ego_speed=8.0)
    agent = host_agent_cls(ego, mr, ids, None, scene_builder_cls=standins.ReplaySceneBuilder,
                           scene_config=standins.OnlineConfig(record_interval=10),
                           prediction_horizon=8, control_horizon=8, **kw)
    agent.calls = []
    return world, ego, agent


def test_constructor_takes_the_reference_arguments(host_agent_cls):
    world, ego, agent = _make(host_agent_cls, n_coincide=1, random_mcc=True, plot_boundary=False,
                              ego_spawn_idx=85, spawn_shifts=[None])
    assert agent.record_interval == 10 and agent.n_burn_interval == 4
    assert agent.steptime == pytest.approx(0.5)                       # 10 x 0.05 s (:275)
    assert sorted(agent._other_vehicles) == [100, 101]
    assert agent.ego_lon == pytest.approx(3.7) and agent.ego_vehicle_id == 1
    g = agent.get_goal()
    np.testing.assert_allclose([g.x, g.y], agent._road_boundary.points[-1])
    agent.start_sensor()
    assert agent.sensor_is_listening
    with pytest.raises(AssertionError):
        host_agent_cls(ego, None, [], None, prediction_horizon=6, control_horizon=8)


def test_run_step_gating(host_agent_cls):
    world, ego, agent = _make(host_agent_cls, step_horizon=2)
    frame = world.tick()
    first = frame
    for i in range(120):
        agent.run_step(frame, i, 8, True)
        frame = world.tick()
    planned = [c[0] - first for c in agent.calls]
    # every record_interval frames, past n_burn_interval periods, on the step_horizon grid
    assert planned == [40, 60, 80, 100]
    assert [c[3] for c in agent.calls] == [40, 60, 80, 100]          # offline_index passed
    # the first x_init is the simulator's flipped state; later ones the warm start
    assert ego.controls[-1] is not None and "target_speed" in ego.controls[-1]


def test_harness_episode_schedule(host_agent_cls, monkeypatch):
    from ccmpc import harness, standins

    def make_world():
        return standins.town03_scene(n_ov=1, ego_xy=(60.0, 81.76), ego_speed=8.0)
    scen = harness.MonteCarloScenario(harness.ScenarioParameters(run_interval=14),
                                      harness.CtrlParameters(control_horizon=8), make_world,
                                      None, motion_planner_cls=host_agent_cls)
    created = []
    orig_init = host_agent_cls.__init__

    def init(self, *a, **k):
        orig_init(self, *a, **k)
        self.calls = []
        created.append(self)
    monkeypatch.setattr(host_agent_cls, "__init__", init)
    stats = scen.episode(0)
    calls = created[0].calls
    assert [c[1] for c in calls] == [8, 7, 6, 5, 4, 3, 2, 1, 8, 8, 8, 8, 8, 8]
    assert [c[2] for c in calls] == [True] * 8 + [False] * 6
    assert [c[3] for c in calls] == [10 * j for j in range(14)]
    assert stats.steps == 140 and not stats.success and not stats.infeasibility
    assert stats.initiallyFeasible


def test_harness_episode_ends_on_goal_and_infeasible(host_agent_cls, monkeypatch):
    from ccmpc import harness, planner, standins

    def make_world():     # 20 m before the harness's goal: within TOL after a few plans
        return standins.town03_scene(n_ov=1, ego_xy=(167.174698 - 20.0, 81.759842),
                                     ego_speed=4.0)
    scen = harness.MonteCarloScenario(harness.ScenarioParameters(run_interval=14),
                                      harness.CtrlParameters(), make_world, None,
                                      motion_planner_cls=host_agent_cls)
    monkeypatch.setattr(host_agent_cls, "calls", [], raising=False)
    stats = scen.episode(0)
    assert stats.success and stats.steps >= 1

    def fail(self, frame, Tsh, shrinking):
        raise planner.InSimulationException("Optimizer failed to find a solution")
    monkeypatch.setattr(host_agent_cls, "_MidlevelAgent__compute_prediction_controls", fail)
    stats = scen.episode(0)
    assert stats.infeasibility and stats.steps == 0


def test_load_refT_index_rule(host_agent_cls):
    """:2777-2787: nearest route point, or the next when the nearest lies after the third."""
    world, ego, agent = _make(host_agent_cls)
    route = np.stack([np.arange(0.0, 80.0, 4.0), np.zeros(20)], 1)
    agent._ref_route = route
    ref = agent.load_refT(0, 8, np.array([10.9, 0.3, 0, 8]))     # nearest 12 (idx 3), then 8, 16
    np.testing.assert_array_equal(ref[:, 0], route[3:11, 0])
    ref = agent.load_refT(0, 8, np.array([13.1, 0.3, 0, 8]))     # nearest 12, then 16, 8
    np.testing.assert_array_equal(ref[:, 0], route[4:12, 0])
    with pytest.raises(IndexError):
        agent.load_refT(0, 8, np.array([75.0, 0.0, 0, 8]))


def test_route_goal_rule():
    """road.py:663-666: nearest route point, then the first point at or beyond its distance +
    distance (right-closed intervals), clamped to the path's end."""
    from ccmpc import standins
    rb = standins.PolylineRoadBoundary(np.stack([np.arange(0.0, 41.0, 2.0), np.zeros(21)], 1))
    np.testing.assert_array_equal(rb.collect_segs_polytopes_and_goal([3.1, 0.0], 9.0).goal,
                                  [14.0, 0.0])       # nearest 4 -> 13 -> (12, 14] -> 14
    np.testing.assert_array_equal(rb.collect_segs_polytopes_and_goal([3.1, 0.0], 10.0).goal,
                                  [14.0, 0.0])       # 14 lies in (12, 14]
    np.testing.assert_array_equal(rb.collect_segs_polytopes_and_goal([30.0, 1.0], 99.0).goal,
                                  [40.0, 0.0])


def test_road_segments_cover_the_route():
    """The stand-in's road polytopes (road.py:468-556 restated for a polyline): every route
    point lies in some polytope, neighbours overlap, a junction disc marks its polytopes, and
    collect_segs_polytopes_and_goal slices [id(beg) - 1, id(end) + 1) as road.py:667-678."""
    from ccmpc import standins
    route = np.stack([np.arange(0.0, 81.0, 2.0), 0.5 * np.arange(0.0, 81.0, 2.0) ** 0.5], 1)
    rb = standins.PolylineRoadBoundary(route, lane_width=3.5, seg_len=10.0,
                                       junctions=[(45.0, 3.3, 6.0)])
    polys, mask = rb.road_segs.polytopes, rb.road_segs.mask
    for p in route:
        assert any(np.all(A @ p <= b + 1e-9) for A, b in polys)
    for i, ((A0, b0), (A1, b1)) in enumerate(zip(polys, polys[1:])):   # a shared point
        q = rb.get_point_from_start(rb.road_segs.distances[i + 1])
        assert np.all(A0 @ q <= b0 + 1e-9) and np.all(A1 @ q <= b1 + 1e-9)
    assert mask.any() and not mask.all()
    seg = rb.collect_segs_polytopes_and_goal([21.0, 2.0], 25.0)
    i0 = int(np.searchsorted(rb.road_segs.distances, rb.distances[10], side="right")) - 1
    assert seg.polytope_ids[0] == max(i0 - 1, 0)
    assert len(seg.polytopes) == len(seg.mask) == len(seg.polytope_ids)
    np.testing.assert_array_equal(seg.mask, mask[seg.polytope_ids])


def test_prediction_output_to_trajectories_over_standin_nodes(host_agent_cls):
    """Trajectron++'s prediction_output_to_trajectories as restated in ccmpc.prediction, over the
    scene builder's nodes (Node.get pads with NaN outside the track): the history is the track's
    last max_h + 1 positions (the sample_boundary route's scene.past), the future is empty in a
    live simulation, the prediction passes through."""
    from ccmpc import prediction
    world, ego, agent = _make(host_agent_cls)
    frame = world.tick()
    for _ in range(131):                          # 14 recorded timesteps, no planning call
        agent.run_step(frame) if agent._first_frame is None or \
            (frame - agent._first_frame) // 10 < 4 else \
            agent._scene_builder.capture_trajectory(frame)
        frame = world.tick()
    scene = agent._scene_builder.get_scene()
    ts = scene.timestep
    assert ts == 13
    preds = {n: np.full((1, 5, 8, 2), float(i)) for i, n in enumerate(scene.nodes)}
    out, hist, fut = prediction.prediction_output_to_trajectories({ts: preds}, dt=scene.dt,
                                                                  max_h=10, ph=8)
    past = scene.past(ts, max_h=10)
    for n in scene.nodes:
        np.testing.assert_array_equal(hist[ts][n], past[n])
        assert hist[ts][n].shape == (11, 2)
        assert fut[ts][n].shape == (0, 2)
        assert out[ts][n] is preds[n]
    # an early timestep: the history is cut at the track's start (NaN rows dropped)
    _, hist2, _ = prediction.prediction_output_to_trajectories({2: preds}, scene.dt, 10, 8)
    for n in scene.nodes:
        np.testing.assert_array_equal(hist2[2][n], scene.past(2, max_h=10)[n])
        assert hist2[2][n].shape == (3, 2)


def test_generate_vehicle_latents_fails_like_the_reference_without_trajectron():
    """prediction.py:13-17: without the trajectron-plus-plus submodule the reference's import
    raises; the restated glue raises the same exception when a Trajectron++ eval_stg is used."""
    from ccmpc import prediction
    with pytest.raises(Exception, match="trajectron"):
        prediction.generate_vehicle_latents(object(), None, np.array([0]))
