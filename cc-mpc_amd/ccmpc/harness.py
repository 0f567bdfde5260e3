"""The Monte-Carlo harness's episode loop (tests/Hz20/__init__.py:37-447, MonteCarloScenario)
over the stand-ins of ccmpc.standins, so the reference's own driver sequence runs through the
library: construct MidlevelAgent with the splatted scenario / control / debug dicts
(:183-193), start its sensor, burn n_burn_interval planning periods of frames (:243-255),
then the shrinking-then-receding loop of the `shrinking_dist` branch (:297-359) calling
run_step(frame, offline_index, T, shrinking) every frame, world.tick() between frames, the
goal-distance checks and the stats the reference logs.

The simulator is replaced (StubWorld / StubVehicle), so spawning, traffic-manager settings,
spectator placement and sleeps (:107-241, :401) are not replayed; everything from the agent's
construction on is.  Each planning step's inputs and outputs are recorded in `steps` for the
parity tests.
"""
import math
import time

from . import planner, standins


class ScenarioParameters(standins.AttrDict):
    """tests/__init__.py:45-117's fields the episode reads (n_burn_interval, run_interval,
    controls, goal) plus the stand-in scene geometry."""

    def __init__(self, n_burn_interval=4, run_interval=22, controls=(), goal=None, **kw):
        super().__init__(n_burn_interval=n_burn_interval, run_interval=run_interval,
                         controls=list(controls), goal=goal, **kw)


class CtrlParameters(standins.AttrDict):
    """tests/__init__.py:119-138 (loop_type: CLOSED_LOOP)."""

    def __init__(self, n_predictions=100, prediction_horizon=8, control_horizon=8,
                 step_horizon=1, n_coincide=1, random_mcc=False, closed_loop=True):
        super().__init__(n_predictions=n_predictions, prediction_horizon=prediction_horizon,
                         control_horizon=control_horizon, step_horizon=step_horizon,
                         n_coincide=n_coincide, random_mcc=random_mcc, closed_loop=closed_loop)


class MonteCarloScenario:
    TOL = 6                                     # :48
    GOAL = (167.174698, -81.759842)             # the goal the loop measures against (:305-306)
    SHRINK_DIST = 36                            # :326

    DEBUG_SETTINGS = dict(plot_boundary=False, log_agent=False, log_cplex=False,
                          plot_scenario=False, plot_simulation=False, plot_overapprox=False)

    def __init__(self, scenario_params, ctrl_params, make_world, eval_stg,
                 motion_planner_cls=planner.MidlevelAgent,
                 scene_builder_cls=standins.ReplaySceneBuilder, record_interval=10,
                 agent_kwargs=None):
        """make_world() -> (world, ego_vehicle, other_vehicle_ids, map_reader): a fresh
        stand-in scene per episode (the reference spawns actors, :129-180)."""
        self.scenario_params, self.ctrl_params = scenario_params, ctrl_params
        self.make_world, self.eval_stg = make_world, eval_stg
        self.motion_planner_cls, self.scene_builder_cls = motion_planner_cls, scene_builder_cls
        self.online_config = standins.OnlineConfig(record_interval=record_interval)
        self.agent_kwargs = dict(agent_kwargs or {})
        self.steps = []                         # per planning step: inputs, outputs, timing
        self.agent = None

    def _run_step(self, agent, frame, *args):
        """agent.run_step, recording the planning steps it takes."""
        n_before = len(getattr(agent, "_step_log", []))
        t0 = time.perf_counter()
        out = agent.run_step(frame, *args)
        dt = time.perf_counter() - t0
        log = getattr(agent, "_step_log", [])
        if len(log) > n_before:
            log[-1]["run_step_ms"] = dt * 1e3
            self.steps.append(log[-1])
        return out

    def episode(self, episode_idx=0):
        self.steps = []
        stats = standins.AttrDict(success=False, infeasibility=False, steps=0, plan_steps=0,
                                  timeOver=False, initiallyFeasible=False)
        world, ego, ov_ids, map_reader = self.make_world()
        agent = None
        try:
            shrinking = True
            shrinkIndex = (self.ctrl_params.control_horizon + 1) * 10 - 1       # :127
            frame = world.tick()
            kw = {k: v for k, v in self.scenario_params.items() if k != "goal"}
            kw.update({k: v for k, v in self.ctrl_params.items() if k != "closed_loop"})
            kw.update(self.DEBUG_SETTINGS)
            kw.update(self.agent_kwargs)
            agent = self.motion_planner_cls(ego, map_reader, ov_ids, self.eval_stg,
                                            scene_builder_cls=self.scene_builder_cls,
                                            scene_config=self.online_config, **kw)
            agent._step_log = []
            self.agent = agent
            agent.start_sensor()
            assert agent.sensor_is_listening
            if self.scenario_params.goal:
                agent.set_goal(**self.scenario_params.goal)
            ri = self.online_config.record_interval
            n_burn_frames = self.scenario_params.n_burn_interval * ri
            if self.ctrl_params.closed_loop:
                run_frames = self.scenario_params.run_interval * ri
            else:
                run_frames = self.ctrl_params.control_horizon * ri - 1
            for idx in range(n_burn_frames):                                  # :248-255
                control = None
                for ctrl in self.scenario_params.controls:
                    if ctrl["interval"][0] <= idx <= ctrl["interval"][1]:
                        control = ctrl["control"]
                        break
                agent.run_step(frame, control=control)
                frame = world.tick()
            T = self.ctrl_params.control_horizon
            once_shrink = False
            offline_index = 0
            gx, gy = self.GOAL
            for idx in range(run_frames):                                     # :261-359
                if not shrinking:                                             # receding
                    stats.timeOver = self._run_step(agent, frame, offline_index, T, shrinking)
                    offline_index += 1
                    frame = world.tick()
                    stats.steps += 1
                    state = agent.get_vehicle_state(flip_y=True)
                    dist = math.sqrt((state[0] - gx) ** 2 + (state[1] - gy) ** 2)
                    if stats.timeOver:
                        break
                    if dist < self.TOL:
                        stats.success = True
                        break
                    if not once_shrink and dist < self.SHRINK_DIST:
                        shrinking = True
                else:                                                         # shrinking
                    T = max(1, shrinkIndex // 10)
                    if T <= self.ctrl_params.control_horizon - 1:
                        stats.initiallyFeasible = True
                    stats.timeOver = self._run_step(agent, frame, offline_index, T, shrinking)
                    offline_index += 1
                    frame = world.tick()
                    stats.steps += 1
                    state = agent.get_vehicle_state(flip_y=True)
                    dist = math.sqrt((state[0] - gx) ** 2 + (state[1] - gy) ** 2)
                    if stats.timeOver:
                        break
                    if dist < self.TOL:
                        stats.success = True
                        break
                    shrinkIndex -= 1
                    if shrinkIndex // 10 < 1:
                        T = self.ctrl_params.control_horizon
                        once_shrink = True
                        shrinking = False
                        shrinkIndex = self.ctrl_params.control_horizon * 10 - 1
        except planner.InSimulationException:
            stats.infeasibility = True
        finally:
            if agent is not None:
                agent.destroy()
            stats.plan_steps = stats.steps / self.online_config.record_interval
        return stats
