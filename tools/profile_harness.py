"""Host profile of the harness loop's planning frames (GPU box, repo root): bench.py's
harness_episode setup, three warm episodes, then cProfile over run_step in two more; prints the
functions by their own time and by cumulative time."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.getcwd()
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]
import torch  # noqa: E402

from ccmpc import harness, planner, standins  # noqa: E402

dev = torch.device("cuda", 0)
stg = standins.SyntheticTrajectron(L=25, ph=8, seed=5, per_particle=True, device=dev)


def make_world():
    return standins.town03_scene(n_ov=1, ego_xy=(60.0, 81.76), ego_speed=8.0, ov_gap=20.0,
                                 ov_speed=8.0, ov_lateral=40.0)


route = make_world()[3].route_points[::2]
prof = cProfile.Profile()
orig = planner.MidlevelAgent.run_step


def run_step(self, *a, **k):
    if getattr(run_step, "on", False):
        prof.enable()
        try:
            return orig(self, *a, **k)
        finally:
            prof.disable()
    return orig(self, *a, **k)


planner.MidlevelAgent.run_step = run_step
for e in range(5):
    run_step.on = e >= 3
    scen = harness.MonteCarloScenario(
        harness.ScenarioParameters(n_burn_interval=4, run_interval=12),
        harness.CtrlParameters(n_predictions=5000, prediction_horizon=8, control_horizon=8),
        make_world, stg, agent_kwargs=dict(n_ideal=1_000_000, reference_trajectory=route,
                                           device=dev))
    t0 = time.perf_counter()
    scen.episode(e)
    print(f"episode {e}: {1e3 * (time.perf_counter() - t0):.2f} ms, plan ms "
          f"{[round(st['run_step_ms'], 3) for st in scen.steps]}", flush=True)
st = pstats.Stats(prof)
st.sort_stats("tottime").print_stats(35)
st.sort_stats("cumulative").print_stats(45)
