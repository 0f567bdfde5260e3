"""Where the drop-in planning step's time goes (GPU box): host-side cProfile of
MidlevelAgent.predict_and_constrain at C2's shape, and (under rocprofv3 --kernel-trace --stats)
the per-kernel durations of the captured step graph.

    python tools/profile_step.py [--steps 300] [--no-cprofile]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--no-cprofile", action="store_true")
    a = ap.parse_args()
    from ccmpc import episode, planner
    O, N, ph = 4, 5000, 8
    dev = torch.device("cuda", 0)
    init, pmf, gmm = episode.synthetic_gmm(O, T=ph, seed=20251015)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]])
             for o in range(O)]
    K = [int(np.count_nonzero(pmf[o] > 0.1)) for o in range(O)]
    eps = np.full((O, max(K)), 0.05 / O)
    ref = np.array([[165.0 + 4.0 * (t + 1), -72.0 + 0.5 * (t + 1)] for t in range(ph)])
    agent = planner.MidlevelAgent(prediction_horizon=ph, device=dev)
    params = episode.Params(O, K, 0)

    def step(seed):
        sampler = dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=seed)
        return agent.predict_and_constrain(params, sampler, eps, ph, ref, minpos, pasts)

    for i in range(20):
        step(i)
    g = next(iter(agent._graphs.values()))
    t0 = time.perf_counter()
    for i in range(a.steps):
        g.graphs[0].replay()
        torch.cuda.current_stream().synchronize()
    print(f"replay + sync: {(time.perf_counter() - t0) / a.steps * 1e6:.1f} us")
    g.bind()
    for i in range(10):
        g.launch(direct=True)
        g.wait()
    t0 = time.perf_counter()
    for i in range(a.steps):
        g.launch(direct=True)
        g.wait()
    print(f"direct launches + sync: {(time.perf_counter() - t0) / a.steps * 1e6:.1f} us")
    t0 = time.perf_counter()
    for i in range(a.steps):
        g.launch(direct=True)
    torch.cuda.current_stream().synchronize()
    print(f"direct launches, host only: {(time.perf_counter() - t0) / a.steps * 1e6:.1f} us")
    t0 = time.perf_counter()
    for i in range(a.steps):
        g.graphs[0].replay()
    torch.cuda.current_stream().synchronize()
    print(f"graph replays, host only: {(time.perf_counter() - t0) / a.steps * 1e6:.1f} us")
    t0 = time.perf_counter()
    for i in range(a.steps):
        g.set_inputs(i, init, pmf, gmm, minpos, ref, np.zeros((sum(K), 3)) + 1,
                     np.zeros((sum(K), 2)), np.zeros((sum(K), 2)) + 1)
    print(f"set_inputs: {(time.perf_counter() - t0) / a.steps * 1e6:.1f} us")
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(100 + i)
    print(f"whole step: {(time.perf_counter() - t0) / a.steps * 1e6:.1f} us")
    if not a.no_cprofile:
        pr = cProfile.Profile()
        pr.enable()
        for i in range(a.steps):
            step(5000 + i)
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
