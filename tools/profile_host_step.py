"""Host-side profile of the drop-in planning step at the C2 shape (GPU box): cProfile over
MidlevelAgent.predict_and_constrain, sorted by own time -- where the Python around the graph
replay goes."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ccmpc import episode, planner  # noqa: E402


def main():
    O, N, ph = 4, 5000, 8
    dev = torch.device("cuda", 0)
    init, pmf, gmm = episode.synthetic_gmm(O, T=ph, seed=20251015)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]]) for o in range(O)]
    K = [int(np.count_nonzero(pmf[o] > 0.1)) for o in range(O)]
    eps = np.full((O, max(K)), 0.05 / O)
    ref = np.array([[165.0 + 4.0 * (t + 1), -72.0 + 0.5 * (t + 1)] for t in range(ph)])
    agent = planner.MidlevelAgent(prediction_horizon=ph, device=dev)
    params = episode.Params(O, K, 0)

    def step(i):
        agent.predict_and_constrain(params, dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N,
                                                 seed=i), eps, ph, ref, minpos, pasts)
    for i in range(30):
        step(i)
    pr = cProfile.Profile()
    pr.enable()
    for i in range(500):
        step(100 + i)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
