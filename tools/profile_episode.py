"""cProfile of the C1 episode replay's host side (GPU box): where a planning step's ~1 ms goes."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import torch  # noqa: E402

from ccmpc import episode  # noqa: E402

dev = torch.device("cuda:0")
episode.EpisodeReplay(O=1, N=5000, n_ideal=1_000_000, receding_steps=4, device=dev).run()
rep = episode.EpisodeReplay(O=1, N=5000, n_ideal=1_000_000, receding_steps=4, device=dev)
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    rep = episode.EpisodeReplay(O=1, N=5000, n_ideal=1_000_000, receding_steps=4, device=dev)
    rep.run(sync=False)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
