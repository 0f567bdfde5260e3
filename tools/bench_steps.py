"""The planning-step lines of bench.py alone (GPU box, repo root): the drop-in step at the C2
shape (per-latent and per-particle) and at 100 000 particles, the C1 episode and the harness
episode, without the CPU legs.  One JSON object per line.

    python tools/bench_steps.py [dropin|dropin_pp|dropin_100k|episode|harness ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

SEED = 20251015  # bench.py's --seed default, so the QP lines are the same scenes


def main():
    which = sys.argv[1:] or ["dropin", "dropin_pp", "dropin_100k", "episode", "harness"]
    dev = torch.device("cuda", 0)
    runs = {
        "dropin": lambda: bench.dropin_step(dev, with_cpu=False),
        "dropin_pp": lambda: bench.dropin_step(dev, with_cpu=False, per_particle=True),
        "dropin_100k": lambda: bench.dropin_step(dev, steps=100, with_cpu=False, O=1,
                                                 N=100_000, label="C1 (n_predictions = 100 000)"),
        "dropin_pred": lambda: bench.dropin_step_predictions(dev),
        "dropin_pred_100k": lambda: bench.dropin_step_predictions(dev, steps=100, O=1,
                                                                  N=100_000, n_sets=4),
        "dropin_pred_dev": lambda: bench.dropin_step_predictions(dev, on_device=True),
        "dropin_pred_100k_dev": lambda: bench.dropin_step_predictions(
            dev, steps=100, O=1, N=100_000, n_sets=4, on_device=True),
        "qp": lambda: bench.planning_qp(dev, SEED, with_cpu=False),
        "qp1_t8": lambda: bench.planning_qp(dev, SEED, scenes=1, with_cpu=False),
        "qp1_t12": lambda: bench.planning_qp(dev, SEED, scenes=1, T=12, with_cpu=False),
        "qp_t12": lambda: bench.planning_qp(dev, SEED, T=12, with_cpu=False),
        "qp1_t12_solved": lambda: bench.planning_qp(
            dev, SEED, scenes=1, T=12, with_cpu=False,
            first=bench.planning_qp(dev, SEED, T=12, with_cpu=False)["first_solved_scene"]),
        "milp": lambda: bench.v8_milp(dev, with_cpu=False),
        "episode": lambda: bench.episode_c1(dev, with_cpu=False),
        "harness": lambda: bench.harness_episode(dev),
    }
    for w in which:
        print(json.dumps({w: runs[w]()}), flush=True)


if __name__ == "__main__":
    main()
