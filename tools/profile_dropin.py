"""The drop-in planning steps of bench.py (C2 synthetic, C2 per-particle, C1 at 100k particles)
without their CPU legs, for `rocprofv3 --kernel-trace --stats -- python3 tools/profile_dropin.py`
(per-kernel durations of the step graphs).  ONLY=c2,pp,c1 selects."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    only = os.environ.get("ONLY", "c2,pp,c1").split(",")
    runs = {"c2": dict(), "pp": dict(per_particle=True),
            "c1": dict(O=1, N=100_000, label="C1 (n_predictions = 100 000)")}
    for name in only:
        r = bench.dropin_step(dev, steps=200, with_cpu=False, eager_steps=10, **runs[name])
        print(json.dumps({name: {k: r[k] for k in ("dropin_step_us_median", "graph_replay_us",
                                                    "graph_branch")}}), flush=True)


if __name__ == "__main__":
    main()
