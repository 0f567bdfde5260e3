"""A/B of the planning QP kernel's wave count or method (GPU box, repo root):

    python tools/ab_qp.py            one child per CCMPC_QP_WAVES value (1, 4)
    python tools/ab_qp.py method     one child per CCMPC_QP_METHOD value (ipm, gi)

Each child runs bench.planning_qp (64 crossing scenes, one launch) and one single-scene solve
(the planning step's own QP, as solve_planning_qp runs it) and prints one JSON line."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]
    import numpy as np
    import torch
    import bench
    dev = torch.device("cuda", 0)
    batch = bench.planning_qp(dev, 20251015, with_cpu=False)
    single = bench.planning_qp(dev, 20251015, scenes=1, with_cpu=False)
    print(json.dumps({"waves": os.environ.get("CCMPC_QP_WAVES", "1"),
                      "method": os.environ.get("CCMPC_QP_METHOD", "default"),
                      "batch64_kernel_us": batch["kernel_us"], "batch_solved": batch["solved"],
                      "batch_iters_max": batch.get("iters_solved_max"),
                      "single_kernel_us": single["kernel_us"],
                      "single_iters": single.get("iters_solved_max"),
                      "max_abs_du_vs_oracle": batch.get("max_abs_du_vs_oracle")}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
    elif len(sys.argv) > 1 and sys.argv[1] == "method":
        for m in ("ipm", "gi", "ipm", "gi"):
            env = dict(os.environ, CCMPC_QP_METHOD=m)
            subprocess.run([sys.executable, __file__, "child"], env=env, check=True)
    else:
        for w in ("1", "4", "1", "4"):
            env = dict(os.environ, CCMPC_QP_WAVES=w)
            subprocess.run([sys.executable, __file__, "child"], env=env, check=True)
