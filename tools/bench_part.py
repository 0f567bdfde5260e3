"""Run named bench.py lines alone on the GPU box (repo root):
    python tools/bench_part.py dropin_step_predictions dropin_step v8_milp
Each prints one JSON line (the function's default arguments; CPU legs skipped where the
function takes with_cpu)."""
import inspect
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for name in sys.argv[1:]:
        fn = getattr(bench, name)
        kw = {"with_cpu": False} if "with_cpu" in inspect.signature(fn).parameters else {}
        if os.environ.get("WITH_CPU") == "1" and kw:
            kw["with_cpu"] = True
        print(json.dumps({name: fn(dev, **kw)}), flush=True)


if __name__ == "__main__":
    main()
