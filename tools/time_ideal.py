"""A/B timing of the fused ideal rollout (ccmpc_ideal_minkowski_cycle) across libccmpc builds
(GPU box, repo root):

    python tools/time_ideal.py main build_x ...     (names: csrc/<name>/libccmpc.so)

Each variant runs in a child process; one line per (T, cells): the launch's average device
time (bench.time_kernel_live) and a checksum of the moments (equal checksums = same bits).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [(7, 1), (7, 2), (4, 1), (1, 1)]


def child():
    sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]
    import torch
    import bench
    from ccmpc import engine, risk, synthetic
    dev = torch.device("cuda", 0)
    ovs, ref, _ = synthetic.scene(20251022, O=1, N=100000, T=8, K=2)
    store = engine.ParticleStore.from_cells(ovs[0], device=dev)
    mean, cov = engine.moments(store)
    cr = torch.as_tensor(risk.cell_risk(risk.eps_ura([2]), [2], 8), device=dev)
    ws = engine.Workspace(dev)
    for T, cells in CASES:
        src = torch.arange(cells, dtype=torch.int32, device=dev)
        reft = torch.as_tensor(ref[None, :T], device=dev)
        fn = lambda: engine.ideal_minkowski_cycle(mean, cov, src, T, 1_000_000, reft, cr, seed=3,
                                                  workspace=ws)
        out = fn()
        torch.cuda.synchronize(dev)
        ts = [bench.time_kernel_live(fn, dev, per_graph=4, replays=5) for _ in range(3)]
        flat = [v for v in (out if isinstance(out, (tuple, list)) else [out])
                if isinstance(v, torch.Tensor) and v.is_floating_point()]
        chk = float(sum(v.double().abs().sum().item() for v in flat))
        print(json.dumps({"T": T, "cells": cells, "us": [round(t * 1e6, 2) for t in ts],
                          "checksum": repr(chk)}), flush=True)


def main():
    if sys.argv[1:2] == ["--child"]:
        child()
        return
    for v in sys.argv[1:]:
        env = dict(os.environ)
        if v != "main":
            env["CCMPC_LIB"] = os.path.join(ROOT, "cc-mpc_amd", "csrc", v, "libccmpc.so")
        print(f"== {v}", flush=True)
        r = subprocess.run([sys.executable, "-u", __file__, "--child"], env=env, cwd=ROOT)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
