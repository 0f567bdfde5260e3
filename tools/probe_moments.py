"""Run one bench configuration's moments kernel (or full cycle) in a loop, for rocprofv3.

    python tools/probe_moments.py C4 moments 200
    python tools/probe_moments.py C5 cycle 100
    python tools/probe_moments.py ALL time 0      (graph-timed us per launch, every config)
    ROTATE=3 python tools/probe_moments.py C4full cycle 30   (launches rotate over 3 copies of
                                                              the store: every launch from HBM)
"""
import os

import numpy as np
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import torch  # noqa: E402

from ccmpc import cycle, engine, synthetic  # noqa: E402

CONFIGS = {"C2": (4, 5000, 8, 1), "C3": (1, 100000, 8, 1), "C4": (4, 20000, 12, 8),
           "C5": (8, 50000, 40, 1), "C3-1e3": (1, 1000, 8, 1), "C3-2e4": (1, 20000, 8, 1),
           "C4full": (4, 20000, 12, 64), "C4-f32": (4, 20000, 12, 8)}


def build(name, dev):
    O, N, T, scenes = CONFIGS[name]
    cells, K, refs = [], [], []
    for sc in range(scenes):
        ovs, ref, _ = synthetic.scene(1000 + sc, O=O, N=N, T=T)
        cells += [c for o in ovs for c in o]
        K += [len(o) for o in ovs]
        refs.append(ref)
    if name.endswith("-f32"):            # the sampler's store format: f32 relative to an origin
        origin = np.tile(np.array([150.0, -120.0]), (len(cells), 1))
        store = engine.ParticleStore.from_cells(cells, device=dev, dtype=torch.float32,
                                                origin=origin)
    else:
        store = engine.ParticleStore.from_cells(cells, device=dev)
    return store, cycle.MinkowskiCycle(store, K, refs[0])


def time_all(dev):
    sys.path.insert(0, ROOT)
    from bench import time_kernel_live
    for name in CONFIGS:
        store, cyc = build(name, dev)
        tm = time_kernel_live(lambda: engine.moments(store, cyc.mean, cyc.cov, cyc.ws), dev,
                              per_graph=10, replays=5)
        tc = time_kernel_live(cyc.run, dev, per_graph=10, replays=5)
        print(f"{name}: moments {tm * 1e6:8.2f} us   cycle {tc * 1e6:8.2f} us", flush=True)


def main():
    name, what, iters = sys.argv[1], sys.argv[2], int(sys.argv[3])
    if what == "time":
        time_all(torch.device("cuda:0"))
        return
    O, N, T, scenes = CONFIGS[name]
    dev = torch.device("cuda:0")
    cells, K, refs = [], [], []
    for sc in range(scenes):
        ovs, ref, _ = synthetic.scene(1000 + sc, O=O, N=N, T=T)
        cells += [c for o in ovs for c in o]
        K += [len(o) for o in ovs]
        refs.append(ref)
    store = engine.ParticleStore.from_cells(cells, device=dev)
    cyc = cycle.MinkowskiCycle(store, K, refs[0])
    cycles = [cyc]
    for _ in range(int(os.environ.get("ROTATE", "1")) - 1):
        sys.path.insert(0, ROOT)
        from bench import clone_cycle
        cycles.append(clone_cycle(cyc))
    fns = [c.run if what == "cycle" else
           (lambda c=c: engine.moments(c.store, c.mean, c.cov, c.ws)) for c in cycles]
    for i in range(iters):
        fns[i % len(fns)]()
    torch.cuda.synchronize()
    print(f"{name} {what} x{iters}: {sum(store.counts)} particles, {store.n_cells} cells")


if __name__ == "__main__":
    main()
