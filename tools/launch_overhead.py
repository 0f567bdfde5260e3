"""Per-step cost of the C2 cycle under different host launch paths (GPU box):

  graph      torch.cuda.CUDAGraph.replay() per step (what bench.py times)
  ctypes     one ccmpc_minkowski_cycle C-ABI call per step, no graph
  events     device time per step from HIP events around the same replay loop
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import torch  # noqa: E402

from ccmpc import cycle, engine, synthetic  # noqa: E402


def timed(fn, steps, dev):
    for _ in range(50):
        fn()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    host = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    return host / steps * 1e6, wall / steps * 1e6, e0.elapsed_time(e1) * 1e3 / steps


def main():
    dev = torch.device("cuda:0")
    ovs, ref, _ = synthetic.scene(0, O=4, N=5000, T=8)
    K = [len(o) for o in ovs]
    store = engine.ParticleStore.from_cells([c for o in ovs for c in o], device=dev)
    cyc = cycle.MinkowskiCycle(store, K, ref)
    cyc_g = cycle.MinkowskiCycle(store, K, ref).capture()
    cyc_b = cycle.MinkowskiCycle(store, K, ref).bind()
    for name, fn in (("graph replay", cyc_g.replay), ("ctypes direct", cyc.run),
                     ("bound launch", cyc_b.launch)):
        h, w, d = timed(fn, 2000, dev)
        print(f"{name:14s}: host enqueue {h:7.2f} us/step, wall {w:7.2f} us/step, "
              f"device {d:7.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
