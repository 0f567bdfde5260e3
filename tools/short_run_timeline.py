"""Where a short timed run (the driver's --steps 20) loses time against the per-launch
figure: the bench's C2 step launched K times after the bench's own warm-up / sync / barrier
sequence, with a HIP event after every launch and host stamps around the loop (GPU box)."""
import os
import sys
import time

ROOT = os.getcwd()
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]
import numpy as np
import torch

import bench

bench.spin_sync(0)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
from ccmpc import cycle, engine, synthetic  # noqa: E402

ovs, ref, _ = synthetic.scene(0, O=4, N=5000, T=8)
K = [len(o) for o in ovs]
store = engine.ParticleStore.from_cells([c for o in ovs for c in o], device=dev)
cyc = cycle.MinkowskiCycle(store, K, ref)
step = cyc.bind().launch
for K_steps in (20, 20, 20, 200, 2000):
    for _ in range(5):
        step()
    torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    th = np.empty(K_steps)
    t0 = time.perf_counter()
    e0.record()
    ta = time.perf_counter()
    for i in range(K_steps):
        step()
        th[i] = time.perf_counter()
    e1.record()
    tb = time.perf_counter()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    gpu = e0.elapsed_time(e1) * 1e3
    dh = np.diff(np.concatenate([[ta], th]))
    print(f"K={K_steps}: host {1e6 * (t1 - t0) / K_steps:.2f} us/step, events {gpu / K_steps:.2f} "
          f"us/step; host launch costs first 5 {np.round(1e6 * dh[:5], 2)} median "
          f"{1e6 * np.median(dh):.2f} us; event record {1e6 * (ta - t0):.1f} us; sync wait "
          f"after the last enqueue {1e6 * (t1 - tb):.1f} us")
