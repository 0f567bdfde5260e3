"""The headline loop's fixed cost (GPU box): bench.py's timed region (K direct C-ABI launches of
the C2 cycle between synchronisations) at several K, with the host's issue time of the K
launches apart, so elapsed = fixed + K * per-launch can be read off.

    python tools/launch_overhead.py
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from ccmpc import cycle, engine, synthetic
    spun = bench.spin_sync(0)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ovs, ref, _ = synthetic.scene(20251015, O=4, N=5000, T=8)
    store = engine.ParticleStore.from_cells([c for o in ovs for c in o], device=dev)
    cyc = cycle.MinkowskiCycle(store, [len(o) for o in ovs], ref)
    step = cyc.bind().launch
    for _ in range(200):
        step()
    torch.cuda.synchronize(dev)
    print("spin sync:", spun)
    t = []
    for _ in range(200):
        t0 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t.append(time.perf_counter() - t0)
    print(f"empty synchronize: {1e6 * statistics.median(t):.2f} us")
    for K in (1, 2, 5, 10, 20, 50, 200):
        iss, tot = [], []
        for _ in range(30):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(K):
                step()
            t1 = time.perf_counter()
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter()
            iss.append(t1 - t0)
            tot.append(t2 - t0)
        mi, mt = statistics.median(iss), statistics.median(tot)
        print(f"K {K:4d}: issue {1e6 * mi / K:6.2f} us/launch, elapsed {1e6 * mt:8.1f} us "
              f"= {1e6 * mt / K:6.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
