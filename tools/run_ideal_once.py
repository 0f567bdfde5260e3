"""Eager launches of the fused ideal rollout for a profiler pass (GPU box, repo root):

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ideal -- python tools/run_ideal_once.py

T = 7, one cell of 1e6 samples, 5 launches (the first warms the allocator and code object).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import torch  # noqa: E402
from ccmpc import engine, risk, synthetic  # noqa: E402


def main(T=7, launches=5):
    dev = torch.device("cuda", 0)
    ovs, ref, _ = synthetic.scene(20251022, O=1, N=100000, T=8, K=2)
    store = engine.ParticleStore.from_cells(ovs[0], device=dev)
    mean, cov = engine.moments(store)
    cr = torch.as_tensor(risk.cell_risk(risk.eps_ura([2]), [2], 8), device=dev)
    ws = engine.Workspace(dev)
    src = torch.zeros(1, dtype=torch.int32, device=dev)
    reft = torch.as_tensor(ref[None, :T], device=dev)
    for _ in range(launches):
        engine.ideal_minkowski_cycle(mean, cov, src, T, 1_000_000, reft, cr, seed=3, workspace=ws)
    torch.cuda.synchronize(dev)
    print("ok", flush=True)


if __name__ == "__main__":
    main()
