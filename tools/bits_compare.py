"""Bit-for-bit comparison of two libccmpc.so builds on the cycle's outputs (GPU box, repo root):

    python tools/bits_compare.py build_r0 main      ("main" = the in-tree library)

Each build runs in a child process that dumps every configuration's mean, covariance,
half-space records and lower probabilities (one-launch cycle, plus the moments-only launch) to
gpurun_out/bits_<build>.npz; the parent then compares the two dumps byte for byte.  Used to
show that a change to the reduction's shape (tree levels, gathers) keeps the same bits.
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (name, O, N, T, scenes, store dtype): the C3 sweep (one cell per OV, up to 2-level trees),
# C2, a Scheme4 single cell, the C4 batch and C5 (deferred root at T = 40)
CONFIGS = [("C2", 4, 5000, 8, 1, "f32"), ("C3-1e3", 1, 1000, 8, 1, "f32"),
           ("C3-2e4", 1, 20000, 8, 1, "f32"), ("C3-1e5", 1, 100000, 8, 1, "f32"),
           ("C3-2e5", 1, 200000, 8, 1, "f32"), ("C3-1e5-f64", 1, 100000, 8, 1, "f64"),
           ("T12-1e5", 1, 100000, 12, 1, "f32"), ("T20-1e5", 1, 100000, 20, 1, "f32"),
           ("C4/8", 4, 20000, 12, 8, "f32"), ("C5", 8, 50000, 40, 1, "f32")]


def dump(out):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]
    import torch
    from ccmpc import cycle, engine, synthetic
    dev = torch.device("cuda", 0)
    res = {}
    for name, O, N, T, scenes, dt in CONFIGS:
        cells, K, refs = [], [], []
        for sc in range(scenes):
            ovs, ref, _ = synthetic.scene(20251015 + 1000 + sc, O=O, N=N, T=T)
            cells += [c for o in ovs for c in o]
            K.append([len(o) for o in ovs])
            refs.append(ref)
        store = engine.ParticleStore.from_cells(
            cells, device=dev, dtype=torch.float64 if dt == "f64" else torch.float32)
        cyc = cycle.MinkowskiCycle(store, [k for ks in K for k in ks], np.array(refs),
                                   scene_K=K)
        cyc.run()
        torch.cuda.synchronize()
        for k, v in (("mean", cyc.mean), ("cov", cyc.cov), ("rec", cyc.rec),
                     ("prob_lower", cyc.prob_lower)):
            res[f"{name}/{k}"] = v.cpu().numpy().copy()
        engine.moments(store, cyc.mean, cyc.cov, cyc.ws)
        torch.cuda.synchronize()
        res[f"{name}/mom_cov"] = cyc.cov.cpu().numpy().copy()
        print(f"{name}: {int(sum(store.counts))} particles, {store.n_cells} cells", flush=True)
        del store, cyc
        torch.cuda.empty_cache()
    np.savez(out, **res)


def main():
    if sys.argv[1] == "--dump":
        dump(sys.argv[2])
        return
    paths = []
    for v in sys.argv[1:3]:
        env = dict(os.environ)
        if v != "main":
            env["CCMPC_LIB"] = os.path.join(ROOT, "cc-mpc_amd", "csrc", v, "libccmpc.so")
        out = os.path.join(ROOT, "gpurun_out", f"bits_{v}.npz")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        print(f"== {v}", flush=True)
        subprocess.run([sys.executable, __file__, "--dump", out], env=env, check=True,
                       timeout=600)
        paths.append(out)
    a, b = np.load(paths[0]), np.load(paths[1])
    bad = 0
    for k in a.files:
        same = a[k].tobytes() == b[k].tobytes()
        bad += not same
        if not same:
            x, y = a[k], b[k]
            if k.endswith("/rec"):             # half-space records: decisions exact?  d, Q rel
                sys.path[:0] = [os.path.join(ROOT, "cc-mpc_amd")]
                from ccmpc import _lib
                x = x.reshape(-1, 128).view(_lib.HALFSPACE_DTYPE).reshape(-1)
                y = y.reshape(-1, 128).view(_lib.HALFSPACE_DTYPE).reshape(-1)
                dec = all(np.array_equal(x[f], y[f]) for f in ("which", "side", "status"))
                rel = max(float(np.max(np.abs(x[f] - y[f]) / (np.abs(x[f]) + 1e-300)))
                          for f in ("d", "q00", "q11", "r00", "r11"))
                print(f"DIFF {k}: which/side/status identical: {dec}; max rel d/Q/QR {rel:.2e}")
            else:
                rel = float(np.max(np.abs(x - y)) / max(np.max(np.abs(x)), 1e-300))
                print(f"DIFF {k}: {np.count_nonzero(x != y)} of {x.size} elements differ, "
                      f"max |diff| / max |a| = {rel:.2e}")
    print(f"{len(a.files) - bad} of {len(a.files)} arrays bit-identical")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
