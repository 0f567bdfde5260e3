"""Compare ccmpc_sample_bucket with sampler + ccmpc_bucket cell by cell (diagnostic)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from test_gpu_sample_bucket import _inputs  # noqa: E402
from ccmpc import engine as e  # noqa: E402

gpu = torch.device("cuda", 0)
def heavy(O, L, T, seed, hot):
    init, pmf, gmm = _inputs(O, L, T, seed)
    pmf[:] = 0.85 / (L - 1)
    pmf[:, 3] = 0.15 if hot else 0.05
    pmf /= pmf.sum(1, keepdims=True)
    return init, pmf, gmm


for (O, L, T, N, seed, kept) in [(1, 25, 8, 3000, 1, "h"), (1, 25, 8, 4000, 1, "h"), (1, 25, 8, 5000, 1, "h"),
                                 (1, 25, 8, 8192, 1, "h"), (1, 25, 1, 5000, 1, "h"), (1, 25, 8, 600, 1, "h")]:
    init, pmf, gmm = heavy(O, L, T, seed, True) if kept == "h" else _inputs(O, L, T, seed, kept)
    minpos = np.tile([150.0, -120.0], (O, 1))
    z, st = e.sample_unicycle(init, pmf, gmm, N, T, seed=seed, device=gpu)
    b, K, pw, cw = e.bucket(z, st, pmf, minpos)
    zf, f, Kf, pf, cf = e.sample_bucket(init, pmf, gmm, N, T, minpos, seed=seed, device=gpu, with_z=True)
    zz = z.cpu().numpy()
    print("shape", (O, L, T, N), "K", K, "z equal", np.array_equal(zz, zf.cpu().numpy()))
    kept_m = pmf > 0.1
    for o in range(O):
        rare = ~kept_m[o][zz[o]]
        print(f"  ov {o}: R {rare.sum()} natives {[int((zz[o] == l).sum()) for l in np.flatnonzero(kept_m[o])]}")
    print("  cnt two-step", b.sync_counts(), "off", b.offsets)
    print("  cnt fused   ", f.sync_counts(), "off", f.offsets)
    print("  pmf eq", np.array_equal(pw.cpu().numpy(), pf.cpu().numpy()), "centre eq",
          np.array_equal(cw.cpu().numpy(), cf.cpu().numpy()), cw.cpu().numpy()[:2], cf.cpu().numpy()[:2])
