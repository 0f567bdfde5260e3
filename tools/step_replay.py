"""Replay one planning-step graph many times (GPU box), for rocprofv3 passes over the step's
kernels (profiles/collect_configs.sh STEP configs):

    python tools/step_replay.py CFG ITERS

CFG:
  step_c2            C2 shape (4 OVs x 5000, ph 8), the synthetic sampler route
  step_c1_100k       C1's 100 000 particles (1 OV), the synthetic sampler route
  step_pred_c2       C2 shape on generate_vehicle_latents' 5-tuple, host arrays (pinned pack)
  step_pred_dev_c2   the same as device tensors (keep_on_device)
  step_pred_dev_100k C1's 100 000 on device tensors
Each iteration is MidlevelAgent.predict_and_constrain (graph replay + wait + 9-tuple); the
graph is captured during the warm-up, so the profile holds only replays.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cc-mpc_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

CFGS = {
    "step_c2": dict(O=4, N=5000, src="sampler"),
    "step_c1_100k": dict(O=1, N=100_000, src="sampler"),
    "step_pred_c2": dict(O=4, N=5000, src="pred_host"),
    "step_pred_dev_c2": dict(O=4, N=5000, src="pred_dev"),
    "step_pred_dev_100k": dict(O=1, N=100_000, src="pred_dev"),
}


def main():
    cfg, iters = sys.argv[1], int(sys.argv[2])
    c = CFGS[cfg]
    from ccmpc import engine, episode, planner
    dev = torch.device("cuda", 0)
    O, N, ph = c["O"], c["N"], 8
    init, pmf, gmm = episode.synthetic_gmm(O, T=ph, seed=20251015)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]]) for o in range(O)]
    K = [int(np.count_nonzero(pmf[o] > 0.1)) for o in range(O)]
    eps = np.full((O, max(K)), 0.05 / O)
    ego = np.array([165.0, -72.0])
    ref = np.array([ego + [4.0 * (t + 1), 0.5 * (t + 1)] for t in range(ph)])
    agent = planner.MidlevelAgent(prediction_horizon=ph, device=dev)
    params = episode.Params(O, K, 0)
    sets = []
    if c["src"] != "sampler":
        for k in range(2):
            z, store = engine.sample_unicycle(init, pmf, gmm, N, ph, seed=900 + k, device=dev)
            pos = store.pos.cpu().numpy()
            pred = np.zeros((O + 1, N, ph, 2), np.float32)
            for o in range(O):
                off = store.offsets[o]
                pred[o + 1] = pos[:, off:off + N].reshape(ph, 2, N).transpose(2, 0, 1)
            zz = np.zeros((O + 1, N), np.int64)
            zz[1:] = z.cpu().numpy()
            if c["src"] == "pred_dev":
                pred, zz = torch.as_tensor(pred, device=dev), torch.as_tensor(zz, device=dev)
            sets.append(dict(source="predictions", predictions=pred, z=zz,
                             rows=list(range(1, O + 1)), latent_pmf=pmf, N=N))

    def one(i):
        s = sets[i % 2] if sets else dict(init_state=init, latent_pmf=pmf, gmm=gmm, N=N, seed=i)
        agent.predict_and_constrain(params, s, eps, ph, ref, minpos, pasts)
    for i in range(10):
        one(i)
    torch.cuda.synchronize()
    for i in range(iters):
        one(i)
    torch.cuda.synchronize()
    print(f"{cfg}: {iters} steps")


if __name__ == "__main__":
    main()
