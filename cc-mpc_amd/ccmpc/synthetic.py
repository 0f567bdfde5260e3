"""Synthetic inputs shaped like the reference's planning step.

No datasets, weights or CARLA are available, so every benchmark input is synthetic and seeded:
* particle clouds: per (OV, mode) a shared heading/speed mode plus per-particle heading-rate and
  speed perturbations integrated over T steps of dt = 0.5 s (the structure of Trajectron++
  unicycle rollouts), around the Town03 scene-4 T-intersection (x ~ 180..200, y ~ -90..-70,
  v8ideal/__init__.py:836);
* mode split: a peaked latent pmf, modes with pmf > 0.1 kept (ovehicle.py:58);
* reference trajectory: ego ahead of the OVs, ref[t] = p_ego + (4 (t+1), 0.5 (t+1)).
"""
import numpy as np

DT = 0.5


def latent_pmf(rng, n_latent=25, sharp=2.5):
    logits = rng.normal(0.0, sharp, size=n_latent)
    p = np.exp(logits - logits.max())
    return p / p.sum()


def split_counts(rng, N, K):
    """N particles over K kept modes (multinomial, every mode >= 2 particles)."""
    w = rng.dirichlet(np.full(K, 4.0))
    c = np.maximum(np.round(w * N).astype(int), 2)
    c[-1] = max(N - c[:-1].sum(), 2)
    return c


def mode_cloud(rng, n, T, p0=None):
    """(n, T, 2) float64 world-frame trajectories of one (OV, mode) cell."""
    if p0 is None:
        p0 = np.array([rng.uniform(180, 200), rng.uniform(-90, -70)])
    heading = rng.uniform(-np.pi, np.pi)
    speed = rng.uniform(3.0, 10.0)
    dh = rng.normal(0, 0.15, size=(n, 1))
    dv = rng.normal(0, 1.0, size=(n, 1))
    t = np.arange(1, T + 1)[None, :] * DT
    h = heading + dh * t
    v = np.maximum(speed + dv * t, 0.0)
    x = p0[0] + np.cumsum(v * np.cos(h) * DT, axis=1) + rng.normal(0, 0.03, size=(n, T))
    y = p0[1] + np.cumsum(v * np.sin(h) * DT, axis=1) + rng.normal(0, 0.03, size=(n, T))
    return np.stack((x, y), axis=-1)


def scene(seed, O=4, N=5000, T=8, K=None):
    """One planning step: list over OVs of list over kept modes of (N_k, T, 2) clouds,
    plus ref_traj (T, 2) and each OV's past[-1]."""
    rng = np.random.default_rng(np.random.Philox(seed))
    ovs, pasts = [], []
    for _ in range(O):
        k = K if K is not None else int(rng.integers(1, 4))
        p0 = np.array([rng.uniform(180, 200), rng.uniform(-90, -70)])
        counts = split_counts(rng, N, k)
        ovs.append([mode_cloud(rng, int(c), T, p0) for c in counts])
        pasts.append(p0 - np.array([2.0, 0.5]))
    ego = np.array([165.0, -60.0])
    ref = np.array([ego + np.array([4.0 * (t + 1), 0.5 * (t + 1)]) for t in range(T)])
    return ovs, ref, np.array(pasts)
