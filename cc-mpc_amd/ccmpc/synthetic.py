"""Synthetic inputs shaped like the reference's planning step.

No datasets, weights or CARLA are available, so every benchmark input is synthetic and seeded:
* particle clouds: per (OV, mode) a shared heading/speed mode plus per-particle heading-rate and
  speed perturbations integrated over T steps of dt = 0.5 s (the structure of Trajectron++
  unicycle rollouts), around the Town03 scene-4 T-intersection (x ~ 180..200, y ~ -90..-70,
  v8ideal/__init__.py:836);
* mode split: a peaked latent pmf, modes with pmf > 0.1 kept (ovehicle.py:58);
* reference trajectory: ego ahead of the OVs, ref[t] = p_ego + (4 (t+1), 0.5 (t+1)), with the
  ego placed per seed (ego_offset), so every scene of a batch has its own ref_traj.
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


EGO = np.array([165.0, -60.0])


def ego_offset(seed):
    """Seed-dependent placement of a scene's ego (a separate Philox stream, so the OV clouds of a
    seed do not change with it): every scene of a batch has its own reference trajectory, and a
    batched cycle that read another scene's ref_traj would show in its records."""
    rng = np.random.default_rng(np.random.Philox(key=int(seed) ^ 0x5EED0E90))
    return rng.uniform(-4.0, 4.0, size=2)


def ego_ref(seed, T):
    """ref_traj[t] = p_ego + (4 (t+1), 0.5 (t+1)) for the seed's ego."""
    ego = EGO + ego_offset(seed)
    return np.array([ego + np.array([4.0 * (t + 1), 0.5 * (t + 1)]) for t in range(T)])


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
    ref = ego_ref(seed, T)
    return ovs, ref, np.array(pasts)


def crossing_scene(seed, O=2, N=400, T=8, K=2, lateral=8.0):
    """A planning step whose obstacles cross the ego's path, so half-spaces bind in the QP:
    the ego drives the reference trajectory of `scene` at ~8 m/s; each OV starts `lateral` m
    beside the reference point of a random step and heads across it, K modes per OV.
    Returns (cells: list of (N/K, T, 2) clouds in (OV, mode) order, K per OV, ref (T, 2),
    goal (2,), x_init [x, y, psi, v], pasts (O, 2))."""
    rng = np.random.default_rng(np.random.Philox(seed))
    ego = EGO + ego_offset(seed)               # the whole scene moves with its ego
    ref = np.array([ego + np.array([4.0 * (t + 1), 0.5 * (t + 1)]) for t in range(T)])
    goal = ref[-1] + np.array([4.0, 0.5])
    x_init = np.array([ego[0], ego[1], np.arctan2(0.5, 4.0), 8.0 + rng.uniform(-1, 1)])
    cells, Ks, pasts = [], [], []
    for _ in range(O):
        t0 = int(rng.integers(T // 3, T))
        side = 1.0 if rng.uniform() < 0.5 else -1.0
        p0 = ref[t0] + side * lateral * np.array([-0.124, 0.992]) + rng.normal(0, 1.0, 2)
        heading = np.arctan2(-side * 0.992, side * 0.124) + rng.normal(0, 0.4)
        for _k in range(K):
            n = int(N // K)
            h = heading + rng.normal(0, 0.3) + rng.normal(0, 0.1, size=(n, 1))
            v = np.maximum(1.0 + rng.uniform(0, 1.5) + rng.normal(0, 0.3, size=(n, 1)), 0.0)
            tt = np.arange(1, T + 1)[None, :] * DT
            hh = h + 0.05 * tt
            x = p0[0] + np.cumsum(v * np.cos(hh) * DT, axis=1) + rng.normal(0, 0.05, (n, T))
            y = p0[1] + np.cumsum(v * np.sin(hh) * DT, axis=1) + rng.normal(0, 0.05, (n, T))
            cells.append(np.stack((x, y), axis=-1))
        pasts.append(p0 - np.array([1.0, 0.2]))
        Ks.append(K)
    return cells, Ks, ref, goal, x_init, np.array(pasts)
