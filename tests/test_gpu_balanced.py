"""Balanced mode of the particle-store kernels (n_particles_bound > 2^18, cells <= grid / 2):
the grid is the device's resident capacity and the chunk is searched on the device from the
cell counts (gram.hpp, locate_balanced).  Parity against np.mean / np.cov (ddof=1) on ragged
cells -- an empty cell, cells smaller than one 16-particle line, cells spanning dozens of
chunks -- and consistency with the power-of-two path and with the fused cycle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

COUNTS = [0, 3, 17, 1994, 40_000, 123_457, 250_000, 5, 2_051]   # 417,527 particles > 2^18


def _cells(T, counts, seed):
    rng = np.random.default_rng(seed)
    return [190 + np.cumsum(rng.normal(0, 0.5, size=(n, T, 2)), axis=1) for n in counts]


def _numpy_moments(cell):
    N, T, _ = cell.shape
    X = cell.transpose(1, 2, 0).reshape(2 * T, N)
    return X.mean(axis=1), np.cov(X)


def _fro_rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


# T = 28 / 40: 16x16 tiles with RB = 4 / 5, whose cells of 2..kRootFanIn items take the
# deferred root (root_finalize_kernel) and larger ones the combine tree
@pytest.mark.parametrize("T,dtype", [(8, torch.float64), (11, torch.float64),
                                     (20, torch.float64), (11, torch.float32),
                                     (28, torch.float64), (40, torch.float64),
                                     (40, torch.float32)])
def test_balanced_moments_match_numpy(gpu, T, dtype):
    import ccmpc.engine as eng
    cells = _cells(T, COUNTS, seed=T)
    origin = np.array([[190.0, 190.0]] * len(cells)) if dtype == torch.float32 else None
    store = eng.ParticleStore.from_cells(cells, device=gpu, dtype=dtype, origin=origin)
    assert store.n_bound > 2 ** 18
    mean, cov = eng.moments(store)
    mean, cov = mean.cpu().numpy(), cov.cpu().numpy()
    for j, c in enumerate(cells):
        if c.shape[0] == 0:
            assert np.all(np.isnan(mean[j])) and np.all(np.isnan(cov[j]))
            continue
        if dtype == torch.float32:       # the reference sees the float32-rounded positions
            c = (c - 190.0).astype(np.float32).astype(np.float64) + 190.0
        m_ref, c_ref = _numpy_moments(c)
        np.testing.assert_allclose(mean[j].reshape(-1), m_ref, rtol=1e-13)
        if c.shape[0] > 1:
            assert _fro_rel(cov[j], c_ref) < 1e-11, (j, c.shape[0])
        np.testing.assert_array_equal(cov[j], cov[j].T)


@pytest.mark.parametrize("T", [8, 12, 40])
def test_balanced_equals_power_of_two_items(gpu, T):
    """The same cells through both paths: the capacity alone moves the launch into balanced
    mode (the chunk is computed from the actual counts, not from the bound)."""
    import ccmpc.engine as eng
    cells = _cells(T, [3000, 7, 20_000, 0, 9_999], seed=100 + T)
    small = eng.ParticleStore.from_cells(cells, device=gpu)
    big = eng.ParticleStore.from_cells(cells, device=gpu, capacity=2 ** 20)
    assert small.n_bound <= 2 ** 18 < big.n_bound
    m1, c1 = eng.moments(small)
    m2, c2 = eng.moments(big)
    torch.testing.assert_close(m2, m1, rtol=1e-13, atol=0, equal_nan=True)
    torch.testing.assert_close(c2, c1, rtol=1e-10, atol=1e-12, equal_nan=True)


@pytest.mark.parametrize("T", [8, 12])
def test_balanced_cycle_fused_equals_two_calls(gpu, T):
    from ccmpc import cycle, synthetic
    ovs, ref, _ = synthetic.scene(11, O=4, N=80_000, T=T)
    import ccmpc.engine as eng
    store = eng.ParticleStore.from_cells([c for o in ovs for c in o], device=gpu)
    assert store.n_bound > 2 ** 18
    cyc = cycle.MinkowskiCycle(store, [len(o) for o in ovs], ref)
    cyc.run_unfused()
    a = (cyc.mean.clone(), cyc.cov.clone(), cyc.rec.clone(), cyc.prob_lower.clone())
    for _ in range(3):                     # counters must come back to zero every launch
        cyc.rec.zero_()
        cyc.run()
    assert torch.equal(a[0], cyc.mean) and torch.equal(a[1], cyc.cov)
    assert torch.equal(a[2], cyc.rec) and torch.equal(a[3], cyc.prob_lower)
    assert np.all(cyc.records()["status"] == 0)
