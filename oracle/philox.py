"""Philox4x32-10 counter RNG and the Box-Muller normals the HIP kernels draw.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): this is the CPU checker's copy of
the counter-based generator in ``cc-mpc_amd/csrc/ccmpc_rng.hpp``.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.

The reference draws its randomness from unseeded generators
(``v8ideal/__init__.py:2664`` ``np.random.multivariate_normal``, ``:2699-2700``
``RandomState(None).standard_normal``, and the Trajectron++ sampler), so its draws cannot be
reproduced.  Parity is pinned by making every draw a pure function of a counter:

    key     = (seed & 0xffffffff, seed >> 32)
    counter = (c0, c1, c2, c3)          # meaning fixed per stream, see STREAM_* below

Two 32-bit words make one 53-bit uniform; two uniforms make one Box-Muller pair.
"""
import numpy as np

_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = np.uint64(0x9E3779B9)
_W1 = np.uint64(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)
_S32 = np.uint64(32)

# Stream tags (counter word c3).  Must match ccmpc_rng.hpp.
STREAM_IDEAL_Z = 0x1DEA0001      # predict_ideal step noise Z (v8ideal/__init__.py:2700)
STREAM_IDEAL_X0 = 0x1DEA0002     # predict_ideal shared initial draw (v8ideal/__init__.py:2664)
STREAM_SAMPLER_EPS = 0x5A4D0001  # GMM2D action noise (Trajectron++ GMM2D.rsample)
STREAM_SAMPLER_Z = 0x5A4D0002    # latent z draw (Trajectron++ DiscreteLatent.sample_p)


def philox4x32(c0, c1, c2, c3, seed):
    """Vectorised Philox4x32-10.  c* broadcastable uint32 arrays; returns 4 uint32 arrays."""
    c0 = np.asarray(c0, dtype=np.uint64) & _MASK
    c1 = np.asarray(c1, dtype=np.uint64) & _MASK
    c2 = np.asarray(c2, dtype=np.uint64) & _MASK
    c3 = np.asarray(c3, dtype=np.uint64) & _MASK
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = np.uint64(int(seed) & 0xFFFFFFFF)
    k1 = np.uint64((int(seed) >> 32) & 0xFFFFFFFF)
    for rnd in range(10):
        p0 = _M0 * c0
        p1 = _M1 * c2
        hi0, lo0 = p0 >> _S32, p0 & _MASK
        hi1, lo1 = p1 >> _S32, p1 & _MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0), lo1, (hi0 ^ c3 ^ k1), lo0
        if rnd != 9:
            k0 = (k0 + _W0) & _MASK
            k1 = (k1 + _W1) & _MASK
    return (c0.astype(np.uint32), c1.astype(np.uint32),
            c2.astype(np.uint32), c3.astype(np.uint32))


def uniform53(a, b):
    """Two uint32 words -> float64 in [0, 1) with 53 random bits."""
    a = np.asarray(a, dtype=np.uint64) >> np.uint64(5)
    b = np.asarray(b, dtype=np.uint64) >> np.uint64(6)
    return (a.astype(np.float64) * 67108864.0 + b.astype(np.float64)) * (1.0 / 9007199254740992.0)


def normal_pair(c0, c1, c2, c3, seed):
    """One Box-Muller pair (z0, z1) per counter, float64."""
    w0, w1, w2, w3 = philox4x32(c0, c1, c2, c3, seed)
    u1 = 1.0 - uniform53(w0, w1)          # (0, 1]
    u2 = uniform53(w2, w3)                # [0, 1)
    r = np.sqrt(-2.0 * np.log(u1))
    ang = 2.0 * np.pi * u2
    return r * np.cos(ang), r * np.sin(ang)


def uniform_single(c0, c1, c2, c3, seed):
    """One float64 uniform in [0, 1) per counter (first two words)."""
    w0, w1, _, _ = philox4x32(c0, c1, c2, c3, seed)
    return uniform53(w0, w1)
