"""Device-side building blocks over the C ABI: particle stores, moments, half-space kernels.

PyTorch is used only for device memory, streams and graphs; every numeric step is a HIP kernel
in libccmpc.so.  All functions enqueue on torch's current stream and never synchronise, so a
whole constraint-generation cycle can be captured into a hipGraph (torch.cuda.CUDAGraph).
"""
import ctypes

import numpy as np
import torch

from . import _lib

F64, F32 = _lib.CCMPC_F64, _lib.CCMPC_F32


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def require_device(device):
    device = torch.device(device)
    if device.type != "cuda":
        raise _lib.CcmpcError("ccmpc runs on the GPU only (no CPU fallback); got device "
                              f"{device}")
    if not torch.cuda.is_available():
        raise _lib.CcmpcError("no HIP device visible: the ccmpc path needs an MI355X")
    _lib.load()
    return device


def _round4(x):
    return (int(x) + 3) // 4 * 4


class ParticleStore:
    """Plane-major SoA particle clouds of several cells (see include/ccmpc.h).

    pos[(2t + c), off[j] + i] = coordinate c of particle i of cell j at step t.
    Cell offsets are 4-aligned and ld is a multiple of 4 (16-byte vector loads).
    F64 stores hold world coordinates; F32 stores hold coordinates relative to ``origin[j]``.
    """

    def __init__(self, T, counts, dtype=torch.float64, device="cuda", origin=None,
                 capacity=None):
        self.device = require_device(device)
        self.T = int(T)
        counts = [int(c) for c in counts]
        offs, cur = [], 0
        for c in counts:
            offs.append(cur)
            cur = _round4(cur + max(c, 0))
        self.n_bound = cur if capacity is None else max(cur, int(capacity))
        self.ld = max(_round4(self.n_bound), 4)
        self.dtype = dtype
        self.pos = torch.zeros((2 * self.T, self.ld), dtype=dtype, device=self.device)
        self.counts = counts
        self.cell_off = torch.tensor(offs, dtype=torch.int64, device=self.device)
        self.cell_cnt = torch.tensor(counts, dtype=torch.int64, device=self.device)
        self.offsets = offs
        if origin is None:
            self.origin = None
        else:
            self.origin = torch.as_tensor(np.asarray(origin, dtype=np.float64).reshape(-1, 2),
                                          device=self.device)

    @property
    def n_cells(self):
        return len(self.counts)

    @property
    def ccmpc_dtype(self):
        return F64 if self.dtype == torch.float64 else F32

    @classmethod
    def from_cells(cls, cells, device="cuda", dtype=torch.float64, origin=None):
        """cells: list of (N_j, T, 2) arrays (the reference's pred_positions[k] layout).
        For a float32 store, ``origin`` (n_cells, 2) is subtracted in float64 before the cast."""
        T = cells[0].shape[1]
        store = cls(T, [c.shape[0] for c in cells], dtype=dtype, device=device, origin=origin)
        host = np.zeros((2 * T, store.ld), dtype=np.float64 if dtype == torch.float64
                        else np.float32)
        for j, c in enumerate(cells):
            c = np.asarray(c, dtype=np.float64)
            if origin is not None:
                c = c - np.asarray(origin, dtype=np.float64).reshape(-1, 2)[j]
            n = c.shape[0]
            o = store.offsets[j]
            host[:, o:o + n] = c.transpose(1, 2, 0).reshape(2 * T, n)
        store.pos.copy_(torch.from_numpy(host))
        return store

    def cell_positions(self, j):
        """(N_j, T, 2) float64 host copy of one cell (world frame)."""
        n, o = self.counts[j], self.offsets[j]
        x = self.pos[:, o:o + n].double().cpu().numpy().reshape(self.T, 2, n).transpose(2, 0, 1)
        if self.origin is not None:
            x = x + self.origin[j].cpu().numpy()
        return x


class Workspace:
    """Grow-only device scratch buffer (pre-size it before graph capture)."""

    def __init__(self, device="cuda"):
        self.device = torch.device(device)
        self.buf = torch.empty(0, dtype=torch.uint8, device=self.device)

    def get(self, nbytes):
        nbytes = max(int(nbytes), 16)
        if self.buf.numel() < nbytes:
            self.buf = torch.empty(nbytes + 4096, dtype=torch.uint8, device=self.device)
        return self.buf


def moments(store, out_mean=None, out_cov=None, workspace=None):
    """Per-cell mean [C, T, 2] and covariance [C, 2T, 2T] (ddof = 1) of a ParticleStore."""
    lib = _lib.load()
    C, T = store.n_cells, store.T
    if out_mean is None:
        out_mean = torch.empty((C, T, 2), dtype=torch.float64, device=store.device)
    if out_cov is None:
        out_cov = torch.empty((C, 2 * T, 2 * T), dtype=torch.float64, device=store.device)
    need = lib.ccmpc_moments_workspace_bytes(T, C, store.n_bound)
    ws = (workspace or Workspace(store.device)).get(need)
    _lib.check(lib.ccmpc_moments(_p(store.pos), store.ccmpc_dtype, store.ld, T, _p(store.origin),
                                 _p(store.cell_off), _p(store.cell_cnt), C, store.n_bound,
                                 _p(ws), ws.numel(), _p(out_mean), _p(out_cov), _stream()),
               "ccmpc_moments")
    return out_mean, out_cov


def minkowski(mean, cov, ref_traj, cell_risk, cell_ref=None, R=3.4, tol=1e-8, maxiter=1000,
              out_rec=None, out_prob_lower=None):
    """Half-space records [C, T(T-1)/2] (raw bytes, see records.halfspaces) + prob_lower [C, T]."""
    lib = _lib.load()
    C, T = mean.shape[0], mean.shape[1]
    P = T * (T - 1) // 2
    if out_rec is None:
        out_rec = torch.empty((C, max(P, 1), 128), dtype=torch.uint8, device=mean.device)
    if out_prob_lower is None:
        out_prob_lower = torch.empty((C, T), dtype=torch.float64, device=mean.device)
    _lib.check(lib.ccmpc_minkowski(_p(mean), _p(cov), T, C, _p(ref_traj), _p(cell_ref),
                                   _p(cell_risk), float(R), float(tol), int(maxiter),
                                   _p(out_rec), _p(out_prob_lower), _stream()),
               "ccmpc_minkowski")
    return out_rec, out_prob_lower


def affine(mean, cov, ref_traj, cell_gamma, cell_ref=None, R=3.4, out_rec=None):
    lib = _lib.load()
    C, T = mean.shape[0], mean.shape[1]
    if out_rec is None:
        out_rec = torch.empty((C, T, 128), dtype=torch.uint8, device=mean.device)
    _lib.check(lib.ccmpc_affine(_p(mean), _p(cov), T, C, _p(ref_traj), _p(cell_ref),
                                _p(cell_gamma), float(R), _p(out_rec), _stream()),
               "ccmpc_affine")
    return out_rec


def ideal_rollout(prev_mean, prev_cov, src_cell, T, n_samples, x0=None, Z=None, seed=0,
                  rng_cell=None):
    """Materialised predict_ideal trajectories as an F64 ParticleStore + per-cell status."""
    lib = _lib.load()
    C = src_cell.shape[0]
    T_src = prev_mean.shape[1]
    store = ParticleStore(T, [n_samples] * C, dtype=torch.float64, device=prev_mean.device,
                          capacity=C * n_samples)
    status = torch.empty(C, dtype=torch.int32, device=prev_mean.device)
    _lib.check(lib.ccmpc_ideal_rollout(_p(prev_mean), _p(prev_cov), T_src, _p(src_cell), C, T,
                                       n_samples, _p(x0), _p(Z), int(seed) & (2**64 - 1),
                                       _p(rng_cell), _p(store.pos), store.ld, _p(status),
                                       _stream()),
               "ccmpc_ideal_rollout")
    return store, status


def ideal_moments(prev_mean, prev_cov, src_cell, T, n_samples, x0=None, seed=0, rng_cell=None,
                  workspace=None, out_mean=None, out_cov=None, out_status=None):
    """predict_ideal fused with the moment reduction: mean [C,T,2], cov [C,2T,2T], status [C]."""
    lib = _lib.load()
    C = src_cell.shape[0]
    T_src = prev_mean.shape[1]
    dev = prev_mean.device
    if out_mean is None:
        out_mean = torch.empty((C, T, 2), dtype=torch.float64, device=dev)
    if out_cov is None:
        out_cov = torch.empty((C, 2 * T, 2 * T), dtype=torch.float64, device=dev)
    if out_status is None:
        out_status = torch.empty(C, dtype=torch.int32, device=dev)
    need = lib.ccmpc_ideal_moments_workspace_bytes(T, C, n_samples)
    ws = (workspace or Workspace(dev)).get(need)
    _lib.check(lib.ccmpc_ideal_moments(_p(prev_mean), _p(prev_cov), T_src, _p(src_cell), C, T,
                                       n_samples, _p(x0), int(seed) & (2**64 - 1), _p(rng_cell),
                                       _p(ws), ws.numel(), _p(out_mean), _p(out_cov),
                                       _p(out_status), _stream()),
               "ccmpc_ideal_moments")
    return out_mean, out_cov, out_status


def halfspaces(rec_bytes):
    """Device record bytes -> numpy structured array (HALFSPACE_DTYPE); synchronises."""
    return rec_bytes.cpu().numpy().reshape(-1).view(_lib.HALFSPACE_DTYPE).reshape(
        rec_bytes.shape[:-1])


def affine_records(rec_bytes):
    return rec_bytes.cpu().numpy().reshape(-1).view(_lib.AFFINE_DTYPE).reshape(
        rec_bytes.shape[:-1])
