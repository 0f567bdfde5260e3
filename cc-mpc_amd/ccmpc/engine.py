"""Device-side building blocks over the C ABI: particle stores, moments, half-space kernels.

PyTorch is used only for device memory, streams and graphs; every numeric step is a HIP kernel
in libccmpc.so.  All functions enqueue on torch's current stream and never synchronise, so a
whole constraint-generation cycle can be captured into a hipGraph (torch.cuda.CUDAGraph).
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib

F64, F32 = _lib.CCMPC_F64, _lib.CCMPC_F32


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(device_index=None):
    """torch's current stream on the current (or given) device as a raw handle.  The raw
    getter skips building a torch.cuda.Stream object (~2 us of host time per call, and the
    planning step makes several)."""
    if _raw_stream is not None:
        idx = torch.cuda.current_device() if device_index is None else device_index
        return ctypes.c_void_p(_raw_stream(idx))
    s = torch.cuda.current_stream() if device_index is None else torch.cuda.current_stream(
        device_index)
    return ctypes.c_void_p(s.cuda_stream)


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


# Cell offsets and ld of the stores built here, in particles: a multiple of 4 is what the
# kernels need (16-byte vector loads); 32 puts every load group of a cell on whole 128-byte
# lines (a 16-particle f64 step, a 32-particle Scheme4 / f32 step), so the waves that stream
# neighbouring groups never share a line.  Measured against 4 (profiles/r03/ab3_store_align32.log):
# C5 85.9 -> 81.1 us cold, the per-GPU C4 batch 37.4 -> 36.0 us cold, C2 / C3 unchanged.
# CCMPC_STORE_ALIGN overrides it (A/B).
STORE_ALIGN = int(os.environ.get("CCMPC_STORE_ALIGN", "32"))


def _round_to(x, a):
    return (int(x) + a - 1) // a * a


class ParticleStore:
    """Plane-major SoA particle clouds of several cells (see include/ccmpc.h).

    pos[(2t + c), off[j] + i] = coordinate c of particle i of cell j at step t.
    Cell offsets and ld are multiples of `align` particles (STORE_ALIGN = 32 by default; the
    kernels need a multiple of 4: 16-byte vector loads).
    F64 stores hold world coordinates; F32 stores hold coordinates relative to ``origin[j]``.
    """

    def __init__(self, T, counts, dtype=torch.float64, device="cuda", origin=None,
                 capacity=None, align=None):
        self.device = require_device(device)
        self.T = int(T)
        counts = [int(c) for c in counts]
        al = STORE_ALIGN if align is None else int(align)
        if al < 4 or al % 4:
            raise ValueError("store alignment must be a multiple of 4 particles")
        offs, cur = [], 0
        for c in counts:
            offs.append(cur)
            cur = _round_to(cur + max(c, 0), al)
        self.n_bound = cur if capacity is None else max(cur, int(capacity))
        self.ld = max(_round_to(self.n_bound, al), al)
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
        return int(self.cell_cnt.shape[0])

    @property
    def ccmpc_dtype(self):
        return F64 if self.dtype == torch.float64 else F32

    @classmethod
    def from_cells(cls, cells, device="cuda", dtype=torch.float64, origin=None, capacity=None):
        """cells: list of (N_j, T, 2) arrays (the reference's pred_positions[k] layout).
        For a float32 store, ``origin`` (n_cells, 2) is subtracted in float64 before the cast.
        ``capacity`` raises the particle bound the kernels are sized for (n_particles_bound)."""
        T = cells[0].shape[1]
        store = cls(T, [c.shape[0] for c in cells], dtype=dtype, device=device, origin=origin,
                    capacity=capacity)
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

    def sync_counts(self):
        """Fetch device-side cell offsets/counts (after ccmpc_bucket); synchronises."""
        self.counts = [int(c) for c in self.cell_cnt.cpu().tolist()]
        self.offsets = [int(c) for c in self.cell_off.cpu().tolist()]
        return self.counts

    def cell_positions(self, j):
        """(N_j, T, 2) float64 host copy of one cell (world frame)."""
        if self.counts is None:
            self.sync_counts()
        n, o = self.counts[j], self.offsets[j]
        x = self.pos[:, o:o + n].double().cpu().numpy().reshape(self.T, 2, n).transpose(2, 0, 1)
        if self.origin is not None:
            x = x + self.origin[j].cpu().numpy()
        return x


class Workspace:
    """Grow-only device scratch buffer (pre-size it before graph capture).

    Allocated zero-filled: its head holds the per-cell arrival counters of the one-launch
    reductions, which must start at zero and which every call leaves at zero (ccmpc.h).
    One Workspace per stream."""

    def __init__(self, device="cuda"):
        self.device = torch.device(device)
        self.buf = torch.zeros(0, dtype=torch.uint8, device=self.device)

    def get(self, nbytes):
        nbytes = max(int(nbytes), 16)
        if self.buf.numel() < nbytes:
            self.buf = torch.zeros(nbytes + 4096, dtype=torch.uint8, device=self.device)
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


def minkowski_cycle(store, ref_traj, cell_risk, cell_ref=None, R=3.4, tol=1e-8, maxiter=1000,
                    workspace=None, out_mean=None, out_cov=None, out_rec=None,
                    out_prob_lower=None):
    """moments + Minkowski half-spaces in ONE launch (ccmpc_minkowski_cycle)."""
    lib = _lib.load()
    C, T = store.n_cells, store.T
    dev = store.device
    P = max(T * (T - 1) // 2, 1)
    out_mean = out_mean if out_mean is not None else torch.empty((C, T, 2), dtype=torch.float64,
                                                                 device=dev)
    out_cov = out_cov if out_cov is not None else torch.empty((C, 2 * T, 2 * T),
                                                              dtype=torch.float64, device=dev)
    out_rec = out_rec if out_rec is not None else torch.empty((C, P, 128), dtype=torch.uint8,
                                                              device=dev)
    out_prob_lower = (out_prob_lower if out_prob_lower is not None
                      else torch.empty((C, T), dtype=torch.float64, device=dev))
    need = lib.ccmpc_moments_workspace_bytes(T, C, store.n_bound)
    ws = (workspace or Workspace(dev)).get(need)
    _lib.check(lib.ccmpc_minkowski_cycle(
        _p(store.pos), store.ccmpc_dtype, store.ld, T, _p(store.origin), _p(store.cell_off),
        _p(store.cell_cnt), C, store.n_bound, _p(ws), ws.numel(), _p(ref_traj), _p(cell_ref),
        _p(cell_risk), float(R), float(tol), int(maxiter), _p(out_mean), _p(out_cov),
        _p(out_rec), _p(out_prob_lower), _stream()), "ccmpc_minkowski_cycle")
    return out_mean, out_cov, out_rec, out_prob_lower


def ideal_minkowski_cycle(prev_mean, prev_cov, src_cell, T, n_samples, ref_traj, cell_risk,
                          x0=None, seed=0, rng_cell=None, cell_ref=None, R=3.4, tol=1e-8,
                          maxiter=1000, workspace=None):
    """Shrinking-horizon step in one launch: predict_ideal -> moments -> half-spaces."""
    lib = _lib.load()
    C = src_cell.shape[0]
    T_src = prev_mean.shape[1]
    dev = prev_mean.device
    P = max(T * (T - 1) // 2, 1)
    out_mean = torch.empty((C, T, 2), dtype=torch.float64, device=dev)
    out_cov = torch.empty((C, 2 * T, 2 * T), dtype=torch.float64, device=dev)
    status = torch.empty(C, dtype=torch.int32, device=dev)
    rec = torch.empty((C, P, 128), dtype=torch.uint8, device=dev)
    pl = torch.empty((C, T), dtype=torch.float64, device=dev)
    need = lib.ccmpc_ideal_moments_workspace_bytes(T, C, n_samples)
    ws = (workspace or Workspace(dev)).get(need)
    _lib.check(lib.ccmpc_ideal_minkowski_cycle(
        _p(prev_mean), _p(prev_cov), T_src, _p(src_cell), C, T, n_samples, _p(x0),
        int(seed) & (2**64 - 1), _p(rng_cell), _p(ws), ws.numel(), _p(ref_traj), _p(cell_ref),
        _p(cell_risk), float(R), float(tol), int(maxiter), _p(out_mean), _p(out_cov), _p(status),
        _p(rec), _p(pl), _stream()), "ccmpc_ideal_minkowski_cycle")
    return out_mean, out_cov, status, rec, pl


# L4 in one workgroup per (cell, t) (ccmpc_l4, one launch) while the average cell holds at most
# this many particles; the split form (ccmpc_l4_split, two launches) above it.  The two sum the
# headings in different orders (same result to rounding), so the step graph and the eager calls
# choose by this one rule.
_L4_ONE_WG_MAX = int(os.environ.get("CCMPC_L4_ONE_WG_MAX", "8192"))


def l4_one_workgroup(n_cells, n_bound):
    return n_bound <= _L4_ONE_WG_MAX * max(int(n_cells), 1)


def l4(store, past_last, bbox, with_yaw=False, with_vertices=False, split=None,
       workspace=None):
    """Headings, L4 outer approximation and t=0 yaw stats per (cell, t): ccmpc_l4_split (every
    (cell, t) over several workgroups, two launches) or, split=False, ccmpc_l4 (one workgroup
    per (cell, t)); split=None chooses by l4_one_workgroup.  Returns dict(A [C,T,4,2], b [C,T,4],
    yaw_mean [C,T], yaw0_var [C], yaw?, vertices?)."""
    lib = _lib.load()
    C, T, dev = store.n_cells, store.T, store.device
    if split is None:
        split = not l4_one_workgroup(C, store.n_bound)
    out = dict(A=torch.empty((C, T, 4, 2), dtype=torch.float64, device=dev),
               b=torch.empty((C, T, 4), dtype=torch.float64, device=dev),
               yaw_mean=torch.empty((C, T), dtype=torch.float64, device=dev),
               yaw0_var=torch.empty((C,), dtype=torch.float64, device=dev))
    out["yaw"] = (torch.empty((T, store.ld), dtype=torch.float64, device=dev) if with_yaw
                  else None)
    out["vertices"] = (torch.empty((T * 8, store.ld), dtype=torch.float64, device=dev)
                       if with_vertices else None)
    # both small host inputs in one host-to-device copy
    pb = torch.as_tensor(np.stack([np.asarray(past_last, np.float64).reshape(C, 2),
                                   np.asarray(bbox, np.float64).reshape(C, 2)]), device=dev)
    past_last, bbox = pb[0], pb[1]
    if split:
        need = lib.ccmpc_l4_workspace_bytes(T, C, store.n_bound)
        ws = (workspace or Workspace(dev)).get(need)
        _lib.check(lib.ccmpc_l4_split(
            _p(store.pos), store.ccmpc_dtype, store.ld, T, _p(store.origin), _p(store.cell_off),
            _p(store.cell_cnt), C, store.n_bound, _p(past_last), _p(bbox), _p(ws), ws.numel(),
            _p(out["A"]), _p(out["b"]), _p(out["yaw_mean"]), _p(out["yaw0_var"]),
            _p(out["yaw"]), _p(out["vertices"]), _stream()), "ccmpc_l4_split")
        out["_keepalive"] = (past_last, bbox, ws)
        return out
    _lib.check(lib.ccmpc_l4(_p(store.pos), store.ccmpc_dtype, store.ld, T, _p(store.origin),
                            _p(store.cell_off), _p(store.cell_cnt), C, _p(past_last), _p(bbox),
                            _p(out["A"]), _p(out["b"]), _p(out["yaw_mean"]), _p(out["yaw0_var"]),
                            _p(out["yaw"]), _p(out["vertices"]), _stream()), "ccmpc_l4")
    out["_keepalive"] = (past_last, bbox)
    return out


def sample_unicycle(init_state, latent_pmf, gmm, N, T, dt=0.5, seed=0, device="cuda", ov_base=0,
                    z=None, eps=None, per_particle=False):
    """GMM-latent particle sampler (ccmpc_sample_unicycle_ex).

    init_state (O, 4); latent_pmf (O, L) p(z|x) (only used when z is drawn here; may be None
    when z is given).  gmm: per (OV, latent, step) parameters (O, L, T, 5), or with
    per_particle=True every sample's own parameters as p_y_xz's autoregressive decoder emits
    them, (O, N, T, 5) -- host array or device tensor; (O, T, 5, N) device layout is built here.
    z: injected latent ids (O, N) (torch's one-hot z argmax, prediction.py:103) or None for the
    Philox draw; eps: injected standard-normal noise (O, N, T, 2) float32 or None for Philox.
    ov_base = global id of the first OV (keys the Philox streams; see ccmpc.dist).
    Returns (z [O,N] int32, F32 ParticleStore in sample order: one cell per OV)."""
    lib = _lib.load()
    dev = require_device(device)
    O, L, t_init, t_cdf, t_gmm, layout, t_z, t_eps = _sampler_inputs(
        init_state, latent_pmf, gmm, N, T, dev, z, eps, per_particle)
    # the sampler writes OV o at o * round4(N): the kernel's own layout (align 4)
    store = ParticleStore(T, [N] * O, dtype=torch.float32, device=dev, origin=np.zeros((O, 2)),
                          align=4)
    out_z = torch.empty((O, N), dtype=torch.int32, device=dev)
    _lib.check(lib.ccmpc_sample_unicycle_ex(
        _p(t_init), _p(t_cdf), L, _p(t_gmm), layout, _p(t_z), _p(t_eps), O, N, T, float(dt),
        int(seed) & (2**64 - 1), None, int(ov_base), _p(out_z), _p(store.pos), store.ld,
        _stream()),
        "ccmpc_sample_unicycle_ex")
    store._keepalive = (t_init, t_cdf, t_gmm, t_z, t_eps)
    return out_z, store


def load_predictions(predictions, z, n_latent, rows=None, device="cuda"):
    """generate_vehicle_latents' predictions (nodes, N, T, 2) float32 scene-relative and z
    (nodes, N) int64 / int32 (prediction.py:93-105; host arrays or device tensors) -> the
    sample-order F32 store + int32 z that ccmpc_bucket reads (ccmpc_load_predictions), OV o
    = node rows[o] (default: every node).  Returns (z [O, N] int32, ParticleStore)."""
    lib = _lib.load()
    dev = require_device(device)
    pred = torch.as_tensor(predictions, device=dev)
    if pred.dtype != torch.float32 or pred.dim() != 4 or pred.shape[3] != 2:
        raise ValueError("predictions must be (nodes, N, T, 2) float32")
    pred = pred.contiguous()
    zt = torch.as_tensor(z, device=dev).contiguous()
    if zt.dtype not in (torch.int64, torch.int32) or tuple(zt.shape) != tuple(pred.shape[:2]):
        raise ValueError("z must be (nodes, N) int64 or int32")
    n_nodes, N, T = int(pred.shape[0]), int(pred.shape[1]), int(pred.shape[2])
    rows = list(range(n_nodes)) if rows is None else [int(r) for r in rows]
    if any(r < 0 or r >= n_nodes for r in rows):
        raise ValueError(f"rows outside [0, {n_nodes})")
    O = len(rows)
    t_rows = torch.as_tensor(np.asarray(rows, np.int32), device=dev)
    store = ParticleStore(T, [N] * O, dtype=torch.float32, device=dev, origin=np.zeros((O, 2)),
                          align=4)
    out_z = torch.empty((O, N), dtype=torch.int32, device=dev)
    stride = store.offsets[1] if O > 1 else N
    z_bad = torch.zeros(O, dtype=torch.int32, device=dev)
    _lib.check(lib.ccmpc_load_predictions(
        _p(pred), _p(zt), zt.element_size(), _p(t_rows), O, N, T, int(n_latent), _p(store.pos),
        store.ld, stride, _p(out_z), _p(z_bad), _stream()), "ccmpc_load_predictions")
    raise_bad_latents(z_bad.cpu().numpy(), n_latent)
    store._keepalive = (pred, zt, t_rows)
    return out_z, store


def raise_bad_latents(z_bad, n_latent):
    """IndexError where make_ovehicles' `veh_latent_predictions[zn[jdx]]` (v8ideal/__init__.py:
    488-491, a list of n_latent entries) raises it: z_bad[o] = OV o's ids outside
    [-n_latent, n_latent), counted on the device."""
    bad = [int(b) for b in np.asarray(z_bad).reshape(-1)]
    if any(bad):
        o = next(j for j, b in enumerate(bad) if b)
        raise IndexError(f"list index out of range: {bad[o]} latent id(s) of OV {o} outside "
                         f"[-{n_latent}, {n_latent}) (make_ovehicles' per-latent list)")


def _sampler_inputs(init_state, latent_pmf, gmm, N, T, dev, z, eps, per_particle):
    """Device copies of a sampler call's inputs (ccmpc_sample_unicycle_ex's layouts)."""
    init_state = np.asarray(init_state, np.float64).reshape(-1, 4)
    O = init_state.shape[0]
    t_z = t_eps = t_cdf = None
    if z is not None:
        t_z = torch.as_tensor(z, device=dev).to(torch.int32).reshape(O, N).contiguous()
    if latent_pmf is not None:
        pmf = np.asarray(latent_pmf, np.float64).reshape(O, -1)
        L = pmf.shape[1]
        t_cdf = torch.as_tensor(np.cumsum(pmf, axis=1), device=dev)
    elif t_z is not None:
        # the latent count: the per-latent table's, else any id below 64 (the kernel's bound)
        L = (int(gmm.shape[1]) if hasattr(gmm, "shape") else len(gmm[0])) if not per_particle else 64
    else:
        raise ValueError("latent_pmf is needed when z is drawn by the sampler")
    if t_z is not None and t_z.numel():
        lo, hi = int(t_z.min().item()), int(t_z.max().item())
        if lo < 0 or hi >= L:
            raise ValueError(f"injected z outside [0, {L}): [{lo}, {hi}]")
    if per_particle:
        if t_z is None:
            raise ValueError("per-particle GMM parameters need the injected z")
        g = torch.as_tensor(gmm, device=dev).to(torch.float32).reshape(O, N, T, 5)
        t_gmm = g.permute(0, 2, 3, 1).contiguous()           # (O, T, 5, N): particle-minor
        layout = _lib.GMM_PER_PARTICLE
    else:
        t_gmm = torch.as_tensor(np.ascontiguousarray(np.asarray(
            gmm.cpu() if torch.is_tensor(gmm) else gmm, np.float32).reshape(O, L, T, 5)),
            device=dev)
        layout = _lib.GMM_PER_LATENT
    if eps is not None:
        e = torch.as_tensor(eps, device=dev).to(torch.float32).reshape(O, N, T, 2)
        t_eps = e.permute(0, 2, 3, 1).contiguous()           # (O, T, 2, N)
    t_init = torch.as_tensor(init_state, device=dev)
    return O, L, t_init, t_cdf, t_gmm, layout, t_z, t_eps


def _bucket_plan(pmf, filter_pmf, max_k):
    """Kept modes of every OV (p(z|x) > filter, host data as in prediction.py:77-79): K per
    OV, max_k, keep_map [O, L] (kept index or -1), cell_base [O]."""
    O, L = pmf.shape
    keep = [np.argwhere(pmf[o] > filter_pmf).ravel() for o in range(O)]
    K = [int(k.size) for k in keep]
    if min(K) == 0:
        raise ValueError("attempt to get argmin of an empty sequence: an OV has no latent mode "
                         f"with p(z|x) > {filter_pmf} (ovehicle.py:96-97 fails the same way)")
    max_k = max(K) if max_k is None else max_k
    keep_map = -np.ones((O, L), np.int32)
    for o in range(O):
        keep_map[o, keep[o]] = np.arange(K[o], dtype=np.int32)
    cell_base = np.concatenate([[0], np.cumsum(K)[:-1]]).astype(np.int32)
    return K, max_k, keep_map, cell_base


FUSED_MAX_N = 1 << 18          # ccmpc_sample_bucket / ccmpc_bucket_predictions


def sample_bucket(init_state, latent_pmf, gmm, N, T, minpos, dt=0.5, seed=0, device="cuda",
                  ov_base=0, z=None, eps=None, per_particle=False, filter_pmf=0.1, max_k=None,
                  with_z=False, workspace=None):
    """Sampler + bucketing as one placement pass (ccmpc_sample_bucket, N <= 262144): the draws of
    sample_unicycle with the same arguments, bucketed as bucket() buckets them (each cell the
    same particles in the same order, the same pmf / init_center bits; only the cell offsets
    differ).  latent_pmf (O, L) is required (it decides the kept modes).

    Returns (bucketed F32 ParticleStore, K per OV, cell_pmf [n_cells] device, init_center
    [n_cells, 2] device), and the sample-order z [O, N] first when with_z.  workspace: an
    optional uint8 device tensor, zero-filled once by the caller and reused across calls."""
    lib = _lib.load()
    dev = require_device(device)
    if latent_pmf is None:
        raise ValueError("latent_pmf decides the kept modes: it is required")
    if not 1 <= int(N) <= FUSED_MAX_N:
        raise ValueError(f"sample_bucket takes N in [1, {FUSED_MAX_N}]: use sample_unicycle + "
                         "bucket beyond")
    O, L, t_init, t_cdf, t_gmm, layout, t_z, t_eps = _sampler_inputs(
        init_state, latent_pmf, gmm, N, T, dev, z, eps, per_particle)
    pmf = np.asarray(latent_pmf, np.float64).reshape(O, L)
    K, max_k, keep_map, cell_base = _bucket_plan(pmf, filter_pmf, max_k)
    region, cur, n_bound = [], 0, 0
    for o in range(O):
        region.append(cur)
        cur = _round4(cur + K[o] * (N + 4))          # room for every cell's worst case
        n_bound = _round4(n_bound + N + 4 * K[o])    # the particles themselves (+ alignment)
    n_cells = int(sum(K))
    origin = np.repeat(np.asarray(minpos, np.float64).reshape(-1, 2), K, axis=0)
    out = ParticleStore(T, [0] * n_cells, dtype=torch.float32, device=dev, origin=origin,
                        capacity=cur)
    out.counts = None                                   # device-side until sync_counts()
    out.n_bound = n_bound
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)
    t_keep, t_nk, t_base = t(keep_map), t(np.asarray(K, np.int32)), t(cell_base)
    t_min = t(np.asarray(minpos, np.float64).reshape(-1, 2))
    t_reg = t(np.asarray(region, np.int64))
    pmf_out = torch.empty(n_cells, dtype=torch.float64, device=dev)
    centre = torch.empty((n_cells, 2), dtype=torch.float64, device=dev)
    out_z = torch.empty((O, N), dtype=torch.int32, device=dev) if with_z else None
    need = lib.ccmpc_sample_bucket_workspace_bytes(O, N, T, max_k)
    if need == 0:
        raise ValueError("shape not supported by ccmpc_sample_bucket")
    ws = workspace if workspace is not None else torch.zeros(need, dtype=torch.uint8, device=dev)
    _lib.check(lib.ccmpc_sample_bucket(
        _p(t_init), _p(t_cdf), L, _p(t_gmm), layout, _p(t_z), _p(t_eps), O, N, T, float(dt),
        int(seed) & (2**64 - 1), None, int(ov_base), _p(t_keep), _p(t_nk), _p(t_base), max_k,
        _p(t_min), _p(t_reg), _p(ws), ws.numel(), _p(out_z), _p(out.pos), out.ld,
        _p(out.cell_off), _p(out.cell_cnt), _p(pmf_out), _p(centre), _stream()),
        "ccmpc_sample_bucket")
    out._keepalive = (t_init, t_cdf, t_gmm, t_z, t_eps, t_keep, t_nk, t_base, t_min, t_reg, ws)
    if with_z:
        return out_z, out, K, pmf_out, centre
    return out, K, pmf_out, centre


def bucket_predictions(predictions, z, latent_pmf, minpos, rows=None, filter_pmf=0.1,
                       max_k=None, device="cuda", workspace=None):
    """make_ovehicles on generate_vehicle_latents' predictions (nodes, N, T, 2) float32 and z
    (nodes, N) int64 / int32 (prediction.py:93-105; host arrays or device tensors) in one
    placement pass (ccmpc_bucket_predictions): the cells load_predictions + bucket give, bit
    for bit (only the cell offsets differ).  OV o = node rows[o] (default: every node);
    latent_pmf (O, L).  Raises IndexError where the reference's list index does (an id outside
    [-L, L)).  Returns (bucketed F32 ParticleStore, K per OV, cell_pmf, init_center)."""
    lib = _lib.load()
    dev = require_device(device)
    pred = torch.as_tensor(predictions, device=dev)
    if pred.dtype != torch.float32 or pred.dim() != 4 or pred.shape[3] != 2:
        raise ValueError("predictions must be (nodes, N, T, 2) float32")
    pred = pred.contiguous()
    zt = torch.as_tensor(z, device=dev).contiguous()
    if zt.dtype not in (torch.int64, torch.int32) or tuple(zt.shape) != tuple(pred.shape[:2]):
        raise ValueError("z must be (nodes, N) int64 or int32")
    n_nodes, N, T = int(pred.shape[0]), int(pred.shape[1]), int(pred.shape[2])
    rows = list(range(n_nodes)) if rows is None else [int(r) for r in rows]
    if any(r < 0 or r >= n_nodes for r in rows):
        raise ValueError(f"rows outside [0, {n_nodes})")
    pmf = np.asarray(latent_pmf, np.float64)
    O, L = pmf.shape
    if O != len(rows):
        raise ValueError(f"latent_pmf has {O} rows for {len(rows)} OVs")
    if not 1 <= N <= FUSED_MAX_N:
        raise ValueError(f"bucket_predictions takes N in [1, {FUSED_MAX_N}]: use "
                         "load_predictions + bucket beyond")
    K, max_k, keep_map, cell_base = _bucket_plan(pmf, filter_pmf, max_k)
    region, cur, n_bound = [], 0, 0
    for o in range(O):
        region.append(cur)
        cur = _round4(cur + K[o] * (N + 4))
        n_bound = _round4(n_bound + N + 4 * K[o])
    n_cells = int(sum(K))
    mp = np.asarray(minpos, np.float64).reshape(-1, 2)
    mp = np.tile(mp, (O, 1)) if mp.shape[0] == 1 else mp
    origin = np.repeat(mp, K, axis=0)
    out = ParticleStore(T, [0] * n_cells, dtype=torch.float32, device=dev, origin=origin,
                        capacity=cur)
    out.counts = None
    out.n_bound = n_bound
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)
    t_keep, t_nk, t_base = t(keep_map), t(np.asarray(K, np.int32)), t(cell_base)
    t_min, t_reg = t(mp), t(np.asarray(region, np.int64))
    t_rows = t(np.asarray(rows, np.int32))
    pmf_out = torch.empty(n_cells, dtype=torch.float64, device=dev)
    centre = torch.empty((n_cells, 2), dtype=torch.float64, device=dev)
    z_bad = torch.empty(O, dtype=torch.int32, device=dev)
    need = lib.ccmpc_sample_bucket_workspace_bytes(O, N, T, max_k)
    if need == 0:
        raise ValueError("shape not supported by ccmpc_bucket_predictions")
    ws = workspace if workspace is not None else torch.empty(need, dtype=torch.uint8, device=dev)
    _lib.check(lib.ccmpc_bucket_predictions(
        _p(pred), _p(zt), zt.element_size(), _p(t_rows), O, N, T, L, _p(t_keep), _p(t_nk),
        _p(t_base), max_k, _p(t_min), _p(t_reg), _p(ws), ws.numel(), _p(out.pos), out.ld,
        _p(out.cell_off), _p(out.cell_cnt), _p(pmf_out), _p(centre), _p(z_bad), _stream()),
        "ccmpc_bucket_predictions")
    raise_bad_latents(z_bad.cpu().numpy(), L)
    out._keepalive = (pred, zt, t_rows, t_keep, t_nk, t_base, t_min, t_reg, ws)
    return out, K, pmf_out, centre


def affine(mean, cov, ref_traj, cell_gamma, cell_ref=None, R=3.4, out_rec=None):
    lib = _lib.load()
    C, T = mean.shape[0], mean.shape[1]
    if out_rec is None:
        out_rec = torch.empty((C, T, 128), dtype=torch.uint8, device=mean.device)
    _lib.check(lib.ccmpc_affine(_p(mean), _p(cov), T, C, _p(ref_traj), _p(cell_ref),
                                _p(cell_gamma), float(R), _p(out_rec), _stream()),
               "ccmpc_affine")
    return out_rec


TANGENT_CHOOSE = -2  # CCMPC_TANGENT_CHOOSE: the reference's const_idx = None


def affine_scale(mean, cov, ref_traj, cell_risk, tangent=None, const_idx=None, cell_ref=None,
                 R=3.4, out_rec=None, scaled=True):
    """GMM-affine half-spaces with the recursive-feasibility covariance scale
    (ccmpc_affine_scale; v8ideal/__init__.py:2074-2456).  tangent [C, T] float64 and
    const_idx [C, T] int32 carry the previous frame's slopes / tangent indices (T < ph);
    None -> slopes from ref_traj and the closest tangent (T == ph).  scaled=False is
    compute_obstacle_constraints_GMM_affine_robust (:1541-1878): scale = 1."""
    lib = _lib.load()
    C, T = mean.shape[0], mean.shape[1]
    dev = mean.device
    if out_rec is None:
        out_rec = torch.empty((C, T, 128), dtype=torch.uint8, device=dev)
    tg = ci = None
    if tangent is not None:
        tg = torch.as_tensor(np.asarray(tangent, np.float64).reshape(C, T), device=dev)
        ci = torch.as_tensor(np.asarray(const_idx, np.int32).reshape(C, T), device=dev)
    _lib.check(lib.ccmpc_affine_scale(_p(mean), _p(cov), T, C, _p(ref_traj), _p(cell_ref),
                                      _p(cell_risk), float(R), int(bool(scaled)), _p(tg),
                                      _p(ci), _p(out_rec),
                                      _stream()), "ccmpc_affine_scale")
    out_rec._keepalive = (tg, ci)
    return out_rec


def ideal_rollout(prev_mean, prev_cov, src_cell, T, n_samples, x0=None, Z=None, seed=0,
                  rng_cell=None):
    """Materialised predict_ideal trajectories as an F64 ParticleStore + per-cell status."""
    lib = _lib.load()
    C = src_cell.shape[0]
    T_src = prev_mean.shape[1]
    store = ParticleStore(T, [n_samples] * C, dtype=torch.float64, device=prev_mean.device, align=4,
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


def bucket(z, sample_store, latent_pmf, minpos, filter_pmf=0.1, max_k=None):
    """GPU bucketing (ccmpc_bucket) of a sampler output (z [O,N], sample-order F32 store with
    one cell per OV) into kept-mode cells.  latent_pmf (O, L) is host data, as in the reference
    (latent_probs come back to the host in prediction.py:77-79).

    Returns (bucketed F32 ParticleStore with origin = minpos per cell, K per OV, cell_pmf
    [n_cells] device, init_center [n_cells, 2] device).  Device-side counts: store.counts holds
    capacity bounds until ``store.sync_counts()``.
    """
    lib = _lib.load()
    dev = sample_store.device
    pmf = np.asarray(latent_pmf, np.float64)
    O, L = pmf.shape
    N = int(z.shape[1])
    T = sample_store.T
    K, max_k, keep_map, cell_base = _bucket_plan(pmf, filter_pmf, max_k)
    region, cur = [], 0
    for o in range(O):
        region.append(cur)
        cur = _round4(cur + N + 4 * K[o])
    n_cells = int(sum(K))
    origin = np.repeat(np.asarray(minpos, np.float64).reshape(-1, 2), K, axis=0)
    out = ParticleStore(T, [0] * n_cells, dtype=torch.float32, device=dev, origin=origin,
                        capacity=cur)
    out.counts = None                                   # device-side until sync_counts()
    out.n_bound = cur
    t = lambda a, dt=None: torch.as_tensor(np.ascontiguousarray(a), device=dev)
    t_keep, t_nk, t_base = t(keep_map), t(np.asarray(K, np.int32)), t(cell_base)
    t_min = t(np.asarray(minpos, np.float64).reshape(-1, 2))
    t_reg = t(np.asarray(region, np.int64))
    pmf_out = torch.empty(n_cells, dtype=torch.float64, device=dev)
    centre = torch.empty((n_cells, 2), dtype=torch.float64, device=dev)
    need = lib.ccmpc_bucket_workspace_bytes(O, N, L, max_k)
    ws = torch.zeros(max(need, 16), dtype=torch.uint8, device=dev)   # zero-filled head: counters
    _lib.check(lib.ccmpc_bucket(_p(z), _p(sample_store.pos), sample_store.ld, T, O, N, L,
                                _p(t_keep), _p(t_nk), _p(t_base), max_k, _p(t_min), _p(t_reg),
                                _p(ws), ws.numel(), _p(out.pos), out.ld, _p(out.cell_off),
                                _p(out.cell_cnt), _p(pmf_out), _p(centre), _stream()),
               "ccmpc_bucket")
    out._keepalive = (t_keep, t_nk, t_base, t_min, t_reg, ws)
    return out, K, pmf_out, centre
