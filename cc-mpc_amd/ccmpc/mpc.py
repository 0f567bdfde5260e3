"""The planning step's QP on the GPU: the caller side of the constraint path.

v8ideal's do_highlevel_control (v8ideal/__init__.py:2850-3110) builds a cvxpy problem over the
2T controls and hands it to CPLEX, once per planning step and agent.  With the road-boundary
MILP off (the reference default, :217) that problem is a convex QP; here it is assembled and
solved on the device, batched over scenes, straight from the generators' records:

  ltv(x_init, T)              ccmpc_mpc_ltv  -- VehicleModel.get_optimization_ltv about u = 0
                              (dynamics/bicycle_v2.py:260-308, the planner's u_init, :537)
  PlanningQP.solve(...)       ccmpc_mpc_qp   -- one interior-point solve per scene

Every tensor is a torch device tensor; nothing here synchronises except the explicit
``.cpu()`` of results by the caller.  There is no CPU fallback.
"""
import ctypes
import math

import numpy as np
import torch

from . import _lib, engine

U_ORDER_F, U_ORDER_C = 0, 1            # CCMPC_U_ORDER_*: cvxpy's default reshape is 'F'
REC_HALFSPACE, REC_AFFINE = 0, 1       # CCMPC_REC_KIND_*
QP_OK, QP_MAXITER, QP_NUMERIC, QP_SKIPPED_ROWS = 0, 1, 2, 4


class MPCParams(ctypes.Structure):
    """ccmpc_mpc_params: the objective weights and limits of __make_global_params
    (v8ideal/__init__.py:86-109)."""
    _fields_ = [(name, ctypes.c_double) for name in (
        "w_final", "w_ref", "w_accel", "w_joint", "w_turning", "w_ch_accel", "w_ch_joint",
        "w_ch_turning", "min_a", "max_a", "max_delta", "max_v")]

    @classmethod
    def reference_defaults(cls, max_steer_deg=70.0):
        """The reference's values; max_delta = 0.5 * the ego wheel's max_steer_angle, which
        CARLA supplies (:106-109) -- 70 degrees unless given."""
        return cls(w_final=6.0, w_ref=3.0, w_accel=0.5, w_joint=0.2, w_turning=1.0,
                   w_ch_accel=0.5, w_ch_joint=0.1, w_ch_turning=2.0, min_a=-7.0, max_a=4.0,
                   max_delta=0.5 * math.radians(max_steer_deg), max_v=10.0)

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


def ltv(x_init, T, Ts=0.5, lon=3.7):
    """(x_bar [S, 4T], Gamma [S, 4T, 2T]) of VehicleModel(T, Ts, l_r=0.5 lon, L=lon)
    .get_optimization_ltv(x_init, [0, 0]) for every scene (make_local_params, :550-557)."""
    x = torch.as_tensor(np.asarray(x_init, np.float64).reshape(-1, 4))
    dev = engine.require_device("cuda")
    x = x.to(dev)
    S = x.shape[0]
    xbar = torch.empty((S, 4 * T), dtype=torch.float64, device=dev)
    gamma = torch.empty((S, 4 * T, 2 * T), dtype=torch.float64, device=dev)
    lib = _lib.load()
    _lib.check(lib.ccmpc_mpc_ltv(engine._p(x), S, int(T), float(Ts), 0.5 * float(lon),
                                 float(lon), engine._p(xbar), engine._p(gamma),
                                 engine._stream()), "ccmpc_mpc_ltv")
    return xbar, gamma


class PlanningQP:
    """Batched do_highlevel_control QP for S scenes sharing a horizon.

    ``scene_cells[s]`` is the number of record cells (OV modes) of scene s; the records of all
    scenes are one [cells][P] block as the cycle writes it (P = T(T-1)/2 half-spaces, or T
    affine records)."""

    def __init__(self, scene_cells, T, T_full=None, kind=REC_HALFSPACE, params=None,
                 u_order=U_ORDER_F, max_iter=60, tol=1e-9, device="cuda"):
        self.device = engine.require_device(device)
        self.T = int(T)
        self.T_full = int(T_full or T)
        self.kind = int(kind)
        self.params = params or MPCParams.reference_defaults()
        self.u_order, self.max_iter, self.tol = int(u_order), int(max_iter), float(tol)
        cells = [int(c) for c in scene_cells]
        self.S = len(cells)
        self.max_cells = max(cells) if cells else 0
        off = np.concatenate(([0], np.cumsum(cells))).astype(np.int64)
        self.n_cells = int(off[-1])
        self.scene_cell = torch.as_tensor(off, device=self.device)
        lib = _lib.load()
        need = lib.ccmpc_mpc_qp_workspace_bytes(self.S, self.T, self.max_cells, self.kind)
        self.ws = torch.zeros(max(int(need), 16), dtype=torch.uint8, device=self.device)
        dev, S, T = self.device, self.S, self.T
        self.u = torch.empty((S, 2 * T), dtype=torch.float64, device=dev)
        self.X = torch.empty((S, T, 4), dtype=torch.float64, device=dev)
        self.cost = torch.empty(S, dtype=torch.float64, device=dev)
        self.status = torch.empty(S, dtype=torch.int32, device=dev)
        self.iters = torch.empty(S, dtype=torch.int32, device=dev)

    def _need(self, t, name, shape, dtype=torch.float64):
        """The kernel reads raw pointers: refuse anything that is not the contiguous device
        array it assumes (a wrong shape would read out of bounds on the GPU)."""
        dev = self.device
        on_dev = isinstance(t, torch.Tensor) and t.device.type == dev.type and (
            dev.index is None or t.device.index == dev.index)
        if not on_dev or t.dtype != dtype or not t.is_contiguous():
            raise ValueError(f"{name}: contiguous {dtype} tensor on {self.device} required")
        if shape is not None and tuple(t.shape) != tuple(shape):
            raise ValueError(f"{name}: shape {tuple(t.shape)}, expected {tuple(shape)}")

    def solve(self, gamma, xbar, goal, ref, rec, u_prev=None, ubar=None):
        """Enqueue the S solves.  gamma [S, 4T_full, 2T_full], xbar [S, 4T_full],
        goal [S, 2], ref [S, n_ref, 2], rec the records (uint8 [cells, P, 128] tensor)."""
        lib = _lib.load()
        S, T, Tf = self.S, self.T, self.T_full
        ref = ref.reshape(S, -1, 2)
        if Tf > T and u_prev is None:
            raise ValueError("u_prev (the executed controls) is required when T < T_full")
        self._need(gamma, "gamma", (S, 4 * Tf, 2 * Tf))
        self._need(xbar, "xbar", (S, 4 * Tf))
        self._need(goal, "goal", (S, 2))
        self._need(ref, "ref", None)
        if ref.shape[1] < 1:
            raise ValueError("ref: at least one reference point per scene")
        P = T * (T - 1) // 2 if self.kind == REC_HALFSPACE else T
        if P > 0 and self.n_cells > 0:
            self._need(rec, "rec", None, torch.uint8)
            if rec.numel() < self.n_cells * P * 128 or (rec.dim() == 3 and rec.shape[1] != P):
                raise ValueError(f"rec: [cells >= {self.n_cells}, {P}, 128] records expected")
        if u_prev is not None and Tf > T:
            self._need(u_prev, "u_prev", (S, 2 * (Tf - T)))
        if ubar is not None:
            self._need(ubar, "ubar", (S, 2 * Tf))
        p = engine._p
        _lib.check(lib.ccmpc_mpc_qp(
            self.S, self.T, self.T_full, p(gamma), p(xbar), p(ubar), p(u_prev), p(goal), p(ref),
            ref.shape[1], p(rec), self.kind, p(self.scene_cell), self.max_cells,
            ctypes.byref(self.params), self.u_order, self.max_iter, self.tol, p(self.ws),
            self.ws.numel(), p(self.u), p(self.X), p(self.cost), p(self.status),
            p(self.iters), engine._stream()), "ccmpc_mpc_qp")
        return self.u, self.X, self.cost, self.status, self.iters

    def U(self, u=None):
        """U = reshape(u, (T, 2)) in the order the objective used (cvxpy default 'F')."""
        u = self.u if u is None else u
        if self.u_order == U_ORDER_F:
            return u.reshape(-1, 2, self.T).transpose(1, 2)
        return u.reshape(-1, self.T, 2)
