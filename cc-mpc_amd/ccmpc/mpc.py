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
import os

import numpy as np
import torch

from . import _lib, engine

# the planning frame's LTV rebuild inside the QP's launch (ccmpc_mpc_qp_ltv); 0: its own kernel
_FUSED_LTV = os.environ.get("CCMPC_QP_FUSED_LTV", "1") == "1"

U_ORDER_F, U_ORDER_C = 0, 1            # CCMPC_U_ORDER_*: cvxpy's default reshape is 'F'
REC_HALFSPACE, REC_AFFINE = 0, 1       # CCMPC_REC_KIND_*
REC_HALFSPACE_COMPACT, REC_AFFINE_COMPACT = 2, 3   # the same, as 32-byte ccmpc_gather_rec
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


class QpLtv(ctypes.Structure):
    """ccmpc_qp_ltv: the fused LTV rebuild's inputs (x_init a device pointer)."""
    _fields_ = [("x_init", ctypes.c_void_p), ("Ts", ctypes.c_double), ("l_r", ctypes.c_double),
                ("L", ctypes.c_double)]


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

    def solve(self, gamma, xbar, goal, ref, rec, u_prev=None, ubar=None, ltv=None):
        """Enqueue the S solves.  gamma [S, 4T_full, 2T_full], xbar [S, 4T_full],
        goal [S, 2], ref [S, n_ref, 2], rec the records (uint8 [cells, P, 128] tensor, or
        [cells, P, 32] ccmpc_gather_rec for the *_COMPACT kinds).  ltv = (x_init [S, 4] device
        tensor, Ts, lon): rebuild the LTV model about u = 0 in the same launch
        (ccmpc_mpc_qp_ltv) -- gamma / xbar are then its outputs."""
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
        P = T * (T - 1) // 2 if self.kind in (REC_HALFSPACE, REC_HALFSPACE_COMPACT) else T
        B = 32 if self.kind >= REC_HALFSPACE_COMPACT else 128    # record bytes
        if P > 0 and self.n_cells > 0:
            self._need(rec, "rec", None, torch.uint8)
            if rec.numel() < self.n_cells * P * B or (rec.dim() == 3 and (
                    rec.shape[1] != P or rec.shape[2] != B)):
                raise ValueError(f"rec: [cells >= {self.n_cells}, {P}, {B}] records expected")
        if u_prev is not None and Tf > T:
            self._need(u_prev, "u_prev", (S, 2 * (Tf - T)))
        if ubar is not None:
            self._need(ubar, "ubar", (S, 2 * Tf))
        p = engine._p
        if ltv is not None:
            x0, Ts, lon = ltv
            self._need(x0, "x_init", (S, 4))
            if ubar is not None:
                raise ValueError("the fused LTV rebuild is the model about u = 0 (no ubar)")
            spec = QpLtv(x_init=p(x0), Ts=float(Ts), l_r=0.5 * float(lon), L=float(lon))
            _lib.check(lib.ccmpc_mpc_qp_ltv(
                ctypes.byref(spec), self.S, self.T, self.T_full, p(gamma), p(xbar), p(u_prev),
                p(goal), p(ref), ref.shape[1], p(rec), self.kind, p(self.scene_cell),
                self.max_cells, ctypes.byref(self.params), self.u_order, self.max_iter,
                self.tol, p(self.ws), self.ws.numel(), p(self.u), p(self.X), p(self.cost),
                p(self.status), p(self.iters), engine._stream()), "ccmpc_mpc_qp_ltv")
            return self.u, self.X, self.cost, self.status, self.iters
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


class PlanningQPStep:
    """One scene's planning QP as the planner calls it every frame, with its host traffic in
    two pinned packs (ccmpc/step.py's Pack): the frame's x_init, reference, goal and executed
    controls go up in one copy kernel, the LTV model (when the frame rebuilds it) and the solve
    run on the device on the generator's device records, and u, X, cost and status come back
    in one copy kernel followed by ccmpc_signal_host, which the host polls -- one wait for the
    whole solve instead of a synchronising copy per tensor (~10 us each).

    The LTV buffers (xbar [1, 4 ph], gamma [1, 4 ph, 2 ph]) belong to the caller: they are
    rebuilt at Tsh == ph and kept below it (v8ideal/__init__.py:2858-2891)."""

    def __init__(self, n_cells, T, T_full, kind=REC_HALFSPACE, params=None, u_order=U_ORDER_F,
                 device="cuda"):
        from . import step
        self.T, self.T_full = int(T), int(T_full)
        T, Tf = self.T, self.T_full
        self.device = engine.require_device(device)
        self.u_order = int(u_order)
        f64, i32, i64 = torch.float64, torch.int32, torch.int64
        self.inp = step.Pack([("gen", (2,), i64), ("x0", (1, 4), f64), ("ref", (1, T, 2), f64),
                              ("goal", (1, 2), f64), ("uprev", (1, max(2 * (Tf - T), 1)), f64)],
                             self.device)
        self.out = step.Pack([("u", (1, 2 * T), f64), ("X", (1, T, 4), f64), ("cost", (1,), f64),
                              ("status", (1,), i32), ("iters", (1,), i32)], self.device)
        self.qp = PlanningQP([n_cells], T, T_full=Tf, kind=kind, params=params,
                             u_order=u_order, device=self.device)
        o = self.out        # the solve writes straight into the output pack's device half
        self.qp.u, self.qp.X, self.qp.cost = o.d("u"), o.d("X"), o.d("cost")
        self.qp.status, self.qp.iters = o.d("status"), o.d("iters")
        self.flags = torch.zeros(2, dtype=i64, pin_memory=True)
        self._flags = self.flags.numpy()
        self.generation = 0

    def solve(self, x_init, goal, ref_traj, rec, xbar, gamma, u_prev=None, ltv=False, Ts=0.5,
              lon=3.7):
        """Enqueue the frame on the current stream and wait for its answer on the host:
        {cost, U_star (T, 2), X_star (T, 4), u (2T,), status, iters}.  ltv: rebuild xbar /
        gamma from x_init first (Tsh == ph)."""
        return self.wait(self.launch(x_init, goal, ref_traj, rec, xbar, gamma, u_prev=u_prev,
                                     ltv=ltv, Ts=Ts, lon=lon))

    def launch(self, x_init, goal, ref_traj, rec, xbar, gamma, u_prev=None, ltv=False, Ts=0.5,
               lon=3.7):
        """solve() without the wait: enqueue the frame on the current stream (behind whatever
        writes `rec` there) and return its generation for wait()."""
        gen = self.prepare(x_init, goal, ref_traj, u_prev)
        self.enqueue(rec, xbar, gamma, ltv=ltv, Ts=Ts, lon=lon)
        return gen

    def prepare(self, x_init, goal, ref_traj, u_prev=None):
        """The host half of launch(): the frame's inputs into the pinned pack and a new
        generation (returned); enqueue() -- or a captured graph holding its calls -- moves
        them to the device."""
        T, Tf = self.T, self.T_full
        i = self.inp
        i.h("x0")[0] = np.asarray(x_init, np.float64).reshape(4)
        i.h("ref")[0] = np.asarray(ref_traj, np.float64)[:T].reshape(T, 2)
        i.h("goal")[0] = np.asarray(goal, np.float64).reshape(2)
        if T < Tf:
            if u_prev is None:
                raise ValueError("u_prev (the executed controls) is required when T < T_full")
            i.h("uprev")[0] = np.asarray(u_prev, np.float64).reshape(2 * (Tf - T))
        self.generation += 1
        i.h("gen")[0] = self.generation
        return self.generation

    def enqueue(self, rec, xbar, gamma, ltv=False, Ts=0.5, lon=3.7):
        """The device half of launch() on the current stream (capturable: every call reads
        the packs at run time): the inputs up, the LTV rebuild (ltv), the QP on `rec`, the
        answer down and the signal of the pack's generation."""
        T, Tf = self.T, self.T_full
        i, o, lib, p = self.inp, self.out, _lib.load(), engine._p
        s = engine._stream()
        chk = _lib.check
        chk(lib.ccmpc_copy_kernel_async(p(i.dev), p(i.host), i.nbytes, s), "ccmpc_copy_async")
        # the LTV rebuild (Tsh == ph) fused into the solve's launch, or (CCMPC_QP_FUSED_LTV=0)
        # as its own kernel first
        if ltv and not _FUSED_LTV:
            chk(lib.ccmpc_mpc_ltv(p(i.d("x0")), 1, Tf, float(Ts), 0.5 * float(lon), float(lon),
                                  p(xbar), p(gamma), s), "ccmpc_mpc_ltv")
        self.qp.solve(gamma, xbar, i.d("goal"), i.d("ref"), rec,
                      u_prev=i.d("uprev") if T < Tf else None,
                      ltv=(i.d("x0"), Ts, lon) if (ltv and _FUSED_LTV) else None)
        chk(lib.ccmpc_copy_signal_async(p(o.host), p(o.dev), o.nbytes, p(self.flags),
                                        p(i.d("gen")), s), "ccmpc_copy_signal_async")

    def wait(self, gen):
        """The answer of launch `gen` on the host (it must be the latest launch: the output pack
        is this step's)."""
        from . import step
        T = self.T
        if gen != self.generation:
            raise RuntimeError(f"planning QP {gen}: overwritten by launch {self.generation}")
        o = self.out
        step.poll_word(self._flags, 0, gen, self.device, f"planning QP {gen}: the")
        u = o.h("u")[0].copy()
        U = u.reshape(2, T).T.copy() if self.u_order == U_ORDER_F else u.reshape(T, 2).copy()
        return {"cost": float(o.h("cost")[0]), "U_star": U, "X_star": o.h("X")[0].copy(),
                "u": u, "status": int(o.h("status")[0]), "iters": int(o.h("iters")[0])}
