"""The v8 MILP obstacle constraints over the L4 outer approximation.

collect/in_simulation/midlevel/v8/__init__.py:692-724 (compute_obstacle_constraints): for
every OV, kept mode k and control step t, the L = 4 faces (A, b) of the L4 polytope that
`ccmpc_l4` computes on the device (:563-575 vertices, :630-671 over-approximation, the same
midlevel/util.py:compute_L4_outerapproximation as v8ideal) become big-M rows

    A[l] . X[t, :2] + M_big (1 - Delta[c, t, l]) + S_big[t, l]  >=  b[l] + diag    (l < L)
    sum_l Delta[c, t, l]  >=  1

with c = sum(K[:ov]) + k, Delta binary (sum K, T, L), diag = half the ego bbox diagonal
(:109) and S_big = M_big * sum(Omicron[~segments.mask], axis=0) repeated over L when road
boundaries are on (:700-702).  With road boundaries off the reference writes
`np.zeros(T, L, dtype=float)`, which numpy rejects (TypeError); S_big = 0 is its intent and
what this module uses.

The rows are produced from the device L4 arrays in one copy; `BigMRows.expr` builds the
reference's constraint list with any variable type that supports + * >= (docplex, cvxpy),
`coo` gives the same rows as a sparse G z >= h for a batched QP/MILP assembly, and
`satisfied` evaluates them numerically.
"""
import os

import numpy as np
import torch

from . import planner

M_BIG = 10_000          # v8/__init__.py:77
N_FACES = 4             # params.L, v8/__init__.py:105


def ego_diag(lon, lat):
    """params.diag (v8/__init__.py:109): half the diagonal of the ego bounding box."""
    return float(np.sqrt(lon ** 2 + lat ** 2) / 2.0)


class BigMRows:
    """Big-M rows of one planning step.  A (C, T, L, 2), rhs = b + diag (C, T, L); cells in
    (ov, k) order, so Delta's first index is the cell index."""

    def __init__(self, A, b, diag, T, M_big=M_BIG):
        self.T = int(T)
        self.A = np.ascontiguousarray(A[:, :self.T])
        self.rhs = np.ascontiguousarray(b[:, :self.T] + float(diag))
        self.M_big = float(M_big)
        self.n_cells = self.A.shape[0]
        self.L = self.A.shape[2]

    def __len__(self):
        """Number of scalar constraints the reference emits: (L + 1) per (cell, t)."""
        return self.n_cells * self.T * (self.L + 1)

    def lhs(self, xy, delta, S_big=None):
        """Numeric left-hand sides (C, T, L) for ego positions xy (T, 2), delta (C, T, L)."""
        xy = np.asarray(xy, float)[:self.T, :2]
        v = np.einsum("ctlj,tj->ctl", self.A, xy) + self.M_big * (1.0 - np.asarray(delta, float))
        if S_big is not None:
            v = v + np.broadcast_to(np.asarray(S_big, float).reshape(self.T, -1), v.shape[1:])
        return v

    def satisfied(self, xy, delta, S_big=None):
        """(C, T) bool: every face row and the sum row of (cell, t) hold."""
        rows = self.lhs(xy, delta, S_big) >= self.rhs
        return rows.all(-1) & (np.asarray(delta).sum(-1) >= 1)

    def outside(self, xy):
        """(C, T) bool: the ego position lies on the far side of at least one face (the
        disjunction the binaries encode, with the tightest choice of Delta)."""
        xy = np.asarray(xy, float)[:self.T, :2]
        return (np.einsum("ctlj,tj->ctl", self.A, xy) >= self.rhs).any(-1)

    def expr(self, X, Delta, S_big=None):
        """The reference's constraint list (v8/__init__.py:708-724), in its order: for ov, k, t
        the L face rows then the sum row.  X (T, >=2) and Delta (C, T, L) may hold solver
        variables."""
        out = []
        for c in range(self.n_cells):
            for t in range(self.T):
                s_t = 0.0 if S_big is None else S_big[t]
                for l in range(self.L):
                    a = self.A[c, t, l]
                    s = s_t if np.ndim(s_t) == 0 else s_t[l]
                    lhs = a[0] * X[t, 0] + a[1] * X[t, 1] + self.M_big * (1 - Delta[c, t, l]) + s
                    out.append(lhs >= self.rhs[c, t, l])
                out.append(sum(Delta[c, t, l] for l in range(self.L)) >= 1)
        return out

    def coo(self):
        """Sparse G z >= h over z = [X[0,0], X[0,1], ..., X[T-1,1], Delta.ravel()] (Delta in
        (C, T, L) order), rows in expr() order.  Returns (row, col, val, h)."""
        C, T, L = self.n_cells, self.T, self.L
        c, t, l = np.meshgrid(np.arange(C), np.arange(T), np.arange(L), indexing="ij")
        block = (c * T + t) * (L + 1)                       # first row of (c, t)
        face_row = (block + l).ravel()
        d_col = 2 * T + ((c * T + t) * L + l).ravel()
        rows = [face_row, face_row, face_row]
        cols = [(2 * t).ravel(), (2 * t + 1).ravel(), d_col]
        vals = [self.A[..., 0].ravel(), self.A[..., 1].ravel(), np.full(d_col.size, -self.M_big)]
        sum_row = (block[..., 0] + L).ravel()
        rows.append(np.repeat(sum_row, L))
        cols.append(d_col)
        vals.append(np.ones(d_col.size))
        h = np.empty(C * T * (L + 1))
        h[face_row] = (self.rhs - self.M_big).ravel()
        h[sum_row] = 1.0
        return (np.concatenate(rows), np.concatenate(cols), np.concatenate(vals), h)


class MidlevelAgentV8(planner.MidlevelAgent):
    """The constraint surface of v8.MidlevelAgent (v8/__init__.py): the MILP generator over
    the same device-side particles, L4 kernel and vertex views as the v8ideal mirror."""

    def __init__(self, prediction_horizon=8, control_horizon=None, M_big=M_BIG, diag=None,
                 **kwargs):
        super().__init__(prediction_horizon=prediction_horizon, control_horizon=control_horizon,
                         **kwargs)
        self.M_big = M_big
        self.diag = diag
        self.L = N_FACES

    def compute_obstacle_constraints(self, params, ovehicles, X, Delta, Omicron, segments):
        """v8/__init__.py:692-724.  Returns (constraints, vertices, A_union, b_union);
        constraints is BigMRows when X is None, else the reference's expression list."""
        diag = getattr(params, "diag", None)
        diag = self.diag if diag is None else diag
        if diag is None:
            raise ValueError("params.diag (ego bbox half diagonal, v8/__init__.py:109) is unset")
        T = self.control_horizon
        scene = self._scene(ovehicles)
        vertices, A_union, b_union = self._l4_lists(scene)
        l4 = scene.l4_host()
        rows = BigMRows(l4["A"], l4["b"], diag, T, self.M_big)
        if X is None:
            return rows, vertices, A_union, b_union
        S_big = None
        if self.road_boundary_constraints:
            S_big = self.M_big * np.sum(Omicron[~segments.mask], axis=0)
            S_big = np.repeat(S_big[..., None], self.L, axis=1)
        return rows.expr(X, Delta, S_big), vertices, A_union, b_union

    def compute_objective(self, X, U, goal):
        """v8/__init__.py:727-753 (the module-level compute_objective, v8's weights)."""
        return compute_objective(X, U, goal)

    def do_highlevel_control(self, params, ovehicles):
        """v8/__init__.py:755-873: the obstacle big-M rows over the device L4 faces,
        compute_objective, and the MILP solved by BranchAndBound on the GPU (CPLEX's role).
        params: x_init [x, y, psi, v] (make_local_params' state; the LTV model is built about
        u = 0 on the device), goal (2,) and, with road_boundary_constraints, segments -- the
        map reader's compute_segs_polytopes_and_goal payload (polytopes [(A, b)], mask;
        road.py:639-678), whose Omicron binaries the same branch and bound takes one polytope
        per step (:676-702); diag as compute_obstacle_constraints reads it.  Returns
        (AttrDict(cost, U_star, X_star, goal, A_union, b_union, vertices, segments, faces[,
        polytopes]), None), or with cost / U_star / X_star None and an InSimulationException
        where the reference's solve fails (:862-873)."""
        from .standins import AttrDict
        segments = getattr(params, "segments", None) if self.road_boundary_constraints else None
        if self.road_boundary_constraints and segments is None:
            raise ValueError("road_boundary_constraints: params.segments (the map reader's "
                             "polytopes and junction mask, v8/__init__.py:759) is required")
        rows, vertices, A_union, b_union = self.compute_obstacle_constraints(
            params, ovehicles, None, None, None, None)
        goal = np.asarray(params.goal, np.float64)
        T = self.control_horizon
        bnb = BranchAndBound(rows, T, params.x_init, goal, lon=self.ego_lon,
                             params=v8_qp_params(self.mpc_params_steer), device=self.device,
                             segments=None if segments is None else RoadSegments(segments))
        sol = bnb.solve()
        self.last_bnb = dict(bnb.stats)
        out = AttrDict(cost=None, U_star=None, X_star=None, goal=goal, A_union=A_union,
                       b_union=b_union, vertices=vertices, segments=segments)
        if sol is None:
            return out, planner.InSimulationException("Optimizer failed to find a solution")
        out.update(cost=sol["cost"], U_star=sol["u"].reshape(T, 2), X_star=sol["X"],
                   faces=sol["faces"])
        if segments is not None:
            out.polytopes = sol["segments"]          # the Omicron column chosen per step
        return out, None



# ---- v8's MILP solve (v8/__init__.py:755-838) ----------------------------------------------
# v8/__init__.py:84-92 (params.objective) and :77-80 (limits)
V8_OBJECTIVE = dict(w_final=3.0, w_ch_accel=0.5, w_ch_turning=2.0, w_ch_joint=0.1, w_accel=0.5,
                    w_turning=1.0, w_joint=0.2)
V8_LIMITS = dict(max_a=3.5, min_a=-7.0, max_v=10.0)


def compute_objective(X, U, goal, objective=None):
    """v8/__init__.py:727-753 (compute_objective): works on numbers or on solver expressions
    (anything with + - * and **); U = u.reshape(T, nu), row-major."""
    obj = V8_OBJECTIVE if objective is None else objective
    cost = obj["w_final"] * (X[-1, 0] - goal[0]) ** 2 + obj["w_final"] * (X[-1, 1] - goal[1]) ** 2
    for u1, u2 in zip(U[:-1, 0], U[1:, 0]):           # util.pairwise: consecutive pairs
        _u = u1 - u2
        cost += obj["w_ch_accel"] * _u * _u
    for u1, u2 in zip(U[:-1, 1], U[1:, 1]):
        _u = u1 - u2
        cost += obj["w_ch_turning"] * _u * _u
    for u1, u2 in zip(U[:-1], U[1:]):
        _u = u1 - u2
        cost += obj["w_ch_joint"] * _u[0] * _u[1]
    cost += obj["w_accel"] * sum(U[:, 0] ** 2)
    cost += obj["w_turning"] * sum(U[:, 1] ** 2)
    cost += 2.0 * obj["w_joint"] * sum(U[:, 0] * U[:, 1])
    return cost


def v8_qp_params(max_steer_deg=70.0, objective=None, limits=None):
    """ccmpc_mpc_params of v8's problem for mpc_qp_kernel: v8's objective is the kernel's with
    no reference term (w_ref = 0) and R2's off-diagonal w_ch_joint / 2 (v8 adds w_ch_joint
    du_0 du_1 once; the kernel's quadratic form counts its off-diagonal twice); solved with
    CCMPC_U_ORDER_C (U = u.reshape(T, nu) of an object array pairs (u[2t], u[2t+1]))."""
    from . import mpc
    import math
    o = dict(V8_OBJECTIVE, **(objective or {}))
    lim = dict(V8_LIMITS, **(limits or {}))
    return mpc.MPCParams(w_final=o["w_final"], w_ref=0.0, w_accel=o["w_accel"],
                         w_joint=o["w_joint"], w_turning=o["w_turning"],
                         w_ch_accel=o["w_ch_accel"], w_ch_joint=0.5 * o["w_ch_joint"],
                         w_ch_turning=o["w_ch_turning"], min_a=lim["min_a"], max_a=lim["max_a"],
                         max_delta=0.5 * math.radians(max_steer_deg), max_v=lim["max_v"])


_GATHER = np.dtype([("n0", "<f8"), ("n1", "<f8"), ("rhs", "<f8"), ("side", "<i2"),
                    ("status", "<i2"), ("t_tau", "<i4")])       # ccmpc_gather_rec


class RoadSegments:
    """The map reader's segment payload (road.py:639-678, collect_segs_polytopes_and_goal:
    polytopes [(A (F, 2), b (F,))] with A x <= b inside, mask True where a polytope covers a
    junction) as padded arrays: A (I, F, 2), b (I, F), live (I, F), junction (I,)."""

    def __init__(self, segments):
        get = (lambda k: segments[k]) if isinstance(segments, dict) else (
            lambda k: getattr(segments, k))
        polys = [(np.asarray(a, np.float64).reshape(-1, 2), np.asarray(b, np.float64).ravel())
                 for a, b in get("polytopes")]
        self.I = len(polys)
        self.junction = np.asarray(get("mask"), bool).reshape(self.I)
        self.F = max([len(b) for _, b in polys] + [1])
        self.A = np.zeros((self.I, self.F, 2))
        self.b = np.zeros((self.I, self.F))
        self.live = np.zeros((self.I, self.F), bool)
        for i, (a, b) in enumerate(polys):
            if a.shape[0] != b.shape[0]:
                raise ValueError(f"segment {i}: A has {a.shape[0]} rows, b {b.shape[0]}")
            self.A[i, :len(b)], self.b[i, :len(b)], self.live[i, :len(b)] = a, b, True
        self.any_open = bool((~self.junction).any())     # some choice relaxes the obstacles


class MilpBnB:
    """Exact best-first branch and bound of the planner's MILPs on the GPU, around
    mpc_qp_kernel: every node's relaxation is one convex QP, and each round's nodes are ONE
    batched launch.  The binaries it branches on:

      faces     v8's Delta: one L4 face a_l . x_t + S_t >= rhs_l per (cell, t) (milp.BigMRows)
      segments  Omicron: one road polytope A_i x_t <= b_i per t (RoadSegments)

    beside `base` rows that every node keeps (the v8ideal generators' half-spaces), of which
    those flagged sbig carry + S_t on their right-hand side as the affine and scale-ideal
    generators write it (v8ideal/__init__.py:1503-1515, :2394-2414).  S_t = M_big per chosen
    non-junction polytope.

    One polytope per t is enough: every Omicron[:, t] with several polytopes is dominated by
    one of its members (one polytope's rows instead of several, and S_t = M_big already
    relaxes every obstacle row it touches -- the L4 faces and the '<=' half-spaces lie within
    metres of the ego, far inside M_big = 1e4 -- while a second non-junction polytope would
    only tighten the '>=' half-spaces further).  The oracle's literal enumeration over every
    subset checks this (tests/test_milp.py).

    A node fixes faces {(c, t): l} and polytopes {t: i}.  Its relaxation keeps the rows that
    hold for every completion: a fixed face only where t's polytope is fixed (or none can
    relax it), shifted by S_t; a fixed polytope's rows; the base rows with S_t where t's
    polytope is fixed, else the '>=' rows unshifted and the sbig '<=' rows left out.  A node
    whose optimum satisfies every step under some polytope (and every (cell, t) disjunction)
    is feasible for the MILP and becomes the incumbent if cheaper; otherwise its most violated
    step is branched -- over the polytopes if t's is free, else over the faces of its most
    violated (cell, t).  Nodes are pruned by their parent's optimum; the objective has no
    binary terms, so the QP optimum is the MILP cost.  Deterministic: the same QP results give
    the same tree."""

    def __init__(self, T, gamma, xbar, goal, ref=None, params=None, u_order=None, T_full=None,
                 u_prev=None, base=None, faces=None, segments=None, M_big=M_BIG, batch=64,
                 tol=1e-7, max_nodes=100000, device="cuda", ltv=None):
        from . import engine, mpc
        self.dev = engine.require_device(device)
        T_full = int(T_full or T)
        # ltv: (x_init (4,), Ts, lon) -- the model about u = 0 rebuilt inside each round's QP
        # launch from x_init in the round's input pack (ccmpc_mpc_qp_ltv), no gamma / xbar given
        self.ltv = None if ltv is None else (np.asarray(ltv[0], np.float64).reshape(4),
                                             float(ltv[1]), float(ltv[2]))
        if self.ltv is None:
            self.gamma = gamma.reshape(1, 4 * T_full, 2 * T_full).to(self.dev)
            self.xbar = xbar.reshape(1, 4 * T_full).to(self.dev)
        else:
            self.gamma = self.xbar = None
        self.u_prev_h = None if u_prev is None else np.asarray(u_prev, np.float64).reshape(-1)
        self.u_prev = None if u_prev is None else torch.as_tensor(
            self.u_prev_h.reshape(1, -1), device=self.dev)
        if T_full > int(T) and self.u_prev is None:
            raise ValueError("u_prev (the executed controls) is required when T < T_full")
        self._host_init(T, goal, ref, params or v8_qp_params(),
                        mpc.U_ORDER_C if u_order is None else u_order, T_full, base, faces,
                        segments, M_big, batch, tol, max_nodes)

    def _host_init(self, T, goal, ref, params, u_order, T_full, base, faces, segments, M_big,
                   batch, tol, max_nodes):
        """Everything but the device model (the tree logic runs on host arrays)."""
        self.T, self.T_full = int(T), int(T_full)
        self.goal = np.asarray(goal, np.float64).reshape(2)
        self.ref = np.asarray(self.goal.reshape(1, 2) if ref is None else ref,
                              np.float64).reshape(-1, 2)
        self.params, self.u_order = params, int(u_order)
        self.M = float(M_big)
        self.batch, self.tol, self.max_nodes = int(batch), float(tol), int(max_nodes)
        T = self.T
        # faces (C, T, L): a_l . x_t >= rhs_l - S_t
        if faces is not None:
            self.fA = np.asarray(faces[0], np.float64)[:, :T]
            self.frhs = np.asarray(faces[1], np.float64)[:, :T]
        else:
            self.fA, self.frhs = np.zeros((0, T, 1, 2)), np.zeros((0, T, 1))
        self.C, self.L = self.frhs.shape[0], self.frhs.shape[2]
        # base rows (Cb, T): n, rhs, side (+1 '>=', -1 '<='), live, sbig
        if base is not None:
            self.bn = np.asarray(base["n"], np.float64).reshape(-1, T, 2)
            self.brhs = np.asarray(base["rhs"], np.float64).reshape(-1, T)
            self.bside = np.asarray(base["side"], np.int64).reshape(-1, T)
            self.blive = np.asarray(base["live"], bool).reshape(-1, T)
            sb = np.asarray(base.get("sbig", False), bool)
            self.bsbig = np.broadcast_to(sb[:, None] if sb.ndim == 1 else sb,
                                         self.brhs.shape).copy()      # per cell or per row
        else:
            self.bn, self.brhs = np.zeros((0, T, 2)), np.zeros((0, T))
            self.bside, self.blive = np.zeros((0, T), np.int64), np.zeros((0, T), bool)
            self.bsbig = np.zeros((0, T), bool)
        self.Cb = self.brhs.shape[0]
        self.seg = segments
        self.F = segments.F if segments is not None else 0
        self.stats = dict(nodes=0, launches=0, qps=0)
        self._qp = {}

    # ---- one round -------------------------------------------------------------------------
    def _records(self, nodes):
        """(S, Cb + C + F, T) compact affine records of the nodes' relaxations (every node's
        rows at once: the fixed faces and polytopes gathered into index arrays)."""
        S, T, Cb, C, seg = len(nodes), self.T, self.Cb, self.C, self.seg
        rec = np.zeros((S, Cb + C + self.F, T), _GATHER)
        rec["status"] = 1                                   # left out unless set below
        rec["t_tau"] = np.arange(T)
        fixed = np.full((S, T), -1, np.int64)               # each step's fixed polytope, or -1
        for s, (_, segs) in enumerate(nodes):
            for t, i in segs.items():
                fixed[s, t] = i
        isfix = fixed >= 0
        if seg is not None:                                 # S_t: M_big on a fixed non-junction
            shift = np.where(isfix & ~seg.junction[np.maximum(fixed, 0)], self.M, 0.0)
        else:
            shift = np.zeros((S, T))
        if Cb:
            keep = np.broadcast_to(self.blive, (S, Cb, T))
            if seg is not None and seg.any_open:    # a free step: S_t may relax the sbig '<='
                keep = keep & ~((self.bsbig & (self.bside == -1))[None] & ~isfix[:, None, :])
            b = rec[:, :Cb]
            b["n0"], b["n1"] = self.bn[None, ..., 0], self.bn[None, ..., 1]
            b["rhs"] = self.brhs[None] + np.where(self.bsbig[None], shift[:, None, :], 0.0)
            b["side"] = self.bside[None]
            b["status"] = np.where(keep, 0, 1)
        fe = [(s, c, t, l) for s, (faces, _) in enumerate(nodes) for (c, t), l in faces.items()]
        if fe:
            s_, c_, t_, l_ = np.array(fe, np.int64).T
            if seg is not None and seg.any_open:            # S_t may relax it: left out
                k = isfix[s_, t_]
                s_, c_, t_, l_ = s_[k], c_[k], t_[k], l_[k]
            at = (s_, Cb + c_, t_)
            rec["n0"][at], rec["n1"][at] = self.fA[c_, t_, l_, 0], self.fA[c_, t_, l_, 1]
            rec["rhs"][at] = self.frhs[c_, t_, l_] - shift[s_, t_]
            rec["side"][at], rec["status"][at] = 1, 0
        se = [(s, t, i) for s, (_, segs) in enumerate(nodes) for t, i in segs.items()]
        if se:
            s_, t_, i_ = (x[:, None] for x in np.array(se, np.int64).T)
            at = (s_, Cb + C + np.arange(self.F)[None, :], t_)
            i_ = i_[:, 0]
            rec["n0"][at], rec["n1"][at] = seg.A[i_, :, 0], seg.A[i_, :, 1]
            rec["rhs"][at], rec["side"][at] = seg.b[i_], -1
            rec["status"][at] = np.where(seg.live[i_], 0, 1)
        return rec

    def _solve_batch(self, nodes):
        """One mpc_qp_kernel launch over the nodes: (u, X, cost, ok) host arrays.  The round's
        traffic is one pinned pack each way (records, goal, reference and executed controls up
        in one copy kernel; u, X, cost, status down in one, then a polled signal), on buffers
        cached per shape across frames (_RoundIO)."""
        from . import mpc
        S, T = len(nodes), self.T
        rec = self._records(nodes)
        io = _RoundIO.get(self, S, rec.shape[1])
        # this frame's model on the cached buffers (the shared model rows may hold another
        # tree's since this shape last ran)
        if io.frame is not self or (io.model is not None and io.model["frame"] is not self):
            io.set_frame(self)
        io.rec_h[...] = rec
        st, u, X, cost = io.run()
        st = st & ~mpc.QP_SKIPPED_ROWS
        self.stats["launches"] += 1
        self.stats["qps"] += S
        return u, X, cost, st == mpc.QP_OK

    # ---- feasibility of a node's optimum -----------------------------------------------------
    def _violations(self, X, faces, segs):
        """Per step t: the smallest (over the polytopes t may take) scaled violation of its
        rows, the polytope that attains it, and per (cell, t) the disjunction's violation under
        that polytope."""
        T, xy, seg = self.T, X[:self.T, :2], self.seg
        nrm = lambda r: 1.0 + np.abs(r)                      # noqa: E731
        opts = [False, True] if (seg is not None and seg.any_open) else [False]
        base_v, face_v = {}, {}
        for open_ in opts:                                   # S_t = M (open) or 0
            sh = self.M if open_ else 0.0
            if self.Cb:
                lhs = np.einsum("ctj,tj->ct", self.bn, xy)
                rhs = self.brhs + np.where(self.bsbig, sh, 0.0)
                v = np.where(self.bside == 1, rhs - lhs, lhs - rhs) / nrm(rhs)
                base_v[open_] = np.where(self.blive, v, -np.inf).max(0)
            else:
                base_v[open_] = np.full(T, -np.inf)
            if self.C:
                fv = (self.frhs - sh - np.einsum("ctlj,tj->ctl", self.fA, xy)) / nrm(self.frhs)
                fv = fv.min(-1)
                for (c, t), l in faces.items():
                    fv[c, t] = (self.frhs[c, t, l] - sh - self.fA[c, t, l] @ xy[t]) / nrm(
                        self.frhs[c, t, l])
                face_v[open_] = fv
            else:
                face_v[open_] = np.full((0, T), -np.inf)
        if seg is None:
            tv = np.maximum(base_v[False], face_v[False].max(0, initial=-np.inf))
            return tv, [None] * T, face_v[False]
        sv = np.einsum("ifj,tj->itf", seg.A, xy) - seg.b[:, None, :]
        sv = np.where(seg.live[:, None, :], sv / nrm(seg.b)[:, None, :], -np.inf).max(-1)
        per = np.empty((seg.I, T))                           # (polytope, t)
        for i in range(seg.I):
            o = bool(not seg.junction[i])
            per[i] = np.maximum(sv[i], np.maximum(base_v[o], face_v[o].max(0, initial=-np.inf)))
        for t, i in segs.items():
            keep = per[i, t]
            per[:, t] = np.inf
            per[i, t] = keep
        choice = np.argmin(per, 0)
        tv = per[choice, np.arange(T)]
        fv = np.stack([face_v[bool(not seg.junction[choice[t]]) and seg.any_open][:, t]
                       for t in range(T)], 1) if self.C else np.zeros((0, T))
        return tv, [int(i) for i in choice], fv

    def _violations_all(self, X, nodes):
        """_violations(X[s], *nodes[s]) for every node of a round at once (no road segments:
        the same operations on the same values, so the same bits; with segments, per node)."""
        if self.seg is not None:
            return [self._violations(Xi, f, g) for Xi, (f, g) in zip(X, nodes)]
        S, T = len(nodes), self.T
        xy = np.asarray(X)[:, :T, :2]
        nrm = lambda r: 1.0 + np.abs(r)                      # noqa: E731
        if self.Cb:
            lhs = np.einsum("ctj,stj->sct", self.bn, xy)
            rhs = self.brhs + np.where(self.bsbig, 0.0, 0.0)
            v = np.where(self.bside == 1, rhs - lhs, lhs - rhs) / nrm(rhs)
            base_v = np.where(self.blive, v, -np.inf).max(1)
        else:
            base_v = np.full((S, T), -np.inf)
        if self.C:
            fv = (self.frhs - 0.0 - np.einsum("ctlj,stj->sctl", self.fA, xy)) / nrm(self.frhs)
            fv = fv.min(-1)
            for s, (faces, _) in enumerate(nodes):
                for (c, t), l in faces.items():
                    fv[s, c, t] = (self.frhs[c, t, l] - 0.0 - self.fA[c, t, l] @ xy[s, t]) / nrm(
                        self.frhs[c, t, l])
        else:
            fv = np.full((S, 0, T), -np.inf)
        tv = np.maximum(base_v, fv.max(1, initial=-np.inf))
        return [(tv[s], [None] * T, fv[s]) for s in range(S)]

    def solve(self):
        """Returns dict(u, X, cost, faces (C, T), segments (T,) chosen polytope per t, nodes,
        launches) or None when the MILP is infeasible (the reference's CPLEX failure path)."""
        import heapq
        if self.seg is not None and self.seg.I == 0:
            return None                     # sum over an empty Omicron column >= 1 fails
        heap, seq, best = [], 0, None
        pending = [(({}, {}), -np.inf)]
        tie = lambda c: 1e-12 * (1 + abs(c))                # noqa: E731
        while pending:
            u, X, cost, ok = self._solve_batch([n for n, _ in pending])
            viol = self._violations_all(X, [n for n, _ in pending])
            for ((faces, segs), _), ui, Xi, ci, oki, vi in zip(pending, u, X, cost, ok, viol):
                self.stats["nodes"] += 1
                if not oki or (best is not None and ci >= best["cost"] - tie(best["cost"])):
                    continue
                tv, choice, fv = vi
                if tv.max() <= self.tol:                    # feasible for the MILP
                    fc = np.zeros((self.C, self.T), np.int64)
                    if self.C:
                        xy = Xi[:self.T, :2]
                        fc = np.argmin(self.frhs - np.einsum("ctlj,tj->ctl", self.fA, xy), -1)
                        for (c, t), l in faces.items():
                            fc[c, t] = l
                    best = dict(u=ui, X=Xi, cost=float(ci), faces=fc,
                                segments=None if self.seg is None else np.array(choice))
                    continue
                t = int(np.argmax(tv))
                kids = []
                if self.seg is not None and t not in segs:
                    for i in range(self.seg.I):
                        kids.append((faces, {**segs, t: i}))
                else:
                    v = fv[:, t].copy() if self.C else np.zeros(0)
                    for (c, tt) in faces:
                        if tt == t:
                            v[c] = -np.inf
                    if v.size and v.max() > self.tol:
                        c = int(np.argmax(v))
                        for l in range(self.L):
                            kids.append(({**faces, (c, t): l}, segs))
                    elif tv[t] <= 1e-6:                     # rows the QP holds, round-off
                        best = dict(u=ui, X=Xi, cost=float(ci), faces=None,
                                    segments=None if self.seg is None else np.array(choice))
                for kid in kids:
                    seq += 1
                    heapq.heappush(heap, (float(ci), seq, kid))
            if self.stats["nodes"] > self.max_nodes:
                raise RuntimeError(f"branch and bound: more than {self.max_nodes} nodes")
            pending = []
            while heap and len(pending) < self.batch:
                bound, _, kid = heapq.heappop(heap)
                if best is not None and bound >= best["cost"] - tie(best["cost"]):
                    heap.clear()                            # every remaining bound is larger
                    break
                pending.append((kid, bound))
        if best is None:
            return None
        best.update(nodes=self.stats["nodes"], launches=self.stats["launches"])
        return best


_MODEL_ROWS = 64          # scenes of the shared per-frame LTV model buffer (_RoundIO)
# CCMPC_MILP_ROUND_GRAPH=0: every round's launches issued one by one (A/B)
_ROUND_GRAPHS = os.environ.get("CCMPC_MILP_ROUND_GRAPH", "1") == "1"


class _RoundIO:
    """A branch-and-bound round's device side for S nodes of `cells` record cells: the batched
    PlanningQP, its inputs and outputs as pinned packs (step.Pack), the LTV model repeated S
    times on the device.  Cached per shape in the process (a frame's rounds and the next
    frames of the same shape reuse it; the tree runs on one host thread)."""
    _cache = {}

    @classmethod
    def get(cls, bnb, S, cells):
        key = (str(bnb.dev), S, cells, bnb.T, bnb.T_full, bnb.ref.shape[0], bnb.u_order,
               bytes(bnb.params), None if bnb.ltv is None else bnb.ltv[1:])
        io = cls._cache.get(key)
        if io is None:
            while len(cls._cache) >= 32:
                cls._cache.pop(next(iter(cls._cache)))
            io = cls._cache[key] = cls(bnb, S, cells)
        return io

    def __init__(self, bnb, S, cells):
        from . import mpc, step
        T, Tf, dev = bnb.T, bnb.T_full, bnb.dev
        f64, i32, i64 = torch.float64, torch.int32, torch.int64
        self.S, self.T, self.Tf, self.dev = S, T, Tf, dev
        nref = bnb.ref.shape[0]
        self.ltv = None if bnb.ltv is None else bnb.ltv[1:]      # (Ts, lon): fused rebuild
        self.inp = step.Pack([("gen", (2,), i64), ("rec", (S * cells, T, 32), torch.uint8),
                              ("goal", (S, 2), f64), ("ref", (S, nref, 2), f64),
                              ("uprev", (S, max(2 * (Tf - T), 1)), f64),
                              ("x0", (S, 4), f64)], dev)
        self.out = step.Pack([("u", (S, 2 * T), f64), ("X", (S, T, 4), f64), ("cost", (S,), f64),
                              ("status", (S,), i32), ("iters", (S,), i32)], dev)
        self.qp = mpc.PlanningQP([cells] * S, T, T_full=Tf, kind=mpc.REC_AFFINE_COMPACT,
                                 params=bnb.params, u_order=bnb.u_order, device=dev)
        o = self.out
        self.qp.u, self.qp.X, self.qp.cost = o.d("u"), o.d("X"), o.d("cost")
        self.qp.status, self.qp.iters = o.d("status"), o.d("iters")
        # the LTV model repeated per scene: rows of one buffer per (device, horizon) shared by
        # every round shape, so a frame fills it once, not once per shape (S <= 64)
        self.model = (_RoundIO._frame_model(dev, Tf) if S <= _MODEL_ROWS and self.ltv is None
                      else None)
        if self.model is not None:
            self.gamma, self.xbar = self.model["gamma"][:S], self.model["xbar"][:S]
        else:
            self.gamma = torch.empty((S, 4 * Tf, 2 * Tf), dtype=f64, device=dev)
            self.xbar = torch.empty((S, 4 * Tf), dtype=f64, device=dev)
        self.rec_h = self.inp.h("rec").reshape(-1).view(_GATHER).reshape(S, cells, T)
        self.flags = torch.zeros(2, dtype=i64, pin_memory=True)
        self._flags = self.flags.numpy()
        self.gen, self.frame = 0, None
        # the round's launches (copy-in, the solve, copy-out + signal) replay as one captured
        # graph from the second round of this shape on (the first runs them eagerly, which also
        # allocates everything the capture must not)
        self.graph, self.runs = None, 0

    def _enqueue(self):
        from . import _lib, engine
        lib, p, s = _lib.load(), engine._p, engine._stream()
        i, o = self.inp, self.out
        _lib.check(lib.ccmpc_copy_kernel_async(p(i.dev), p(i.host), i.nbytes, s),
                   "ccmpc_copy_async")
        self.qp.solve(self.gamma, self.xbar, i.d("goal"), i.d("ref"), i.d("rec"),
                      u_prev=i.d("uprev") if self.Tf > self.T else None,
                      ltv=None if self.ltv is None else (i.d("x0"),) + self.ltv)
        _lib.check(lib.ccmpc_copy_signal_async(p(o.host), p(o.dev), o.nbytes, p(self.flags),
                                               p(i.d("gen")), s), "ccmpc_copy_signal_async")

    _models = {}

    @classmethod
    def _frame_model(cls, dev, Tf):
        key = (str(dev), Tf)
        m = cls._models.get(key)
        if m is None:
            m = cls._models[key] = dict(
                frame=None,
                gamma=torch.empty((_MODEL_ROWS, 4 * Tf, 2 * Tf), dtype=torch.float64, device=dev),
                xbar=torch.empty((_MODEL_ROWS, 4 * Tf), dtype=torch.float64, device=dev))
        return m

    def set_frame(self, bnb):
        """The frame's LTV model (device copies), goal, reference and executed controls."""
        m = self.model
        if self.ltv is not None:            # the model is rebuilt in the launch from x_init
            self.inp.h("x0")[...] = bnb.ltv[0][None]
        elif m is None:
            self.gamma.copy_(bnb.gamma.expand(self.S, -1, -1))
            self.xbar.copy_(bnb.xbar.expand(self.S, -1))
        elif m["frame"] is not bnb:         # the first of this frame's round shapes
            m["gamma"].copy_(bnb.gamma.expand(_MODEL_ROWS, -1, -1))
            m["xbar"].copy_(bnb.xbar.expand(_MODEL_ROWS, -1))
            m["frame"] = bnb
        i = self.inp
        i.h("goal")[...] = bnb.goal
        i.h("ref")[...] = bnb.ref[None]
        if self.Tf > self.T:
            i.h("uprev")[...] = bnb.u_prev_h[None]
        self.frame = bnb

    def run(self):
        """Records (already in the pinned pack) up, the batched solve, the answer down; returns
        host copies (status, u, X, cost)."""
        from . import step
        i, o = self.inp, self.out
        if self.graph is None and self.runs >= 1 and _ROUND_GRAPHS:
            cap = torch.cuda.Stream(device=self.dev)
            torch.cuda.current_stream(self.dev).synchronize()
            cap.synchronize()
            self.graph = step.HipGraph(self.dev, self._enqueue, cap)
        self.gen += 1
        i.h("gen")[0] = self.gen
        if self.graph is not None:
            self.graph.replay()
        else:
            self._enqueue()
        self.runs += 1
        step.poll_word(self._flags, 0, self.gen, self.dev, "branch-and-bound round")
        return (o.h("status").copy(), o.h("u").copy(), o.h("X").copy(), o.h("cost").copy())


class BranchAndBound(MilpBnB):
    """v8's MILP (milp.BigMRows over the device L4 faces; road segments optional) from the
    planner's state: the LTV model about u = 0 from x_init (make_local_params), v8's objective
    (no reference term), U row-major.  solve() as MilpBnB's, with faces (C, T) the chosen
    face per (cell, t)."""

    def __init__(self, rows, T, x_init, goal, lon=3.7, Ts=0.5, params=None, batch=64, tol=1e-7,
                 max_nodes=100000, device="cuda", segments=None):
        from . import engine, mpc
        T = int(T)
        dev = engine.require_device(device)
        super().__init__(T, None, None, goal, params=params or v8_qp_params(),
                         u_order=mpc.U_ORDER_C, faces=(rows.A, rows.rhs), segments=segments,
                         M_big=rows.M_big, batch=batch, tol=tol, max_nodes=max_nodes,
                         device=dev, ltv=(x_init, Ts, lon))
