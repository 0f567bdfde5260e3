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
        l4 = scene.l4()
        rows = BigMRows(l4["A"].cpu().numpy(), l4["b"].cpu().numpy(), diag, T, self.M_big)
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
        """v8/__init__.py:755-873 with road boundaries off: the obstacle big-M rows over the
        device L4 faces, compute_objective, and the MILP solved by BranchAndBound on the GPU
        (CPLEX's role).  params: x_init [x, y, psi, v] (make_local_params' state; the LTV model
        is built about u = 0 on the device) and goal (2,) (compute_segs_polytopes_and_goal's,
        whose map reader is outside the path); diag as compute_obstacle_constraints reads it.
        Returns (AttrDict(cost, U_star, X_star, goal, A_union, b_union, vertices, segments=None),
        None), or with cost / U_star / X_star None and an InSimulationException where the
        reference's solve fails (:862-873)."""
        from .standins import AttrDict
        if self.road_boundary_constraints:
            raise NotImplementedError("the road-boundary variant needs the map reader's segment "
                                      "polytopes (Omicron binaries, v8/__init__.py:676-690)")
        rows, vertices, A_union, b_union = self.compute_obstacle_constraints(
            params, ovehicles, None, None, None, None)
        goal = np.asarray(params.goal, np.float64)
        T = self.control_horizon
        bnb = BranchAndBound(rows, T, params.x_init, goal, lon=self.ego_lon,
                             params=v8_qp_params(self.mpc_params_steer), device=self.device)
        sol = bnb.solve()
        self.last_bnb = dict(bnb.stats)
        out = AttrDict(cost=None, U_star=None, X_star=None, goal=goal, A_union=A_union,
                       b_union=b_union, vertices=vertices, segments=None)
        if sol is None:
            return out, planner.InSimulationException("Optimizer failed to find a solution")
        out.update(cost=sol["cost"], U_star=sol["u"].reshape(T, 2), X_star=sol["X"],
                   faces=sol["faces"])
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


class BranchAndBound:
    """The v8 MILP (obstacle big-M rows over the L4 faces, road boundaries off) solved exactly
    on the GPU: best-first branch and bound over the face choice per (cell, t).  A node fixes
    one face a_l . x_t >= b_l + diag per branched (cell, t); its relaxation is the convex QP
    with those rows alone (the unfixed binaries' big-M rows are vacuous at M_big = 1e4: the
    same relaxation CPLEX starts from), solved by mpc_qp_kernel.  Each round pops up to
    `batch` nodes and solves them as ONE batched launch (a node = a scene of C cells of T
    compact affine records; unfixed (cell, t) rows carry a nonzero status, so the kernel leaves
    them out).  A node whose optimum satisfies every disjunction is MILP-feasible (Delta = its
    satisfied faces) and becomes the incumbent if cheaper; otherwise its most violated
    (cell, t) is branched into the L faces; nodes whose bound (the parent's optimum) is not
    below the incumbent are pruned.  Deterministic: the same QP results give the same tree."""

    def __init__(self, rows, T, x_init, goal, lon=3.7, Ts=0.5, params=None, batch=64, tol=1e-7,
                 max_nodes=100000, device="cuda"):
        from . import engine, mpc
        self.dev = engine.require_device(device)
        self.T = int(T)
        self.A = np.asarray(rows.A, np.float64)[:, :self.T]
        self.rhs = np.asarray(rows.rhs, np.float64)[:, :self.T]
        self.C, self.L = self.A.shape[0], self.A.shape[2]
        self.goal = np.asarray(goal, np.float64).reshape(2)
        self.params = params or v8_qp_params()
        self.batch, self.tol, self.max_nodes = int(batch), float(tol), int(max_nodes)
        self.xbar, self.gamma = mpc.ltv(np.asarray(x_init, np.float64).reshape(1, 4), self.T,
                                        Ts=Ts, lon=lon)
        self._qp = {}
        # per (cell, t, l): the face row as a compact record (side +1: n . x_t >= rhs)
        c, t, l = np.meshgrid(np.arange(self.C), np.arange(self.T), np.arange(self.L),
                              indexing="ij")
        self._face = np.zeros((self.C, self.T, self.L), _GATHER)
        self._face["n0"], self._face["n1"] = self.A[..., 0], self.A[..., 1]
        self._face["rhs"], self._face["side"], self._face["t_tau"] = self.rhs, 1, t
        self.stats = dict(nodes=0, launches=0, qps=0)

    def _solve_batch(self, nodes):
        """One mpc_qp_kernel launch over the nodes: (u, X, cost, ok) host arrays."""
        from . import mpc
        S, C, T = len(nodes), self.C, self.T
        rec = np.zeros((S, C, T), _GATHER)
        rec["status"] = 1                                  # unfixed: left out by the kernel
        rec["t_tau"] = np.arange(T)
        for s, fixed in enumerate(nodes):
            for (c, t), l in fixed.items():
                rec[s, c, t] = self._face[c, t, l]
        qp = self._qp.get(S)
        if qp is None:
            qp = self._qp[S] = mpc.PlanningQP([C] * S, T, kind=mpc.REC_AFFINE_COMPACT,
                                              params=self.params, u_order=mpc.U_ORDER_C,
                                              device=self.dev)
        d_rec = torch.from_numpy(rec.view(np.uint8).reshape(S * C, T, 32)).to(self.dev)
        goal = torch.as_tensor(np.tile(self.goal, (S, 1)), device=self.dev)
        u, X, cost, status, _ = qp.solve(self.gamma.expand(S, -1, -1).contiguous(),
                                         self.xbar.expand(S, -1).contiguous(), goal,
                                         goal.reshape(S, 1, 2).contiguous(), d_rec)
        st = status.cpu().numpy() & ~mpc.QP_SKIPPED_ROWS
        self.stats["launches"] += 1
        self.stats["qps"] += S
        return u.cpu().numpy(), X.cpu().numpy(), cost.cpu().numpy(), st == mpc.QP_OK

    def solve(self):
        """Returns dict(u, X, cost, faces (C, T) chosen face per (cell, t), nodes, launches)
        or None when the MILP is infeasible (the reference's CPLEX failure path)."""
        import heapq
        heap, seq, best = [], 0, None
        pending = [({}, -np.inf)]                          # (fixed faces, parent bound)
        while pending or heap:
            # the next round: the `batch` most promising open nodes (pending are the root /
            # children whose QPs are not solved yet)
            nodes = pending[:self.batch]
            pending = pending[self.batch:]
            if not nodes:
                break
            u, X, cost, ok = self._solve_batch([f for f, _ in nodes])
            for (fixed, _), ui, Xi, ci, oki in zip(nodes, u, X, cost, ok):
                self.stats["nodes"] += 1
                if not oki:
                    continue                               # infeasible subproblem
                if best is not None and ci >= best["cost"] - 1e-12 * (1 + abs(best["cost"])):
                    continue
                slack = np.min(self.rhs - np.einsum("ctlj,tj->ctl", self.A, Xi[:, :2]), -1)
                viol = slack - self.tol * (1.0 + np.abs(self.rhs).max(-1))
                for key in fixed:                          # a fixed face holds (QP rows):
                    viol[key] = -np.inf                    # never branch on it again
                if viol.max() <= 0:                        # every disjunction holds
                    faces = np.argmin(self.rhs - np.einsum("ctlj,tj->ctl", self.A, Xi[:, :2]),
                                      axis=-1)
                    for (cc, t), l in fixed.items():
                        faces[cc, t] = l
                    best = dict(u=ui, X=Xi, cost=float(ci), faces=faces)
                    continue
                cc, t = np.unravel_index(int(np.argmax(viol)), viol.shape)
                for l in range(self.L):
                    child = dict(fixed)
                    child[(int(cc), int(t))] = l
                    seq += 1
                    heapq.heappush(heap, (float(ci), seq, child))
            if self.stats["nodes"] > self.max_nodes:
                raise RuntimeError(f"branch and bound: more than {self.max_nodes} nodes")
            # refill: best-first over the open nodes, bounds pruned against the incumbent
            while heap and len(pending) < self.batch:
                bound, _, child = heapq.heappop(heap)
                if best is not None and bound >= best["cost"] - 1e-12 * (1 + abs(best["cost"])):
                    heap.clear()                           # every remaining bound is larger
                    break
                pending.append((child, bound))
        if best is None:
            return None
        best.update(nodes=self.stats["nodes"], launches=self.stats["launches"])
        return best

