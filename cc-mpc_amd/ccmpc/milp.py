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
