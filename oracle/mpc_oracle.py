"""NumPy/SciPy restatement of the planning step's QP (the caller of the path).

TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py.  The CPU checker of ccmpc_mpc_ltv /
ccmpc_mpc_qp and the CPU baseline bench.py times beside them.

Reference paths are relative to /root/reference/collect/in_simulation/ unless stated.

* LTV model: dynamics/bicycle_v2.py (VehicleModel, :132-308).  The reference drives it through
  python-control 0.9.1 (py38trajectron.freeze.txt), absent here; that package's two calls are
  restated with the SciPy routines it delegates to: ``input_output_response`` integrates the
  nonlinear system with ``scipy.integrate.solve_ivp(method='RK45')`` at the output times, and
  ``matlab.c2d`` (``StateSpace.sample(Ts, 'zoh')``) is ``scipy.signal.cont2discrete(...,
  method='zoh')``.
* QP: midlevel/v8ideal/__init__.py do_highlevel_control :2850-2930 (state map, control bounds),
  compute_state_constraints :610-626, the half-spaces of :926-939 (Minkowski) and :1503-1515
  (affine, S_big = 0 when road_boundary_constraints is off, :1396-1416), and
  compute_objective_referenceTraj :2478-2507.  cvxpy (unpinned in the freeze file, absent here)
  builds ``U = cp.reshape(u, (T, nu))`` column-major by default: U_t = (u[t], u[T + t]).
* Solve: the reference hands the problem to CPLEX (absent).  The oracle solves the same convex
  QP with SciPy's SLSQP, then polishes on the detected active set (equality-constrained KKT
  solve) and certifies the result with the KKT conditions -- a solver-independent check.
  Parity against CPLEX itself is unpinned (no CPLEX output ships with the reference).
"""
import math

import numpy as np
import scipy.integrate
import scipy.interpolate
import scipy.linalg
import scipy.optimize
import scipy.signal

# v8ideal/__init__.py:86-109 (__make_global_params) and :275-278 (steptime)
DEFAULT_PARAMS = dict(w_final=6.0, w_ref=3.0, w_accel=0.5, w_joint=0.2, w_turning=1.0,
                      w_ch_accel=0.5, w_ch_joint=0.1, w_ch_turning=2.0,
                      min_a=-7.0, max_a=4.0, max_v=10.0,
                      max_delta=0.5 * math.radians(70.0))  # 0.5 * limit_delta (CARLA wheel)
STEPTIME = 0.5


# ----------------------------------------------------------------------------------------
# dynamics/bicycle_v2.py
# ----------------------------------------------------------------------------------------
def get_beta(delta, l_r=0.5, L=1.0):                                   # :13-17
    return delta if l_r == L else math.atan((l_r / L) * math.tan(delta))


def get_dbeta_ddelta(delta, l_r=0.5, L=1.0):                           # :19-24
    if l_r == L:
        return 1
    tan2 = math.tan(delta) ** 2
    return (1 + tan2) / ((L / l_r) + (l_r / L) * tan2)


def bicycle_kinematics(t, x, u, params):                               # :26-40
    l_r = params.get("l_r", 0.5)
    L = params.get("L", 1)
    delta = params.get("delta", 0)  # the 'delta' parameter, never set: beta = 0
    psi, v = x[2], x[3]
    u_1, u_2 = u[0], u[1]
    beta = get_beta(delta, l_r=l_r, L=L)
    return np.array([v * math.cos(psi + beta), v * math.sin(psi + beta),
                     (v / L) * math.cos(beta) * math.tan(u_2), u_1])


def get_state_matrix(z, u, l_r=0.5, L=1.0):                            # :103-115
    x, y, psi, v = z
    a, delta = u
    beta = get_beta(delta, l_r=l_r, L=L)
    df3_dv = (1 / L) * math.cos(beta) * math.tan(delta)
    return np.array([[0, 0, -v * math.sin(psi + beta), math.cos(psi + beta)],
                     [0, 0, v * math.cos(psi + beta), math.sin(psi + beta)],
                     [0, 0, 0, df3_dv],
                     [0, 0, 0, 0]], dtype=np.float64)


def get_input_matrix(z, u, l_r=0.5, L=1.0):                            # :117-130
    x, y, psi, v = z
    a, delta = u
    beta = get_beta(delta, l_r=l_r, L=L)
    dbeta = get_dbeta_ddelta(delta, l_r=l_r, L=L)
    tan2 = math.tan(delta) ** 2
    return np.array([[0, -v * math.sin(psi + beta) * dbeta],
                     [0, v * math.cos(psi + beta) * dbeta],
                     [0, (v / L) * (math.cos(beta) * (1 + tan2)
                                    - math.sin(beta) * math.tan(delta) * dbeta)],
                     [1, 0]], dtype=np.float64)


def input_output_response(params, timestamps, U, x0):
    """control.input_output_response for a continuous NonlinearIOSystem (control 0.9.1):
    inputs linearly interpolated between the given times, solve_ivp RK45 evaluated at them."""
    ufun = scipy.interpolate.interp1d(timestamps, U, fill_value="extrapolate")

    def rhs(t, x):
        return bicycle_kinematics(t, x, ufun(t), params)

    sol = scipy.integrate.solve_ivp(rhs, (timestamps[0], timestamps[-1]), x0,
                                    t_eval=timestamps, method="RK45", vectorized=False)
    return sol.y  # (4, T + 1)


class VehicleModel:
    """bicycle_v2.py:132-308 with python-control's two calls restated (module docstring)."""

    def __init__(self, T, Ts, l_r=0.5, L=1.0):
        self.T, self.Ts, self.l_r, self.L = T, Ts, l_r, L
        self.timestamps = np.linspace(0, Ts * T, T + 1)
        self.params = {"l_r": l_r, "L": L}

    def states_from_control(self, x_init, U):                          # :176-198
        U_pad = np.concatenate((U, U[-1][None]))
        return input_output_response(self.params, self.timestamps, U_pad.T,
                                     np.asarray(x_init, np.float64)).T

    def get_nominal_trajectory(self, x_init, u_init):                  # :200-222
        U_bar = np.repeat(np.asarray(u_init, np.float64)[None], self.T, axis=0)
        return self.states_from_control(x_init, U_bar), U_bar

    def get_discrete_time_ltv(self, x_init, u_init):                   # :224-258
        X_bar, U_bar = self.get_nominal_trajectory(x_init, u_init)
        C = np.array([[1, 0, 0, 0], [0, 1, 0, 0]], dtype=np.float64)
        D = np.zeros((2, 2))
        As, Bs = [], []
        for i in range(self.T):
            A = get_state_matrix(X_bar[i], U_bar[i], l_r=self.l_r, L=self.L)
            B = get_input_matrix(X_bar[i], U_bar[i], l_r=self.l_r, L=self.L)
            Ad, Bd, _, _, _ = scipy.signal.cont2discrete((A, B, C, D), self.Ts, method="zoh")
            As.append(Ad)
            Bs.append(Bd)
        return X_bar, U_bar, As, Bs

    def get_optimization_ltv(self, x_init, u_init):                    # :260-308
        X_bar, U_bar, As, Bs = self.get_discrete_time_ltv(x_init, u_init)
        nx, nu = Bs[0].shape
        T = self.T
        B_bar = scipy.linalg.block_diag(*Bs)
        A_bar = np.eye(T * nx)
        if T > 1:
            A_bar[4:, :(T - 1) * nx] -= scipy.linalg.block_diag(*As[1:])
        Gamma = np.linalg.solve(A_bar, B_bar)
        return X_bar[1:].ravel(), U_bar.ravel(), Gamma, nx, nu


# ----------------------------------------------------------------------------------------
# the QP of do_highlevel_control
# ----------------------------------------------------------------------------------------
def u_index(t, c, T, order="F"):
    """U[t, c] of U = reshape(u, (T, 2)); order 'F' is cvxpy's default (:2894)."""
    return t + c * T if order == "F" else 2 * t + c


def obstacle_rows(records, kind, T):
    """(t, a, b) with a . x_t <= b for every record with status 0 (the reference's
    (A, b) = (-n, -d) for side +1, (n, d) for side -1, :926-939; affine rhs, :1503-1515)."""
    rows = []
    for r in records:
        if isinstance(r, dict):          # ccmpc_oracle generator records (always status 0)
            if "tau" in r:
                t, d = int(r["t"]), float(r["d"])
            else:
                t, d = int(r["t"]), float(r["rhs"])
            n = np.asarray(r["n"], np.float64)
            rows.append((t, -n, -d) if int(r["side"]) == 1 else (t, n, d))
            continue
        if int(r["status"]) != 0:
            continue
        if kind == "halfspace":
            t = int(r["t_tau"]) >> 16
            d = float(r["d"])
        else:
            t = int(r["t"])
            d = float(r["rhs"])
        n = np.array([float(r["n0"]), float(r["n1"])])
        if int(r["side"]) == 1:
            rows.append((t, -n, -d))
        else:
            rows.append((t, n, d))
    return rows


def state_map(Gamma_full, xbar_full, T, T_full, u_prev=None, ubar_full=None):
    """x = Gamma_f (u - u_bar[:nu T]) + x_bar[:nx T] (+ Gamma_p u_prev) (:2858-2891).
    Returns (Gf, c) with x = Gf u + c, x of shape (4T,)."""
    nx, nu = 4, 2
    T_prev = T_full - T
    row_off, col_off = nx * T_prev, nu * T_prev
    x_bar = xbar_full[row_off:]
    u_bar = (np.zeros(nu * T_full) if ubar_full is None else ubar_full)[col_off:]
    Gamma = Gamma_full[row_off:, :]
    Gf = Gamma[:nx * T, col_off:col_off + nu * T]
    c = x_bar[:nx * T] - Gf @ u_bar[:nu * T]
    if T_prev:
        c = c + Gamma[:nx * T, :col_off] @ np.asarray(u_prev, np.float64)
    return Gf, c


def objective_value(u, Gf, c, T, goal, ref_traj, p, order="F"):
    """compute_objective_referenceTraj (:2478-2507) evaluated as written."""
    X = (Gf @ u + c).reshape(T, 4)
    U = np.array([[u[u_index(t, 0, T, order)], u[u_index(t, 1, T, order)]] for t in range(T)])
    R1 = np.array([[p["w_accel"], p["w_joint"]], [p["w_joint"], p["w_turning"]]])
    R2 = np.array([[p["w_ch_accel"], p["w_ch_joint"]], [p["w_ch_joint"], p["w_ch_turning"]]])
    cost = p["w_final"] * (X[-1, 0] - goal[0]) ** 2 + p["w_final"] * (X[-1, 1] - goal[1]) ** 2
    for t in range(T):
        r = ref_traj[t] if t < len(ref_traj) else ref_traj[-1]
        cost += p["w_ref"] * (X[t, 0] - r[0]) ** 2 + p["w_ref"] * (X[t, 1] - r[1]) ** 2
    cost += sum(U[t] @ R1 @ U[t] for t in range(T))
    cost += sum((U[t] - U[t - 1]) @ R2 @ (U[t] - U[t - 1]) for t in range(1, T))
    return float(cost)


def assemble_qp(Gf, c, T, goal, ref_traj, rows, p, order="F"):
    """Dense form  min 1/2 u^T H u + f^T u + k  s.t.  G u <= h  of the reference's problem."""
    n = 2 * T
    Pxy = [Gf[4 * t:4 * t + 2] for t in range(T)]
    H = np.zeros((n, n))
    f = np.zeros(n)
    k = 0.0
    for t in range(T):
        r = np.asarray(ref_traj[t] if t < len(ref_traj) else ref_traj[-1], np.float64)
        cxy = c[4 * t:4 * t + 2]
        terms = [(p["w_ref"], r)]
        if t == T - 1:
            terms.append((p["w_final"], np.asarray(goal, np.float64)))
        for wgt, target in terms:
            H += 2.0 * wgt * Pxy[t].T @ Pxy[t]
            f += 2.0 * wgt * Pxy[t].T @ (cxy - target)
            k += wgt * float((cxy - target) @ (cxy - target))
    R1 = np.array([[p["w_accel"], p["w_joint"]], [p["w_joint"], p["w_turning"]]])
    R2 = np.array([[p["w_ch_accel"], p["w_ch_joint"]], [p["w_ch_joint"], p["w_ch_turning"]]])
    E = [np.zeros((2, n)) for _ in range(T)]
    for t in range(T):
        for cc in range(2):
            E[t][cc, u_index(t, cc, T, order)] = 1.0
    for t in range(T):
        H += 2.0 * E[t].T @ R1 @ E[t]
    for t in range(1, T):
        D = E[t] - E[t - 1]
        H += 2.0 * D.T @ R2 @ D
    G, h = [], []
    for j in range(n):  # control bounds (:2874-2878): interleaved (accel, steer) per step,
        cc = j % 2      # min_u = vstack((full(T, min_a), full(T, -max_delta))).T.ravel()
        hi = p["max_a"] if cc == 0 else p["max_delta"]
        lo = p["min_a"] if cc == 0 else -p["max_delta"]
        e = np.zeros(n)
        e[j] = 1.0
        G.append(e)
        h.append(hi)
        G.append(-e)
        h.append(-lo)
    for t in range(T):  # 0 <= v_t <= max_v (:610-626)
        gv = Gf[4 * t + 3]
        G.append(gv)
        h.append(p["max_v"] - c[4 * t + 3])
        G.append(-gv)
        h.append(c[4 * t + 3])
    for t, a, b in rows:
        G.append(a @ Pxy[t])
        h.append(b - a @ c[4 * t:4 * t + 2])
    return H, f, k, np.array(G), np.array(h)


def kkt_residuals(H, f, G, h, u, lam=None):
    """Max violations of primal feasibility, and (given multipliers, else the least-squares
    nonnegative ones on the active set) of stationarity and complementarity."""
    g = G @ u - h
    scale_h = 1.0 + np.max(np.abs(h))
    prim = max(0.0, float(np.max(g))) / scale_h
    act = g > -1e-7 * scale_h
    grad = H @ u + f
    if lam is None:
        lam = np.zeros(len(h))
        if act.any():
            sol = scipy.optimize.nnls(G[act].T, -grad)[0]
            lam[act] = sol
    stat = float(np.max(np.abs(grad + G.T @ lam))) / (1.0 + np.max(np.abs(f)))
    comp = float(np.max(np.abs(lam * g))) / scale_h
    return prim, stat, comp, lam


def is_feasible(G, h):
    """Phase-1 check with SciPy's HiGHS LP: does {u : G u <= h} have a point?"""
    lp = scipy.optimize.linprog(np.zeros(G.shape[1]), A_ub=G, b_ub=h,
                                bounds=[(None, None)] * G.shape[1], method="highs")
    return lp.status == 0


def solve_qp(H, f, G, h, tol=1e-12):
    """SLSQP from u = 0, then an equality-constrained KKT solve on the detected active set
    (drop rows whose multiplier comes out negative, repeat).  Returns (u, lam, active)."""
    n = len(f)
    cons = {"type": "ineq", "fun": lambda u: h - G @ u, "jac": lambda u: -G}
    res = scipy.optimize.minimize(lambda u: 0.5 * u @ H @ u + f @ u, np.zeros(n),
                                  jac=lambda u: H @ u + f, constraints=[cons],
                                  method="SLSQP", options=dict(ftol=tol, maxiter=1000))
    u = res.x
    scale_h = 1.0 + np.max(np.abs(h))
    active = list(np.nonzero(G @ u - h > -1e-6 * scale_h)[0])
    lam = np.zeros(len(h))
    for _ in range(2 * len(h) + 1):
        if active:
            Ga = G[active]
            # linearly independent subset (the problem is strictly convex, rows may repeat)
            _, _, piv = scipy.linalg.qr(Ga.T, pivoting=True, mode="economic")
            rank = np.linalg.matrix_rank(Ga)
            keep = sorted(int(i) for i in piv[:rank])
            Ga = Ga[keep]
            idx = [active[i] for i in keep]
            K = np.block([[H, Ga.T], [Ga, np.zeros((len(idx), len(idx)))]])
            sol = np.linalg.solve(K, np.concatenate((-f, h[idx])))
            u_try, l_try = sol[:n], sol[n:]
        else:
            idx, u_try, l_try = [], np.linalg.solve(H, -f), np.zeros(0)
        viol = G @ u_try - h
        if l_try.size and l_try.min() < -1e-10:
            active = [i for i, lv in zip(idx, l_try) if lv >= -1e-10]
            continue
        if viol.max() > 1e-9 * scale_h:
            active = sorted(set(idx) | {int(np.argmax(viol))})
            continue
        u = u_try
        lam = np.zeros(len(h))
        lam[idx] = l_try
        active = idx
        break
    return u, lam, active


def solve_step(Gamma_full, xbar_full, T, T_full, goal, ref_traj, records, kind, p,
               u_prev=None, order="F"):
    """One planning step's QP: (u*, X*, cost, H, f, G, h, lam)."""
    Gf, c = state_map(Gamma_full, xbar_full, T, T_full, u_prev=u_prev)
    rows = obstacle_rows(records, kind, T)
    H, f, k, G, h = assemble_qp(Gf, c, T, goal, ref_traj, rows, p, order=order)
    if not is_feasible(G, h):  # CPLEX fails -> InSimulationException (:3099-3110)
        return dict(feasible=False, H=H, f=f, k=k, G=G, h=h, Gf=Gf, c=c)
    u, lam, active = solve_qp(H, f, G, h)
    X = (Gf @ u + c).reshape(T, 4)
    return dict(feasible=True, u=u, X=X,
                cost=objective_value(u, Gf, c, T, goal, ref_traj, p, order=order),
                H=H, f=f, k=k, G=G, h=h, lam=lam, active=active, Gf=Gf, c=c)


# ----------------------------------------------------------------------------------------
# v8's MILP planner (midlevel/v8/__init__.py): the big-M obstacle disjunction over the L4
# faces (:692-724) and compute_objective (:727-753), road boundaries off (S_big = 0; the
# reference's own `np.zeros(T, L, dtype=float)` there raises, ccmpc/milp.py), solved exactly
# by branch and bound over the face choice per (cell, t) -- the problem CPLEX solves at
# :769-838 (CPLEX itself is absent; parity with its output is unpinned).
# ----------------------------------------------------------------------------------------
# v8/__init__.py:73-109 (__make_global_params)
V8_PARAMS = dict(w_final=3.0, w_ch_accel=0.5, w_ch_turning=2.0, w_ch_joint=0.1, w_accel=0.5,
                 w_turning=1.0, w_joint=0.2, min_a=-7.0, max_a=3.5, max_v=10.0,
                 max_delta=0.5 * math.radians(70.0))


def v8_compute_objective(X, U, goal, p=V8_PARAMS):
    """v8/__init__.py:727-753 as written (util.pairwise = consecutive pairs), numeric."""
    cost = p["w_final"] * (X[-1, 0] - goal[0]) ** 2 + p["w_final"] * (X[-1, 1] - goal[1]) ** 2
    for u1, u2 in zip(U[:-1, 0], U[1:, 0]):
        cost += p["w_ch_accel"] * (u1 - u2) * (u1 - u2)
    for u1, u2 in zip(U[:-1, 1], U[1:, 1]):
        cost += p["w_ch_turning"] * (u1 - u2) * (u1 - u2)
    for u1, u2 in zip(U[:-1], U[1:]):
        d = u1 - u2
        cost += p["w_ch_joint"] * d[0] * d[1]
    cost += p["w_accel"] * np.sum(U[:, 0] ** 2)
    cost += p["w_turning"] * np.sum(U[:, 1] ** 2)
    cost += 2.0 * p["w_joint"] * np.sum(U[:, 0] * U[:, 1])
    return float(cost)


def v8_qp_params(p=V8_PARAMS):
    """v8's objective in assemble_qp's form: no reference term (w_ref = 0), R1 as v8ideal's,
    and R2's off-diagonal w_ch_joint / 2 (v8 adds w_ch_joint du_0 du_1 once, a quadratic form
    counts the off-diagonal twice).  U = u.reshape(T, nu) of an object array: row-major."""
    q = dict(p)
    q.update(w_ref=0.0, w_ch_joint=0.5 * p["w_ch_joint"])
    return q


def _face_rows(fixed, A, rhs):
    """Rows (t, a, b) in obstacle_rows' `a . x_t <= b` form of the fixed faces: the face
    a_l . x_t >= rhs_l becomes (-a_l) . x_t <= -rhs_l."""
    return [(t, -A[c, t, l], -rhs[c, t, l]) for (c, t), l in sorted(fixed.items())]


def disjunction_slack(A, rhs, X):
    """(C, T): min over faces of rhs_l - a_l . x_t -- > 0 where the ego position lies inside
    every face (the disjunction violated), <= 0 where some face holds."""
    xy = np.asarray(X)[:, :2]
    return np.min(rhs - np.einsum("ctlj,tj->ctl", A, xy[:A.shape[1]]), axis=-1)


def _node_qp(Gf, c, T, goal, A, rhs, fixed, p, order):
    H, f, k, G, h = assemble_qp(Gf, c, T, goal, np.asarray(goal).reshape(1, 2),
                                _face_rows(fixed, A, rhs), p, order=order)
    if not is_feasible(G, h):
        return None
    u, lam, _ = solve_qp(H, f, G, h)
    return dict(u=u, cost=float(0.5 * u @ H @ u + f @ u + k), X=(Gf @ u + c).reshape(T, 4))


def milp_bnb(Gamma_full, xbar_full, T, goal, A, rhs, p=None, order="C", tol=1e-7,
             max_nodes=20000):
    """The v8 MILP's exact optimum by best-first branch and bound: a node fixes one face per
    branched (cell, t); its relaxation is the convex QP with those face rows only (the big-M
    rows of the unfixed binaries are vacuous at M_big = 1e4); a node whose optimum satisfies
    every disjunction is feasible for the MILP (Delta = its satisfied faces); else the most
    violated (cell, t) is branched into its L faces.  Returns dict(u, X, cost, faces (C, T),
    nodes) or None (infeasible)."""
    import heapq
    p = v8_qp_params() if p is None else p
    Gf, c = state_map(Gamma_full, xbar_full, T, T)
    A, rhs = np.asarray(A, float)[:, :T], np.asarray(rhs, float)[:, :T]
    best, nodes, heap, seq = None, 0, [], 0
    root = _node_qp(Gf, c, T, goal, A, rhs, {}, p, order)
    if root is None:
        return None
    heapq.heappush(heap, (root["cost"], seq, {}, root))
    while heap:
        bound, _, fixed, sol = heapq.heappop(heap)
        nodes += 1
        if nodes > max_nodes:
            raise RuntimeError("milp_bnb: node limit")
        if best is not None and bound >= best["cost"] - 1e-12 * (1 + abs(best["cost"])):
            continue
        slack = disjunction_slack(A, rhs, sol["X"])
        scale = tol * (1.0 + np.abs(rhs).max(-1))
        viol = slack - scale
        for key in fixed:                  # the node's QP enforces its fixed faces
            viol[key] = -np.inf
        if viol.max() <= 0:
            faces = np.argmin(rhs - np.einsum("ctlj,tj->ctl", A, sol["X"][:, :2]), axis=-1)
            for (cc, t), l in fixed.items():
                faces[cc, t] = l
            best = dict(sol, faces=faces)
            continue
        cc, t = np.unravel_index(int(np.argmax(viol)), viol.shape)
        for l in range(A.shape[2]):
            child = dict(fixed)
            child[(int(cc), int(t))] = l
            s = _node_qp(Gf, c, T, goal, A, rhs, child, p, order)
            if s is None:
                continue
            seq += 1
            heapq.heappush(heap, (s["cost"], seq, child, s))
    if best is not None:
        best["nodes"] = nodes
    return best


def milp_enumerate(Gamma_full, xbar_full, T, goal, A, rhs, p=None, order="C"):
    """Every face assignment (L^(C T) convex QPs): the exact optimum for tiny problems, an
    independent check of milp_bnb.  Returns dict(u, X, cost, faces) or None."""
    import itertools
    p = v8_qp_params() if p is None else p
    Gf, c = state_map(Gamma_full, xbar_full, T, T)
    A, rhs = np.asarray(A, float)[:, :T], np.asarray(rhs, float)[:, :T]
    C, L = A.shape[0], A.shape[2]
    keys = [(cc, t) for cc in range(C) for t in range(T)]
    best = None
    for combo in itertools.product(range(L), repeat=len(keys)):
        fixed = dict(zip(keys, combo))
        s = _node_qp(Gf, c, T, goal, A, rhs, fixed, p, order)
        if s is not None and (best is None or s["cost"] < best["cost"]):
            best = dict(s, faces=np.array(combo).reshape(C, T))
    return best


# ----------------------------------------------------------------------------------------
# Road boundaries on (road_boundary_constraints=True): the Omicron binaries of v8's
# do_highlevel_control (v8/__init__.py:676-702) and v8ideal's (v8ideal/__init__.py:738-758,
# :2906-2916).  Per segment polytope i (A_i x <= b_i, road.py:639-678) and step t:
#     A_i . X[t, :2] - M_big (1 - Omicron[i, t]) <= b_i,     sum_i Omicron[i, t] >= 1
# and S_t = M_big * sum_i Omicron[i, t] over the non-junction polytopes (segments.mask False),
# added to the obstacle rows: v8's face rows (a . x + M (1 - Delta) + S_t >= b + diag) and, in
# v8ideal, the affine (:1503-1515) and scale-ideal (:2394-2414) rows, both sides
# (n . x >= d + g + S_t, n . x <= d - g + S_t as written); the Minkowski (:926-939) and robust
# (:1828-1849) generators leave S out.  Enumerated literally here: every non-empty Omicron[:, t]
# subset, every unchosen row kept with its + M relaxation.
# ----------------------------------------------------------------------------------------
def road_rows(base, faces, segs, mask, M, seg_choice, face_choice, T):
    """obstacle_rows-form rows (t, a, b: a . x_t <= b) of one assignment.  base: rows dicts
    (t, n, rhs, side +1 '>=' / -1 '<=', sbig); faces (A (C, T, L, 2), rhs (C, T, L)) or None;
    segs [(A_i, b_i)], mask (I,); seg_choice {t: tuple of chosen i} (None without segments);
    face_choice {(c, t): l}."""
    S = np.zeros(T)
    if segs is not None:
        for t in range(T):
            S[t] = M * sum(1 for i in seg_choice[t] if not mask[i])
    rows = []
    for r in base:
        t = int(r["t"])
        b = float(r["rhs"]) + (S[t] if r.get("sbig", False) else 0.0)
        n = np.asarray(r["n"], np.float64)
        rows.append((t, -n, -b) if int(r["side"]) == 1 else (t, n, b))
    if faces is not None:
        A, rhs = faces
        C, _, L = rhs.shape
        for c in range(C):
            for t in range(T):
                for l in range(L):      # a . x + M (1 - delta) + S >= rhs
                    relax = 0.0 if face_choice[(c, t)] == l else M
                    rows.append((t, -A[c, t, l], -(rhs[c, t, l] - relax - S[t])))
    if segs is not None:
        for t in range(T):
            for i, (Ai, bi) in enumerate(segs):
                relax = 0.0 if i in seg_choice[t] else M
                for f in range(len(bi)):
                    rows.append((t, np.asarray(Ai[f], np.float64), float(bi[f]) + relax))
    return rows


def _road_node(Gf, c, T, goal, ref, rows, p, order):
    H, f, k, G, h = assemble_qp(Gf, c, T, goal, ref, rows, p, order=order)
    if not is_feasible(G, h):
        return None
    u, _, _ = solve_qp(H, f, G, h)
    return dict(u=u, cost=float(0.5 * u @ H @ u + f @ u + k), X=(Gf @ u + c).reshape(T, 4))


def road_milp_enumerate(Gamma_full, xbar_full, T, goal, ref, p, base=(), faces=None, segs=None,
                        mask=None, M=10_000.0, order="F", T_full=None, u_prev=None,
                        subsets=True):
    """The MILP's optimum over every assignment: Omicron[:, t] any non-empty subset (subsets)
    or one polytope, Delta one face per (cell, t).  Returns dict(u, X, cost, segs, faces) or
    None (infeasible: no polytope, or no assignment with a feasible QP)."""
    import itertools
    Gf, c = state_map(Gamma_full, xbar_full, T, T_full or T, u_prev=u_prev)
    if segs is not None and len(segs) == 0:
        return None                    # sum over an empty Omicron column >= 1
    if segs is None:
        seg_opts = [None]
    elif subsets:
        I = len(segs)
        seg_opts = [s for k in range(1, I + 1) for s in itertools.combinations(range(I), k)]
    else:
        seg_opts = [(i,) for i in range(len(segs))]
    keys = []
    if faces is not None:
        C, _, L = faces[1].shape
        keys = [(cc, t) for cc in range(C) for t in range(T)]
    best = None
    for sc in itertools.product(seg_opts, repeat=T):
        seg_choice = dict(enumerate(sc))
        for fc in itertools.product(*(range(faces[1].shape[2]) for _ in keys)):
            face_choice = dict(zip(keys, fc))
            rows = road_rows(base, faces, segs, mask, M, seg_choice, face_choice, T)
            s = _road_node(Gf, c, T, goal, ref, rows, p, order)
            if s is not None and (best is None or s["cost"] < best["cost"] - 1e-12):
                best = dict(s, segs=sc, faces=dict(face_choice))
    return best
