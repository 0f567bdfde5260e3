"""NumPy restatement of the v8ideal Monte-Carlo prediction + MVOE chance-constraint path.

TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py.  This module is the CPU checker for the
HIP path and the CPU baseline timed by bench.py.  It must never be imported by the product.

Reference paths below are relative to /root/reference/collect/in_simulation/midlevel/.
The restatement is loop-faithful on purpose (it is also the timed CPU baseline): per-cell,
per-(t, tau) Python loops, np.cov with ddof=1, strided ``poseData[t::Tpred]`` views over a
vstacked (N*T, 2) array, exactly as the reference walks its data.
"""
import numpy as np
import scipy.linalg
import scipy.spatial
import scipy.stats

from . import philox

R_COLLISION = 3.4          # v8ideal/__init__.py:795 / :1394  (EV radius + OV radius)
TARGET_P = 0.9999          # v8ideal/__init__.py:912
EPS_TOTAL = 0.05           # v8ideal/__init__.py:2920
FILTER_PMF = 0.1           # ovehicle.py:26
N_IDEAL = 1_000_000        # v8ideal/__init__.py:2640


# ----------------------------------------------------------------------------------------
# makeconstraint.py math kernels
# ----------------------------------------------------------------------------------------
def compute_mvoe(Sigma1, Sigma2, tol=1e-8, maxiter=1000):
    """MVOE of the Minkowski sum of two centred ellipsoids (v8ideal/makeconstraint.py:7-38).

    Eigenvalues of Sigma1^{-1} Sigma2 drive a scalar fixed point for beta; the outer shape is
    (1 + 1/beta) Sigma1 + (1 + beta) Sigma2.  Returns (beta, Q, iterations).
    """
    lam = np.linalg.eigvals(scipy.linalg.solve(Sigma1, Sigma2)).real
    beta = 1.0
    it = 0
    while it < maxiter:
        it += 1
        nxt = np.sqrt(np.sum(1.0 / (1.0 + beta * lam)) / np.sum(lam / (1.0 + beta * lam)))
        converged = abs(nxt - beta) < tol
        beta = nxt
        if converged:
            break
    Q = (1 + 1.0 / beta) * Sigma1 + (1 + beta) * Sigma2
    return beta, Q, it


def predict_moments(p_t_tau):
    """4xN rows (x_t, y_t, x_tau, y_tau) -> (cov_infer, cov_mu, cov_t)
    (v8ideal/makeconstraint.py:41-70): Schur complement of the tau block."""
    C = np.cov(p_t_tau)
    c_t = C[0:2, 0:2]
    c_x = C[0:2, 2:4]
    c_xT = C[2:4, 0:2]
    c_tau = C[2:4, 2:4]
    cov_mu = c_x @ np.linalg.inv(c_tau) @ c_xT
    return c_t - cov_mu, cov_mu, c_t


def tangent_lines_of_slope_m(mu, Sigma, c, m):
    """Both slope-m tangents of (x-mu)^T Sigma^{-1} (x-mu) = c^2 (makeconstraint.py:134-162)."""
    n = np.array([-m, 1.0])
    q = float(n @ (Sigma @ n))
    if q <= 0:
        return []
    centre = float(n @ mu)
    half = c * np.sqrt(q)
    return [(n, centre + half), (n, centre - half)]


def distance_point_to_line(n, d, a):
    """|n.a - d| / ||n|| (makeconstraint.py:165-173)."""
    return abs(float(n @ a) - d) / np.linalg.norm(n)


def choose_closest_tangent(mu, Sigma, c, m, a, const_idx=None):
    """Pick the tangent closer to point a; strict '<' so index 0 wins ties
    (makeconstraint.py:176-207).  Returns (n, d, which) or a 4-tuple of None."""
    cands = tangent_lines_of_slope_m(mu, Sigma, c, m)
    if not cands:
        return (None, None, None, None)
    if const_idx is None:
        pick, best = None, np.inf
        for idx, (n, d) in enumerate(cands):
            dist = distance_point_to_line(n, d, a)
            if dist < best:
                pick, best = idx, dist
    else:
        pick = const_idx
    return cands[pick][0], cands[pick][1], pick


def compute_scale(cov_infer, cov_mu, cov_t, Gamma_ijt, target_p=TARGET_P):
    """Recursive-feasibility scale factor (makeconstraint.py:259-280)."""
    root_t = np.sqrt(np.linalg.norm(cov_t, 'fro'))
    alpha = np.sqrt(np.linalg.norm(cov_infer, 'fro')) / root_t
    beta = np.sqrt(np.linalg.norm(cov_mu, 'fro')) / root_t
    chi_p = scipy.stats.chi2.ppf(target_p, df=2)
    return (np.sqrt(chi_p) * beta / Gamma_ijt + alpha) ** 2


def compute_lower_bound(cov_infer, cov_mu, cov_t, eps_t=0.05 / 8):
    """Lower bound of the recursive-feasibility probability (makeconstraint.py:282-303)."""
    root_t = np.sqrt(np.linalg.norm(cov_t, 'fro'))
    alpha = np.sqrt(np.linalg.norm(cov_infer, 'fro')) / root_t
    beta = np.sqrt(np.linalg.norm(cov_mu, 'fro')) / root_t
    gamma = scipy.stats.norm.ppf(1 - eps_t)
    return scipy.stats.chi2.cdf((gamma * (1 - alpha) / beta) ** 2, df=2)


# ----------------------------------------------------------------------------------------
# Risk allocation constants (v8ideal/__init__.py:2920-2926, :910-913, :1481-1482)
# ----------------------------------------------------------------------------------------
def eps_ura_matrix(K):
    """eps_ura[i, k] = 0.05 / O for k < K[i] (per mode, not divided by K)."""
    K = np.asarray(K, dtype=int)
    O = len(K)
    maxK = int(max(K)) if O else 0
    e = np.zeros((O, maxK))
    for i in range(O):
        for k in range(int(K[i])):
            e[i, k] = EPS_TOTAL / O
    return e


def risk_constants(eps_ijt, target_p=TARGET_P):
    """(chi_r, chi_p, gamma) for one cell as scipy computes them in the reference loops."""
    chi_r = scipy.stats.chi2.ppf(1 - eps_ijt, df=2)
    chi_p = scipy.stats.chi2.ppf(target_p, df=2)
    gamma = scipy.stats.norm.ppf(1 - eps_ijt)
    return float(chi_r), float(chi_p), float(gamma)


# ----------------------------------------------------------------------------------------
# Particle bucketing (ovehicle.py:24-131, v8ideal/__init__.py:469-505)
# ----------------------------------------------------------------------------------------
class OVehicle:
    """Plain container with the fields the generators read (ovehicle.py:119-131)."""

    def __init__(self, T, past, latent_pmf, pred_positions, pred_yaws, init_center, bbox):
        self.T = T
        self.past = past
        self.latent_pmf = latent_pmf
        self.pred_positions = pred_positions
        self.pred_yaws = pred_yaws
        self.init_center = init_center
        self.bbox = bbox
        self.n_states = latent_pmf.size
        self.n_predictions = sum(p.shape[0] for p in pred_positions)


def _step_yaws(ps, pos_last, T):
    """atan2 heading of each step delta; step 0 measured from past[-1] (ovehicle.py:72-76)."""
    yaws = np.zeros((ps.shape[0], T))
    yaws[:, 0] = np.arctan2(ps[:, 0, 1] - pos_last[1], ps[:, 0, 0] - pos_last[0])
    for t in range(1, T):
        yaws[:, t] = np.arctan2(ps[:, t, 1] - ps[:, t - 1, 1], ps[:, t, 0] - ps[:, t - 1, 0])
    return yaws


def from_trajectron(T, past, latent_pmf, predictions, filter_pmf=FILTER_PMF,
                    bbox=np.array([4.5, 2.5])):
    """Keep modes with pmf > filter, regroup the rest to the nearest kept final-position centre,
    recompute pmf = N_k / N (ovehicle.py:24-117)."""
    n_states = len(predictions)
    pos_last = past[-1]
    keep = np.argwhere(latent_pmf > filter_pmf).ravel()
    K = keep.size
    positions, yaws_list = [], []
    centres = np.zeros((K, 2))
    total = 0
    for j, zv in enumerate(keep):
        ps = predictions[zv]
        positions.append(ps)
        yaws_list.append(_step_yaws(ps, pos_last, T))
        total += ps.shape[0]
        centres[j] = np.mean(ps[:, T - 1], axis=0)
    rare = np.arange(n_states)[np.isin(np.arange(n_states), keep, invert=True)]
    for zv in rare:
        ps = predictions[zv]
        if ps.size == 0:
            continue
        yw = _step_yaws(ps, pos_last, T)
        owner = np.argmin(scipy.spatial.distance_matrix(ps[:, T - 1, :], centres), axis=1)
        for j in range(K):
            sel = owner == j
            if not np.any(sel):
                continue
            positions[j] = np.concatenate((positions[j], ps[sel]))
            yaws_list[j] = np.concatenate((yaws_list[j], yw[sel]))
        total += ps.shape[0]
    pmf = np.zeros(keep.shape)
    for j in range(K):
        pmf[j] = positions[j].shape[0] / float(total)
    return OVehicle(T, past, pmf, positions, yaws_list, centres, bbox)


def make_ovehicles(predictions, z, latent_probs, minpos, pasts, bboxes, T):
    """Sampler output -> list[OVehicle] (v8ideal/__init__.py:469-505).

    predictions: (n_ov, N, T, 2) float32 scene-relative; z: (n_ov, N) int latent ids;
    latent_probs: (n_ov, Z); minpos: (2,) scene origin; pasts: list of (H, 2) world-frame.
    """
    out = []
    for o in range(predictions.shape[0]):
        world = predictions[o] + minpos                     # float32 + float64 -> float64
        pmf = latent_probs[o]
        buckets = [[] for _ in range(pmf.size)]
        for j, p in enumerate(world):                       # per-particle append, as :491-492
            buckets[z[o][j]].append(p)
        buckets = [np.array(b) for b in buckets]
        out.append(from_trajectron(T, pasts[o], pmf, buckets, bbox=bboxes[o]))
    return out


# ----------------------------------------------------------------------------------------
# Vertices and L4 over-approximation (v8ideal/__init__.py:627-640, :694-736;
# midlevel/util.py:104-124, :171-200; utility.npu.vertices_of_bboxes restated)
# ----------------------------------------------------------------------------------------
def vertices_of_bboxes(centers, headings, lw):
    """(N,2),(N,) -> (N,4,2) bbox corners (midlevel/util.py:104-124 reshaped to corners)."""
    C = np.cos(headings)
    S = np.sin(headings)
    rot = np.stack((np.stack((C, S), -1), np.stack((S, -C), -1),
                    np.stack((C, -S), -1), np.stack((S, C), -1),
                    np.stack((-C, -S), -1), np.stack((-S, C), -1),
                    np.stack((-C, S), -1), np.stack((-S, -C), -1)), axis=1)
    disp = 0.5 * rot @ lw
    return (np.tile(centers, (4,)) + disp).reshape(-1, 4, 2)


def compute_L4_outerapproximation(theta, vertices):
    """A = [I;-I] R(theta), b = max over particles and corners of A v (midlevel/util.py:171-200)."""
    At = np.array([[np.cos(theta), np.sin(theta)], [-np.sin(theta), np.cos(theta)]])
    At = np.concatenate((np.eye(2), -np.eye(2))) @ At
    per_corner = [np.max(At @ vertices[:, c].T, axis=1) for c in range(4)]
    return At, np.max(np.stack(per_corner), axis=0)


def vertices_and_l4(ovehicles, ph):
    """vertices[t][k][ov], A_union[t][k][ov], b_union[t][k][ov] over all ph steps."""
    O = len(ovehicles)
    maxK = max(ov.n_states for ov in ovehicles) if O else 0
    vertices = np.empty((ph, maxK, O), dtype=object).tolist()
    A_union = np.empty((ph, maxK, O), dtype=object).tolist()
    b_union = np.empty((ph, maxK, O), dtype=object).tolist()
    for o, ov in enumerate(ovehicles):
        for k in range(ov.n_states):
            for t in range(ph):
                v = vertices_of_bboxes(ov.pred_positions[k][:, t], ov.pred_yaws[k][:, t], ov.bbox)
                vertices[t][k][o] = v
                A, b = compute_L4_outerapproximation(np.mean(ov.pred_yaws[k][:, t]), v)
                A_union[t][k][o] = A
                b_union[t][k][o] = b
    return vertices, A_union, b_union


def milp_obstacle_rows(ovehicles, T, ph, diag, M_big=10_000):
    """v8/__init__.py:692-724 (road boundaries off, S_big = 0): per (ov, k, t) the L4 faces
    as big-M rows.  Returns a list of (c, t, A (4,2), rhs (4,)) with rhs = b + diag and
    c = sum(K[:ov]) + k, plus a checker  holds(xy, delta) -> bool per row, in the reference's
    constraint order (4 face rows then the sum row)."""
    _, A_union, b_union = vertices_and_l4(ovehicles, ph)
    rows, c = [], 0
    for o, ov in enumerate(ovehicles):
        for k in range(ov.n_states):
            for t in range(T):
                rows.append((c, t, A_union[t][k][o], b_union[t][k][o] + diag))
            c += 1

    def holds(xy, delta):
        out = []
        for c, t, A, rhs in rows:
            lhs = A @ xy[t, :2] + M_big * (1 - delta[c, t])
            out.extend(bool(v) for v in lhs >= rhs)
            out.append(bool(np.sum(delta[c, t]) >= 1))
        return out
    return rows, holds


# ----------------------------------------------------------------------------------------
# Generators
# ----------------------------------------------------------------------------------------
def state_stats(ovehicles, ph):
    """t=0 mean / variance of x, y, yaw per (ov, k) (v8ideal/__init__.py:864-875)."""
    O = len(ovehicles)
    maxK = max(ov.n_states for ov in ovehicles) if O else 0
    mx, my, myaw, vx, vy, vyaw = (np.empty((O, maxK), dtype=object).tolist() for _ in range(6))
    for o, ov in enumerate(ovehicles):
        for k in range(ov.n_states):
            pose = np.vstack(ov.pred_positions[k])
            yaw = np.vstack(ov.pred_yaws[k])
            mx[o][k] = np.mean(pose[0::ph, 0])
            my[o][k] = np.mean(pose[0::ph, 1])
            myaw[o][k] = np.mean(yaw[:, 0])
            vx[o][k] = np.cov(pose[0::ph, 0])
            vy[o][k] = np.cov(pose[0::ph, 1])
            vyaw[o][k] = np.cov(yaw[:, 0])
    return (mx, my, myaw), (vx, vy, vyaw)


def minkowski_cell(poseData, Tpred, T, ref_traj, eps_ijt, chi_r, chi_p, R=R_COLLISION, mc=None):
    """One (ov, k) cell of the Minkowski/MVOE generator (v8ideal/__init__.py:893-947).

    ``mc`` selects whose makeconstraint functions run (this module, or the reference module
    loaded by tests/golden/make_golden.py).  Returns (records, prob_lower per t).
    """
    mc = mc if mc is not None else _SELF
    recs = []
    prob_lower_t = np.empty(T)
    eye = np.identity(2)
    for t in range(T):
        p0_t = poseData[t::Tpred, 0]
        p1_t = poseData[t::Tpred, 1]
        mean = np.mean([p0_t, p1_t], axis=1)
        prob_lower = 1.0
        for tau in range(t):
            p0_tau = poseData[tau::Tpred, 0]
            p1_tau = poseData[tau::Tpred, 1]
            cov_infer, cov_mu, cov_t = mc.predict_moments([p0_t, p1_t, p0_tau, p1_tau])
            r1 = mc.compute_mvoe(cov_infer * chi_r, cov_mu * chi_p)
            r2 = mc.compute_mvoe(r1[1], eye * R ** 2)
            m = -(ref_traj[t][0] - mean[0]) / (ref_traj[t][1] - mean[1])
            ref_x = [ref_traj[t][0], ref_traj[t][1]]
            n, d, which = mc.choose_closest_tangent(mean, r2[1], 1, m, ref_x)[:3]
            side = 1 if n @ mean <= d else -1          # +1: n.x >= d ; -1: n.x <= d
            lb = mc.compute_lower_bound(cov_infer, cov_mu, cov_t, eps_ijt)
            prob_lower = min(prob_lower, lb)
            recs.append(dict(t=t, tau=tau, n=np.array(n, dtype=float), d=float(d),
                             which=int(which), side=side, Q=r1[1], QR=r2[1],
                             beta1=float(r1[0]), beta2=float(r2[0]), lb=float(lb),
                             mean=np.array(mean)))
        prob_lower_t[t] = prob_lower
    return recs, prob_lower_t


def minkowski_generator(ovehicles, T, ph, ref_traj, ideal_trajs=None, R=R_COLLISION, mc=None,
                        with_l4=True):
    """compute_obstacle_constraints_GMM_Minkowski_idealprediction restated without cvxpy
    (v8ideal/__init__.py:781-964).  Records are in the reference's append order (ov, k, t, tau).
    """
    K = [ov.n_states for ov in ovehicles]
    O = len(ovehicles)
    eps_ura = eps_ura_matrix(K)
    ov_state_mean, ov_state_cov = state_stats(ovehicles, ph)
    records = []
    prob_lower_save = [None] * T
    moment_source = []                                   # ovehicles_toSave_moments positions
    chi_p = scipy.stats.chi2.ppf(TARGET_P, df=2)
    for o, ov in enumerate(ovehicles):
        src = []
        for k in range(ov.n_states):
            if T < ph:
                poseData = np.vstack(ideal_trajs[o][k])
                src.append(ideal_trajs[o][k])
                Tpred = T
            else:
                poseData = np.vstack(ov.pred_positions[k])
                src.append(ov.pred_positions[k])
                Tpred = ph
            eps_ijt = eps_ura[o, k] / ph
            chi_r = scipy.stats.chi2.ppf(1 - eps_ijt, df=2)
            recs, pl = minkowski_cell(poseData, Tpred, T, ref_traj, eps_ijt, chi_r, chi_p, R, mc)
            for r in recs:
                r['ov'], r['k'] = o, k
            records.extend(recs)
            for t in range(T):                            # last cell wins (:947)
                prob_lower_save[t] = pl[t]
        moment_source.append(src)
    out = dict(records=records, prob_lower_save=prob_lower_save,
               ov_state_mean=ov_state_mean, ov_state_cov=ov_state_cov,
               OVconstraint=_ov_in_junction(ovehicles, ph),
               moments=save_moments(moment_source, T))
    if with_l4:
        out['vertices'], out['A_union'], out['b_union'] = vertices_and_l4(ovehicles, ph)
    return out


def _ov_in_junction(ovehicles, ph):
    """OVconstraint flag for the Town03 scene4 T-intersection (v8ideal/__init__.py:831-851)."""
    flag = False
    for ov in ovehicles:
        inj = None
        for k in range(ov.n_states):
            pose = np.vstack(ov.pred_positions[k])
            mx, my = np.mean(pose[0::ph, 0]), np.mean(pose[0::ph, 1])
            inj = not (mx >= 190 or my <= -80)
        flag = flag or bool(inj)
    return flag


def affine_generator(ovehicles, T, ph, ref_traj, R=R_COLLISION, with_l4=True, mc=None):
    """compute_obstacle_constraints_GMM_affine restated without cvxpy
    (v8ideal/__init__.py:1378-1539).  Constraint: n.x >= d + margin (side +1) or
    n.x <= d - margin (side -1), margin = Gamma * ||sqrtm(cov) [m, -1]^T||_2.
    """
    mc = mc if mc is not None else _SELF
    K = [ov.n_states for ov in ovehicles]
    eps_ura = eps_ura_matrix(K)
    ov_state_mean, ov_state_cov = state_stats(ovehicles, ph)
    records = []
    eye = np.identity(2)
    for o, ov in enumerate(ovehicles):
        for k in range(ov.n_states):
            poseData = np.vstack(ov.pred_positions[k])
            for t in range(T):
                eps_ijt = eps_ura[o, k] / ph
                gamma = scipy.stats.norm.ppf(1 - eps_ijt)
                p0 = poseData[t::ph, 0]
                p1 = poseData[t::ph, 1]
                mean = np.array([np.mean(p0), np.mean(p1)])
                cov = np.cov([p0, p1])
                cov_sqrt = scipy.linalg.sqrtm(cov)
                m = -(ref_traj[t][0] - mean[0]) / (ref_traj[t][1] - mean[1])
                M = np.array([m, -1])
                ref_pose = np.array((ref_traj[t][0], ref_traj[t][1]))
                n, d, which = mc.choose_closest_tangent(mean, eye, R, m, ref_pose)[:3]
                margin = gamma * np.linalg.norm(cov_sqrt @ M.T, 2)
                side = 1 if n @ mean <= d else -1
                rhs = d + margin if side == 1 else d - margin
                records.append(dict(ov=o, k=k, t=t, n=np.array(n), d=float(d), which=int(which),
                                    side=side, margin=float(np.real(margin)),
                                    rhs=float(np.real(rhs)), mean=mean, cov=cov, m=float(m),
                                    gamma=float(gamma)))
    out = dict(records=records, ov_state_mean=ov_state_mean, ov_state_cov=ov_state_cov,
               OVconstraint=False)
    if with_l4:
        out['vertices'], out['A_union'], out['b_union'] = vertices_and_l4(ovehicles, ph)
    return out


M_BIG = 10_000             # params.M_big (v8ideal/__init__.py:86): the mode match's "no such mode"


def match_loaded_modes(mean_loaded, x_init, cur_means, n_states, M_big=M_BIG):
    """Mode matching of compute_obstacle_constraints_GMM_affine_scale_ideal for one OV
    (v8ideal/__init__.py:2190-2276): for each current mode k, the previous frame's mode
    minimising ||x_init - mean'_0|| + sum_t ||mean_t - mean'_{t+1}||, modes >= the current
    n_states (and missing ones) scored M_big, first minimum on ties (np.argmin).
    mean_loaded[mode][t] (2,) or None; cur_means[k][t] (2,).  Returns the chosen mode per k."""
    num_mode = len(mean_loaded)
    picks = []
    for k in range(n_states):
        md = [0.0] * num_mode
        for mode in range(num_mode):
            entry = mean_loaded[mode]
            if entry is None or entry[0] is None:
                md[mode] = M_big
                continue
            v = np.linalg.norm(np.asarray(x_init, float)[:2] - np.asarray(entry[0], float))
            for t in range(len(cur_means[k])):
                v += np.linalg.norm(np.asarray(cur_means[k][t]) - np.asarray(entry[t + 1], float))
            md[mode] = v
        for rest in range(n_states, num_mode):
            md[rest] = M_big
        picks.append(int(np.argmin(md)))
    return picks


def affine_scale_generator(ovehicles, T, ph, ref_traj, x_init=None, loaded=None,
                           ideal_trajs=None, R=R_COLLISION, target_p=TARGET_P, mc=None,
                           scaled=True):
    """compute_obstacle_constraints_GMM_affine_scale_ideal restated without cvxpy
    (v8ideal/__init__.py:2074-2456).  Per (ov, k, t): scale = max(1, max_{tau<t}
    compute_scale(predict_moments(t, tau), Gamma)) (:2320-2340), cov = scale * np.cov(p_t),
    a slope-m tangent of the radius-R circle (choose_closest_tangent with const_idx, :2376), and
    n.x >= d + Gamma sqrt(|cov|_F) |[m, -1]| if n.mean <= d else n.x <= d - ... (:2379-2398).
    At T < ph the clouds are ideal_trajs and m / const_idx come from the previous frame's
    meanNtangent `loaded` = (mean_p0p1, tangent, const_idx) matched per mode; an OV without
    loaded data keeps const_idx = -1 (the reference's initial value: Python's last candidate).
    scaled=False is compute_obstacle_constraints_GMM_affine_robust (:1541-1878): the same
    generator without the scale loop (scale = 1).
    Returns records and meanNtangent = (mean_p0p1, tangent, cov_p0p1, 0, const_idx)."""
    mc = mc if mc is not None else _SELF
    K = [ov.n_states for ov in ovehicles]
    O = len(ovehicles)
    eps_ura = eps_ura_matrix(K)
    use_ideal = T < ph
    tangent_saved, const_saved = {}, {}
    if use_ideal and loaded is not None:
        mean_l, tangent_l, const_l = loaded
        for o, ov in enumerate(ovehicles):
            if o >= len(mean_l) or mean_l[o] is None or len(mean_l[o]) == 0:
                continue
            cur = []
            for k in range(ov.n_states):
                pd = np.vstack(ideal_trajs[o][k])
                cur.append([np.array([np.mean(pd[t::T, 0]), np.mean(pd[t::T, 1])])
                            for t in range(T)])
            for k, idx in enumerate(match_loaded_modes(mean_l[o], x_init, cur, ov.n_states)):
                tangent_saved[(o, k)] = tangent_l[o][idx]
                const_saved[(o, k)] = const_l[o][idx]
    mean_p0p1 = [[[None] * T for _ in range(max(K))] for _ in range(O)]
    tangent = [[[None] * T for _ in range(max(K))] for _ in range(O)]
    cov_p0p1 = [[[None] * T for _ in range(max(K))] for _ in range(O)]
    const_save = [[[None] * T for _ in range(max(K))] for _ in range(O)]
    records = []
    eye = np.identity(2)
    for o, ov in enumerate(ovehicles):
        for k in range(ov.n_states):
            if use_ideal:
                poseData = np.vstack(ideal_trajs[o][k])
                Tpred = T
            else:
                poseData = np.vstack(ov.pred_positions[k])
                Tpred = ph
            for t in range(T):
                const_idx = -1
                eps_ijt = eps_ura[o, k] / ph
                gamma = scipy.stats.norm.ppf(1 - eps_ijt)
                p0 = poseData[t::Tpred, 0]
                p1 = poseData[t::Tpred, 1]
                mean = np.array([np.mean(p0), np.mean(p1)])
                scale = 1.0
                for tau in (range(t) if scaled else ()):
                    p_t_tau = [p0, p1, poseData[tau::Tpred, 0], poseData[tau::Tpred, 1]]
                    cov_infer, cov_mu, cov_t = mc.predict_moments(p_t_tau)
                    scale_temp = mc.compute_scale(cov_infer, cov_mu, cov_t, gamma,
                                                  target_p=target_p)
                    scale = np.max((scale_temp, scale))
                cov = scale * np.cov([p0, p1])
                cov_fro_sqrt = np.sqrt(np.linalg.norm(cov, 'fro'))
                if T == ph:
                    m = -(ref_traj[t][0] - mean[0]) / (ref_traj[t][1] - mean[1])
                    const_idx = None
                elif (o, k) in tangent_saved:
                    m = tangent_saved[(o, k)][t + 1]
                    const_idx = const_saved[(o, k)][t + 1]
                else:
                    m = -(ref_traj[t][0] - mean[0]) / (ref_traj[t][1] - mean[1])
                M = np.array([m, -1])
                ref_pose = np.array((ref_traj[t][0], ref_traj[t][1]))
                n, d, const_idx = mc.choose_closest_tangent(mean, eye, R, m, ref_pose,
                                                            const_idx)[:3]
                margin = gamma * cov_fro_sqrt * np.linalg.norm(M.T, 2)
                side = 1 if n @ mean <= d else -1
                rhs = d + margin if side == 1 else d - margin
                records.append(dict(ov=o, k=k, t=t, n=np.array(n), d=float(d),
                                    which=int(const_idx), side=side, margin=float(margin),
                                    rhs=float(rhs), mean=mean, cov=cov / scale, m=float(m),
                                    scale=float(scale), gamma=float(gamma)))
                mean_p0p1[o][k][t] = mean
                tangent[o][k][t] = m
                cov_p0p1[o][k][t] = cov / scale
                const_save[o][k][t] = const_idx
    return dict(records=records, meanNtangent=(mean_p0p1, tangent, cov_p0p1, 0, const_save))


def save_moments(positions, T):
    """mean / cov per (ov, k, t) and cross_cov[t][tau] = cov(p_t, p_tau)[0:2, 2:4]
    (v8ideal/__init__.py:2575-2618).  ``positions[o][k]`` is (N_k, T, 2)."""
    O = len(positions)
    maxK = max(len(p) for p in positions) if O else 0
    mean_p0p1 = np.empty((O, maxK, T), dtype=object).tolist()
    cov_p0p1 = np.empty((O, maxK, T), dtype=object).tolist()
    cross_cov = np.empty((O, maxK, T, T - 1), dtype=object).tolist()
    for o, cells in enumerate(positions):
        for k, traj in enumerate(cells):
            poseData = np.vstack(traj)
            for t in range(T):
                p_t = [poseData[t::T, 0], poseData[t::T, 1]]
                mean_p0p1[o][k][t] = np.mean(p_t, axis=1)
                cov_p0p1[o][k][t] = np.cov(p_t)
                for tau in range(t):
                    C = np.cov([p_t[0], p_t[1], poseData[tau::T, 0], poseData[tau::T, 1]])
                    cross_cov[o][k][t][tau] = C[0:2, 2:4]
    return dict(mean_p0p1=mean_p0p1, cov_p0p1=cov_p0p1, cross_cov=cross_cov)


def ideal_x0(mean0, cov0, cell, seed):
    """The single shared initial draw x0 ~ MVN(mean_0, cov_0) (v8ideal/__init__.py:2662-2665),
    made reproducible: x0 = mean_0 + chol(cov_0) z, z = Philox pair (0, 0, cell, X0 stream)."""
    z0, z1 = philox.normal_pair(0, 0, cell, philox.STREAM_IDEAL_X0, seed)
    L = np.linalg.cholesky(cov0)
    return mean0 + L @ np.array([float(z0), float(z1)])


def ideal_noise(cell, t, n, seed):
    """Z ~ N(0, I) of shape (n, 2) for one (cell, step) (v8ideal/__init__.py:2699-2700)."""
    idx = np.arange(n, dtype=np.uint64)
    z0, z1 = philox.normal_pair(idx, t, cell, philox.STREAM_IDEAL_Z, seed)
    return np.stack((z0, z1), axis=1)


def ideal_cell_plan(mean, cov, xcov, data_idx, T):
    """Per-step (A_t, L_t, mean_t, mean_{t+1}) of the conditional-Gaussian rollout
    (v8ideal/__init__.py:2671-2696).  Raises LinAlgError on a non-PD conditional covariance,
    as the reference does."""
    plan = []
    for t in range(T):
        C = xcov[data_idx][t + 1][t]
        A = C @ np.linalg.inv(cov[data_idx][t])
        Lc = np.linalg.cholesky(cov[data_idx][t + 1] - A @ C.T)
        plan.append((A, Lc, mean[data_idx][t], mean[data_idx][t + 1]))
    return plan


def predict_ideal(moments, n_states, T, n_samples, x0s=None, Zs=None, seed=0):
    """Affine conditional-Gaussian forward rollout from the previous step's moments
    (v8ideal/__init__.py:2620-2711).  Quirks kept: one x0 shared by all rows; slot t holds
    x_{t+1}; the data_idx fallback when K grew.  x0s[o][k] / Zs[o][k][t] inject the draws;
    otherwise they come from the Philox streams keyed by the global cell index.
    Returns traj_all[o][k] of shape (n_samples, T, 2).
    """
    mean, cov, xcov = moments['mean_p0p1'], moments['cov_p0p1'], moments['cross_cov']
    traj_all = {}
    cell = 0
    for o, K in enumerate(n_states):
        traj_all.setdefault(o, {})
        n_latent = len(mean[o])
        for k in range(K):
            data_idx = k if k < n_latent else max(n_latent - 1, 0)
            if x0s is not None:
                x0 = np.asarray(x0s[o][k], dtype=float)
            else:
                x0 = ideal_x0(mean[o][data_idx][0], cov[o][data_idx][0], cell, seed)
            x = x0 * np.ones((n_samples, 2))
            traj = np.zeros((n_samples, T, 2))
            traj[:, 0, :] = x
            for t in range(T):
                A = xcov[o][data_idx][t + 1][t] @ np.linalg.inv(cov[o][data_idx][t])
                cond_mean = mean[o][data_idx][t + 1] + (x - mean[o][data_idx][t]) @ A.T
                L = np.linalg.cholesky(cov[o][data_idx][t + 1] - A @ xcov[o][data_idx][t + 1][t].T)
                Z = Zs[o][k][t] if Zs is not None else ideal_noise(cell, t, n_samples, seed)
                x = cond_mean + Z @ L.T
                traj[:, t, :] = x
            traj_all[o][k] = traj
            cell += 1
    return traj_all


# ----------------------------------------------------------------------------------------
# Trajectron++ GMM-latent sampler (absent submodule; restated from upstream semantics)
# PARITY UNPINNED: no reference test or fixture covers these internals.
# ----------------------------------------------------------------------------------------
def _rn32(fn, x):
    """float32 transcendental evaluated in float64 and rounded once (as the kernel does)."""
    return fn(np.asarray(x, np.float64)).astype(np.float32)


def unicycle_step(x, y, phi, v, dphi, a, dt):
    """Trajectron++ Unicycle.dynamic: exact integration at constant (dphi, a); straight-line
    branch when |dphi| <= 1e-2 (float32 throughout, as torch runs it; sin/cos rounded from
    float64)."""
    f = np.float32
    dt = f(dt)
    straight = np.abs(dphi) <= f(1e-2)
    w = np.where(straight, f(1.0), dphi).astype(f)
    phi1 = (phi + w * dt).astype(f)
    s0, c0 = _rn32(np.sin, phi), _rn32(np.cos, phi)
    s1, c1 = _rn32(np.sin, phi1), _rn32(np.cos, phi1)
    dsin = ((s1 - s0) / w).astype(f)
    dcos = ((c1 - c0) / w).astype(f)
    aw = (a / w).astype(f)
    xt = x + aw * dcos + v * dsin + aw * s1 * dt
    yt = y - v * dcos + aw * dsin - aw * c1 * dt
    xs = x + v * c0 * dt + (a / f(2)) * c0 * dt * dt
    ys = y + v * s0 * dt + (a / f(2)) * s0 * dt * dt
    nx = np.where(straight, xs, xt).astype(f)
    ny = np.where(straight, ys, yt).astype(f)
    nphi = np.where(straight, phi, phi1).astype(f)
    nv = (v + a * dt).astype(f)
    return nx, ny, nphi, nv


def sample_latents(latent_cdf, n, ov, seed):
    """z ~ Categorical(p(z|x)) by inverse CDF of a Philox uniform (DiscreteLatent.sample_p)."""
    u = philox.uniform_single(np.arange(n, dtype=np.uint64), 0, ov, philox.STREAM_SAMPLER_Z, seed)
    z = np.searchsorted(latent_cdf, u, side='right')
    return np.minimum(z, len(latent_cdf) - 1).astype(np.int32)


def gmm2d_action(p, e0, e1):
    """GMM2D.rsample with one component (Trajectron++ model/components/gmm2d.py): s = exp(log s),
    L = [[s0, 0], [s1 rho, s1 sqrt(clamp(1 - rho^2, 1e-5, 1))]], a = mu + squeeze(L @ eps) --
    the matmul row summed before mu is added.  p: (..., 5) float32 rows."""
    f = np.float32
    s0, s1, rho = _rn32(np.exp, p[..., 2]), _rn32(np.exp, p[..., 3]), p[..., 4]
    omr2 = np.clip(f(1) - rho * rho, f(1e-5), f(1)).astype(f)
    dphi = (p[..., 0] + s0 * e0).astype(f)
    acc = (p[..., 1] + ((s1 * rho) * e0 + (s1 * np.sqrt(omr2)) * e1)).astype(f)
    return dphi, acc


def sample_unicycle(init_state, latent_cdf, gmm, n, T, dt, seed, ov=0, z=None, eps=None,
                    per_particle=False):
    """One OV's particle cloud: z draw, GMM2D reparametrised action per step, Unicycle
    integration.  init_state: (x, y, phi, v) scene-relative; gmm: (Z, T, 5) = mu_dphi, mu_a,
    log_s_dphi, log_s_a, rho per latent, or with per_particle=True (n, T, 5) per sample (p_y_xz's
    autoregressive decoder output).  z: injected ids (n,) or None (Philox inverse CDF of
    latent_cdf); eps: injected noise (n, T, 2) or None (Philox).  Returns z (n,), positions
    (n, T, 2) float32."""
    f = np.float32
    z = (sample_latents(latent_cdf, n, ov, seed) if z is None
         else np.asarray(z, np.int32).reshape(n))
    x = np.full(n, init_state[0], dtype=f)
    y = np.full(n, init_state[1], dtype=f)
    phi = np.full(n, init_state[2], dtype=f)
    v = np.full(n, init_state[3], dtype=f)
    idx = np.arange(n, dtype=np.uint64)
    out = np.empty((n, T, 2), dtype=f)
    g = np.asarray(gmm, dtype=f)
    for t in range(T):
        if eps is None:
            e0, e1 = philox.normal_pair(idx, t, ov, philox.STREAM_SAMPLER_EPS, seed)
            e0, e1 = e0.astype(f), e1.astype(f)
        else:
            e0, e1 = (np.asarray(eps, f)[:, t, c] for c in (0, 1))
        p = g[:, t] if per_particle else g[z, t]
        dphi, acc = gmm2d_action(p, e0, e1)
        x, y, phi, v = unicycle_step(x, y, phi, v, dphi, acc, dt)
        out[:, t, 0] = x
        out[:, t, 1] = y
    return z, out


import sys as _sys  # noqa: E402
_SELF = _sys.modules[__name__]
