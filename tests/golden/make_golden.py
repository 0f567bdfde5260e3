"""Generate the golden fixtures that pin the oracle to the reference.

Runs ONLY in the build container, where /root/reference exists.  It loads the reference's
own math module by file path

    /root/reference/collect/in_simulation/midlevel/v8ideal/makeconstraint.py

(numpy + scipy only; the planner package around it needs carla/cvxpy/Trajectron++ and is not
importable) and records inputs + outputs of its functions as .npz data.  The whole-cycle
fixtures drive the reference's makeconstraint functions through the restated planner glue
(oracle.ccmpc_oracle.minkowski_generator / affine_generator with mc=<reference module>), so the
arithmetic inside every (t, tau) pair is the reference's.

The reference RNG is unseeded (v8ideal/__init__.py:2664, :2699), so every random input is drawn
here from a fixed numpy seed and stored in the fixture.

Usage:  python tests/golden/make_golden.py      (rewrites tests/golden/*.npz)
"""
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import ccmpc_oracle as orc  # noqa: E402

REF_MC = "/root/reference/collect/in_simulation/midlevel/v8ideal/makeconstraint.py"


REF_MID = "/root/reference/collect/in_simulation/midlevel"

# The reference files whose code this script executes, pinned by content: regenerating the
# fixtures from a changed (untrusted) file fails before anything in it runs.
REF_SHA256 = {
    "v8ideal/__init__.py": "779778706a79bea299910e094563eb22a806d35e1614749b74bff54c6e91e807",
    "v8ideal/makeconstraint.py": "36f6fa8528041c6757a1f94f671ae8bcb49ec3fcae36595b063cb03e30e7d910",
    "ovehicle.py": "903dc28df8c0a79f70fabeb15e195005027f889f99478fb0ea3111330f162bb2",
    "util.py": "6f6cccf4de49c17f229b171180b2c0a9589791b10554ed955a310b1d4280016f",
}


def check_reference_file(path):
    import hashlib
    rel = os.path.relpath(path, REF_MID)
    want = REF_SHA256.get(rel)
    got = hashlib.sha256(open(path, "rb").read()).hexdigest()
    if want is None or got != want:
        raise RuntimeError(f"{path}: sha256 {got} is not the pinned {want}; refusing to execute")


# What the executed method bodies may touch of `os`: path joining only (save_moments /
# predict_ideal build their pickle paths with it, :2613, :2627); no filesystem or process calls.
SAFE_OS = __import__("types").SimpleNamespace(
    path=__import__("types").SimpleNamespace(join=os.path.join))


def load_reference():
    check_reference_file(REF_MC)
    spec = importlib.util.spec_from_file_location("ref_makeconstraint", REF_MC)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def reference_function(path, name, cls=None, namespace=None):
    """One function of a reference module whose module-level imports (carla, cvxpy, docplex,
    Trajectron++) are absent here, although its own body needs only numpy/scipy: the function's
    source is taken from the file's syntax tree unchanged (decorators dropped, so a classmethod
    takes its class as a plain first argument) and executed in `namespace`."""
    import ast
    check_reference_file(path)
    tree = ast.parse(open(path).read(), filename=path)
    body = tree.body
    if cls is not None:
        body = next(n for n in body if isinstance(n, ast.ClassDef) and n.name == cls).body
    fn = next(n for n in body if isinstance(n, ast.FunctionDef) and n.name == name)
    fn.decorator_list = []
    ns = dict(namespace or {})
    exec(compile(ast.Module(body=[fn], type_ignores=[]), path, "exec"), ns)
    return ns[name]


def rand_spd(rng, scale=1.0, cond=10.0):
    th = rng.uniform(0, np.pi)
    R = np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
    l1 = scale * rng.uniform(0.5, 2.0)
    l2 = l1 / rng.uniform(1.0, cond)
    return R @ np.diag([l1, l2]) @ R.T


def random_walk_cell(rng, n, T, origin=(190.0, -80.0)):
    """Trajectory cloud (n, T, 2): shared heading/speed mode + per-particle noise that
    accumulates over t, so (t, tau) blocks are strongly correlated like real rollouts."""
    heading = rng.uniform(-np.pi, np.pi)
    speed = rng.uniform(3.0, 10.0)
    p0 = np.array(origin) + rng.uniform(-10, 10, size=2)
    dv = rng.normal(0, 0.8, size=(n, 1))
    dh = rng.normal(0, 0.12, size=(n, 1))
    steps = np.arange(1, T + 1)[None, :] * 0.5
    h = heading + dh * steps
    v = speed + dv
    x = p0[0] + np.cumsum(v * np.cos(h) * 0.5, axis=1) + rng.normal(0, 0.05, size=(n, T))
    y = p0[1] + np.cumsum(v * np.sin(h) * 0.5, axis=1) + rng.normal(0, 0.05, size=(n, T))
    return np.stack((x, y), axis=-1)


def pack_cells(cells):
    counts = np.array([c.shape[0] for c in cells], dtype=np.int64)
    flat = np.concatenate([c.reshape(-1, c.shape[1], 2) for c in cells], axis=0)
    return counts, flat


def make_ovs(cells_per_ov, T):
    ovs = []
    for cells in cells_per_ov:
        K = len(cells)
        pmf = np.array([c.shape[0] for c in cells], dtype=float)
        pmf /= pmf.sum()
        past = np.array([[cells[0][0, 0, 0] - 4.0, cells[0][0, 0, 1] - 1.0]])
        yaws = [orc._step_yaws(c, past[-1], T) for c in cells]
        centres = np.array([c[:, T - 1].mean(0) for c in cells])
        ovs.append(orc.OVehicle(T, past, pmf, list(cells), yaws, centres, np.array([4.5, 2.5])))
        assert ovs[-1].n_states == K
    return ovs


def main():
    ref = load_reference()
    rng = np.random.default_rng(20251015)
    out = {}

    # --- compute_mvoe (makeconstraint.py:7-38) ---------------------------------------
    n = 160
    S1 = np.zeros((n, 2, 2)); S2 = np.zeros((n, 2, 2))
    for i in range(n):
        S1[i] = rand_spd(rng, scale=10 ** rng.uniform(-3, 1), cond=10 ** rng.uniform(0, 3))
        S2[i] = rand_spd(rng, scale=10 ** rng.uniform(-3, 1), cond=10 ** rng.uniform(0, 3))
    S2[0] = np.diag([1e-12, 1e-12]) + S2[0] * 1e-9        # near-degenerate second ellipsoid
    S2[1] = 3.4 ** 2 * np.eye(2)                          # the (Q, R^2 I) call shape
    beta = np.zeros(n); Q = np.zeros((n, 2, 2))
    for i in range(n):
        beta[i], Q[i] = ref.compute_mvoe(S1[i], S2[i])
    np.savez(os.path.join(HERE, "mvoe.npz"), S1=S1, S2=S2, beta=beta, Q=Q)

    # --- predict_moments (makeconstraint.py:41-70) ------------------------------------
    sizes = [5, 17, 64, 250, 1000, 2048]
    pts, offs = [], [0]
    ci, cm, ct = [], [], []
    for s in sizes * 3:
        cell = random_walk_cell(rng, s, 8)
        t, tau = sorted(rng.choice(8, size=2, replace=False))[::-1]
        p = np.stack((cell[:, t, 0], cell[:, t, 1], cell[:, tau, 0], cell[:, tau, 1]))
        a, b, c = ref.predict_moments([p[0], p[1], p[2], p[3]])
        pts.append(p); offs.append(offs[-1] + s)
        ci.append(a); cm.append(b); ct.append(c)
    np.savez(os.path.join(HERE, "predict_moments.npz"), points=np.concatenate(pts, axis=1),
             offsets=np.array(offs), cov_infer=np.array(ci), cov_mu=np.array(cm),
             cov_t=np.array(ct))

    # --- choose_closest_tangent (makeconstraint.py:134-207) ---------------------------
    n = 200
    mu = rng.uniform(-100, 200, size=(n, 2))
    Sig = np.array([rand_spd(rng, scale=rng.uniform(0.1, 20)) for _ in range(n)])
    m = rng.normal(0, 3, size=n)
    a = mu + rng.normal(0, 15, size=(n, 2))
    a[:20] = mu[:20]                                     # equidistant -> strict '<' tie, idx 0
    c = np.where(rng.uniform(size=n) < 0.5, 1.0, 3.4)
    nn = np.zeros((n, 2)); dd = np.zeros(n); ww = np.zeros(n, dtype=np.int64)
    for i in range(n):
        nn[i], dd[i], ww[i] = ref.choose_closest_tangent(mu[i], Sig[i], c[i], m[i], a[i])
    np.savez(os.path.join(HERE, "tangent.npz"), mu=mu, Sigma=Sig, m=m, a=a, c=c,
             n=nn, d=dd, which=ww)

    # --- compute_lower_bound / compute_scale (makeconstraint.py:259-303) ---------------
    n = 120
    CI = np.array([rand_spd(rng, scale=rng.uniform(0.01, 1)) for _ in range(n)])
    CM = np.array([rand_spd(rng, scale=rng.uniform(0.01, 1)) for _ in range(n)])
    CT = CI + CM
    eps = 0.05 / rng.integers(1, 9, size=n) / rng.choice([6, 8, 12, 40], size=n)
    gam = np.array([orc.scipy.stats.norm.ppf(1 - e) for e in eps])
    lb = np.array([ref.compute_lower_bound(CI[i], CM[i], CT[i], eps[i]) for i in range(n)])
    sc = np.array([ref.compute_scale(CI[i], CM[i], CT[i], gam[i]) for i in range(n)])
    np.savez(os.path.join(HERE, "lower_bound.npz"), cov_infer=CI, cov_mu=CM, cov_t=CT,
             eps=eps, gamma=gam, lower_bound=lb, scale=sc)

    # --- whole Minkowski / affine cycles (v8ideal/__init__.py:781-964, :1378-1539) -----
    for name, O, Ks, Ns, T in (("cycle_o2_t8", 2, (2, 1), (300, 180, 420), 8),
                               ("cycle_o1_t12", 1, (2,), (256, 97), 12)):
        cells_per_ov, flat_cells = [], []
        it = iter(Ns)
        for o in range(O):
            cells = [random_walk_cell(rng, next(it), T) for _ in range(Ks[o])]
            cells_per_ov.append(cells)
            flat_cells.extend(cells)
        ovs = make_ovs(cells_per_ov, T)
        ego = np.array(cells_per_ov[0][0][:, 0].mean(0)) + np.array([-12.0, 3.0])
        ref_traj = np.array([ego + np.array([4.0 * (t + 1), 0.5 * (t + 1)]) for t in range(T)])
        mk = orc.minkowski_generator(ovs, T, T, ref_traj, mc=ref, with_l4=True)
        af = orc.affine_generator(ovs, T, T, ref_traj, mc=ref, with_l4=False)
        counts, flat = pack_cells(flat_cells)
        recs = mk["records"]
        A_union = np.array([[mk["A_union"][t][k][o] for t in range(T)]
                            for o in range(O) for k in range(Ks[o])])
        b_union = np.array([[mk["b_union"][t][k][o] for t in range(T)]
                            for o in range(O) for k in range(Ks[o])])
        mom = mk["moments"]
        np.savez(
            os.path.join(HERE, f"{name}.npz"),
            T=T, K=np.array(Ks), counts=counts, positions=flat, ref_traj=ref_traj,
            past=np.array([ov.past[-1] for ov in ovs]),
            rec_cell=np.array([[r["ov"], r["k"], r["t"], r["tau"]] for r in recs]),
            rec_n=np.array([r["n"] for r in recs]), rec_d=np.array([r["d"] for r in recs]),
            rec_which=np.array([r["which"] for r in recs]),
            rec_side=np.array([r["side"] for r in recs]),
            rec_Q=np.array([r["Q"] for r in recs]), rec_QR=np.array([r["QR"] for r in recs]),
            rec_beta=np.array([[r["beta1"], r["beta2"]] for r in recs]),
            rec_lb=np.array([r["lb"] for r in recs]),
            rec_mean=np.array([r["mean"] for r in recs]),
            prob_lower_save=np.array(mk["prob_lower_save"], dtype=float),
            aff_n=np.array([r["n"] for r in af["records"]]),
            aff_d=np.array([r["d"] for r in af["records"]]),
            aff_which=np.array([r["which"] for r in af["records"]]),
            aff_side=np.array([r["side"] for r in af["records"]]),
            aff_margin=np.array([r["margin"] for r in af["records"]]),
            aff_rhs=np.array([r["rhs"] for r in af["records"]]),
            A_union=A_union, b_union=b_union,
            mom_mean=np.array([[mom["mean_p0p1"][o][k][t] for t in range(T)]
                               for o in range(O) for k in range(Ks[o])]),
            mom_cov=np.array([[mom["cov_p0p1"][o][k][t] for t in range(T)]
                              for o in range(O) for k in range(Ks[o])]),
            state_mean=np.array([[mk["ov_state_mean"][j][o][k] for j in range(3)]
                                 for o in range(O) for k in range(Ks[o])], dtype=float),
            state_cov=np.array([[mk["ov_state_cov"][j][o][k] for j in range(3)]
                                for o in range(O) for k in range(Ks[o])], dtype=float),
        )

    # --- predict_ideal (v8ideal/__init__.py:2620-2711), injected x0 and Z --------------
    T = 8
    cells = [[random_walk_cell(rng, 400, T), random_walk_cell(rng, 250, T)]]
    mom = orc.save_moments(cells, T)
    Tn, ns = T - 1, 48
    x0s = [[mom["mean_p0p1"][0][k][0] + rng.normal(0, 0.3, 2) for k in range(2)]]
    Zs = [[[rng.normal(size=(ns, 2)) for _ in range(Tn)] for _ in range(2)]]
    traj = orc.predict_ideal(mom, [2], Tn, ns, x0s=x0s, Zs=Zs)
    np.savez(os.path.join(HERE, "ideal_rollout.npz"),
             mean=np.array([[mom["mean_p0p1"][0][k][t] for t in range(T)] for k in range(2)]),
             cov=np.array([[mom["cov_p0p1"][0][k][t] for t in range(T)] for k in range(2)]),
             xcov=np.array([[[mom["cross_cov"][0][k][t][tau] if tau < t else np.zeros((2, 2))
                              for tau in range(T)] for t in range(T)] for k in range(2)]),
             x0=np.array(x0s[0]), Z=np.array(Zs[0]), traj=np.array([traj[0][k] for k in range(2)]))
    # --- GMM-affine with covariance scale (v8ideal/__init__.py:2074-2456): a T == ph step,
    #     then a T < ph step on injected ideal clouds that loads the first step's meanNtangent
    T, Ks, Ns = 8, (2, 1), (300, 250, 350)
    it = iter(Ns)
    cells_per_ov = [[random_walk_cell(rng, next(it), T) for _ in range(k)] for k in Ks]
    ovs = make_ovs(cells_per_ov, T)
    ego = np.array(cells_per_ov[0][0][:, 0].mean(0)) + np.array([-12.0, 3.0])
    ref1 = np.array([ego + np.array([4.0 * (t + 1), 0.5 * (t + 1)]) for t in range(T)])
    ref2 = ref1 + np.array([2.0, 0.25])
    x_init = np.array([ego[0] + 1.0, ego[1], 0.0, 5.0])
    g1 = orc.affine_scale_generator(ovs, T, T, ref1, mc=ref)
    mean1, tan1, _, _, ci1 = g1["meanNtangent"]
    mom = orc.save_moments(cells_per_ov, T)
    Tn, ns = T - 1, 200
    x0s = [[mom["mean_p0p1"][o][k][0] + rng.normal(0, 0.3, 2) for k in range(Ks[o])]
           for o in range(2)]
    Zs = [[[rng.normal(size=(ns, 2)) for _ in range(Tn)] for _ in range(Ks[o])]
          for o in range(2)]
    ideal = orc.predict_ideal(mom, list(Ks), Tn, ns, x0s=x0s, Zs=Zs)
    g2 = orc.affine_scale_generator(ovs, Tn, T, ref2, x_init=x_init,
                                    loaded=(mean1, tan1, ci1), ideal_trajs=ideal, mc=ref)
    # compute_obstacle_constraints_GMM_affine_robust (:1541-1878): the unscaled twin
    r1 = orc.affine_scale_generator(ovs, T, T, ref1, mc=ref, scaled=False)
    rm1, rt1, _, _, rc1 = r1["meanNtangent"]
    r2 = orc.affine_scale_generator(ovs, Tn, T, ref2, x_init=x_init, loaded=(rm1, rt1, rc1),
                                    ideal_trajs=ideal, mc=ref, scaled=False)
    counts, flat = pack_cells([c for cs in cells_per_ov for c in cs])

    def recs(g, key, dtype=float):
        return np.array([r[key] for r in g["records"]], dtype=dtype)

    np.savez(os.path.join(HERE, "affine_scale.npz"),
             T=T, K=np.array(Ks), counts=counts, positions=flat, ref1=ref1, ref2=ref2,
             x_init=x_init, past=np.array([ov.past[-1] for ov in ovs]),
             ideal=np.array([ideal[o][k] for o in range(2) for k in range(Ks[o])]),
             load_mean=np.array([[mean1[o][k][t] for t in range(T)]
                                 for o in range(2) for k in range(Ks[o])]),
             load_tangent=np.array([[tan1[o][k][t] for t in range(T)]
                                    for o in range(2) for k in range(Ks[o])]),
             load_const=np.array([[ci1[o][k][t] for t in range(T)]
                                  for o in range(2) for k in range(Ks[o])]),
             **{f"s{i}_{key}": recs(g, key, int if key in ("which", "side") else float)
                for i, g in ((1, g1), (2, g2), ("r1", r1), ("r2", r2))
                for key in ("d", "which", "side", "margin", "rhs", "scale", "m")},
             s1_n=np.array([r["n"] for r in g1["records"]]),
             s2_n=np.array([r["n"] for r in g2["records"]]))
    print("golden fixtures written to", HERE)


# ---- reference-code pins for the restated glue (rows a2, a4, a12) ---------------------------
class _Recorder:
    """Stands in for the OVehicle class that from_trajectron instantiates: keeps the
    constructor arguments (ovehicle.py:116-117 -> __init__ :119)."""

    def __init__(self, node, T, past, ground_truth, latent_pmf, pred_positions, pred_yaws,
                 init_center, bbox):
        self.T, self.past, self.latent_pmf = T, past, latent_pmf
        self.pred_positions, self.pred_yaws = pred_positions, pred_yaws
        self.init_center, self.bbox = init_center, bbox
        self.n_states = len(pred_positions)


def _latent_predictions(rng, L, N, T, pmf):
    """Sampler-shaped input of make_ovehicles: float32 scene-relative positions (N, T, 2)
    whose latent z picks a heading/speed mode, and z itself."""
    z = rng.choice(L, size=N, p=pmf)
    heading = rng.uniform(-np.pi, np.pi, size=L)
    speed = rng.uniform(2.0, 9.0, size=L)
    p0 = rng.uniform(30.0, 60.0, size=2)
    h = heading[z][:, None] + rng.normal(0, 0.08, size=(N, 1)) * np.arange(1, T + 1)
    v = speed[z][:, None] + rng.normal(0, 0.5, size=(N, 1))
    x = p0[0] + np.cumsum(v * np.cos(h) * 0.5, axis=1) + rng.normal(0, 0.05, size=(N, T))
    y = p0[1] + np.cumsum(v * np.sin(h) * 0.5, axis=1) + rng.normal(0, 0.05, size=(N, T))
    return np.stack((x, y), axis=-1).astype(np.float32), z.astype(np.int32)


def pin_ovehicles_and_l4(rng):
    """make_ovehicles (v8ideal/__init__.py:469-505) bucketing the sampler's output by z, then
    the reference's own OVehicle.from_trajectron (ovehicle.py:24-117) and, per kept mode and
    step, its own compute_L4_outerapproximation (midlevel/util.py:171-200) over bounding-box
    corners from midlevel/util.py:104-124 (get_vertices_from_centers).  v8ideal itself calls
    utility.npu.vertices_of_bboxes from the un-vendored python-utility submodule for those
    corners; util.py's function gives the same four corners, and b is a max over all of them.
    -> tests/golden/ovehicle_l4.npz"""
    import scipy.spatial  # noqa: F401  (from_trajectron uses scipy.spatial.distance_matrix)
    from_trajectron = reference_function(os.path.join(REF_MID, "ovehicle.py"), "from_trajectron",
                                         cls="OVehicle",
                                         namespace={"np": np, "scipy": scipy_mod(),
                                                    "DEFAULT_BBOX": np.array([4.5, 2.5])})
    util_ns = {"np": np}
    vertices_fn = reference_function(os.path.join(REF_MID, "util.py"), "get_vertices_from_centers",
                                     namespace=util_ns)
    l4_fn = reference_function(os.path.join(REF_MID, "util.py"), "compute_L4_outerapproximation",
                               namespace=util_ns)
    O, L, N, T = 2, 25, 2000, 8
    minpos = np.array([150.0, -120.0])
    bbox = np.array([4.5, 2.5])
    preds, zs, pmfs, pasts = [], [], [], []
    out = {"K": [], "counts": [], "positions": [], "yaws": [], "A": [], "b": [], "yaw_mean": []}
    pmf_out = np.zeros((O, L))
    centre = np.zeros((O, L, 2))
    for o in range(O):
        pmf = np.exp(rng.normal(0, 1.2, L))
        pmf[rng.choice(L, 3, replace=False)] += 3.0 * pmf.sum() / L   # a few kept modes
        pmf /= pmf.sum()
        pred, z = _latent_predictions(rng, L, N, T, pmf)
        past = (pred[0, 0].astype(np.float64) + minpos - np.array([3.0, 1.0]))[None]
        # make_ovehicles: world = float32 prediction + float64 minpos, appended per particle
        veh_predict = pred + minpos
        buckets = [[] for _ in range(L)]
        for j, p in enumerate(veh_predict):
            buckets[z[j]].append(p)
        buckets = [np.array(b) for b in buckets]
        ov = from_trajectron(_Recorder, None, T, None, past, pmf, buckets, filter_pmf=0.1,
                             bbox=bbox)
        preds.append(pred)
        zs.append(z)
        pmfs.append(pmf)
        pasts.append(past)
        out["K"].append(ov.n_states)
        pmf_out[o, :ov.n_states] = ov.latent_pmf
        centre[o, :ov.n_states] = ov.init_center
        for k in range(ov.n_states):
            ps, yw = ov.pred_positions[k], ov.pred_yaws[k]
            out["counts"].append(ps.shape[0])
            out["positions"].append(ps)
            out["yaws"].append(yw)
            A_k, b_k, m_k = [], [], []
            for t in range(T):
                theta = np.mean(yw[:, t])
                vert = vertices_fn(ps[:, t], yw[:, t], bbox).reshape(-1, 4, 2)
                A, b = l4_fn(theta, vert)
                A_k.append(A)
                b_k.append(b)
                m_k.append(theta)
            out["A"].append(A_k)
            out["b"].append(b_k)
            out["yaw_mean"].append(m_k)
    np.savez(os.path.join(HERE, "ovehicle_l4.npz"), T=T, minpos=minpos, bbox=bbox,
             pred=np.array(preds), z=np.array(zs), latent_pmf=np.array(pmfs),
             past=np.array(pasts), K=np.array(out["K"]), counts=np.array(out["counts"]),
             positions=np.concatenate(out["positions"]), yaws=np.concatenate(out["yaws"]),
             pmf_out=pmf_out, init_center=centre, A=np.array(out["A"]), b=np.array(out["b"]),
             yaw_mean=np.array(out["yaw_mean"]))


def scipy_mod():
    import scipy
    import scipy.spatial  # noqa: F401
    return scipy


IDEAL_N = 1_000_000              # predict_ideal's own n_samples (v8ideal/__init__.py:2640)
IDEAL_ROWS = 512


def ideal_rows(n=IDEAL_N, rows=IDEAL_ROWS, seed=99):
    """The sample indices the fixture keeps: the first half of `rows`, then a seeded spread."""
    rest = np.random.default_rng(seed).choice(np.arange(rows // 2, n), rows - rows // 2,
                                              replace=False)
    return np.concatenate((np.arange(rows // 2), np.sort(rest)))


def ideal_noise(zseed, cells, T, n=IDEAL_N):
    """The injected standard normals, in predict_ideal's draw order ((ov, k) cells, then t):
    [cell][t] -> (n, 2)."""
    g = np.random.default_rng(zseed)
    return [[g.standard_normal((n, 2)) for _ in range(T)] for _ in range(cells)]


def pin_predict_ideal(rng):
    """The reference's own MidlevelAgent.predict_ideal (v8ideal/__init__.py:2620-2711) run with
    n_samples = 1e6 as written, its moments pickle, x0 draw and unseeded RandomState
    (:2664, :2699) replaced by injected values: x0 per cell, and standard normals from a seeded
    generator in the function's own draw order.  The fixture keeps the inputs, IDEAL_ROWS
    sample rows of every cell's (1e6, T, 2) output and the output's per-cell mean / covariance.
    -> tests/golden/ideal_ref.npz"""
    import logging
    import types
    T_src, T, K = 8, 7, 2
    cells = [random_walk_cell(rng, 600, T_src), random_walk_cell(rng, 450, T_src)]
    mom = orc.save_moments([cells], T_src)                       # the inputs only
    x0s = [mom["mean_p0p1"][0][k][0] + rng.normal(0, 0.3, 2) for k in range(K)]
    zseed = 1234
    noise = ideal_noise(zseed, K, T)

    class _FakeFile:
        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

    x0_iter, z_iter = iter(x0s), iter([z for cell in noise for z in cell])

    class _RandomState:
        def __init__(self, seed=None):
            pass

        def standard_normal(self, shape):
            z = next(z_iter)
            assert z.shape == tuple(shape)
            return z

    fake_random = types.SimpleNamespace(
        multivariate_normal=lambda mean, cov, size=1: np.asarray(next(x0_iter)).reshape(1, 2),
        RandomState=_RandomState)
    np_proxy = types.ModuleType("numpy_injected")
    np_proxy.__dict__.update({k: getattr(np, k) for k in dir(np) if not k.startswith("__")})
    np_proxy.random = fake_random
    ns = {"np": np_proxy, "os": SAFE_OS, "logging": logging, "open": lambda *a, **k: _FakeFile(),
          "pickle": types.SimpleNamespace(load=lambda f: mom)}
    predict_ideal = reference_function(os.path.join(REF_MID, "v8ideal", "__init__.py"),
                                       "predict_ideal", cls="MidlevelAgent", namespace=ns)
    ovs = [types.SimpleNamespace(past=np.zeros((1, 2)), n_states=K)]
    traj = predict_ideal(None, ovs, T, 0, types.SimpleNamespace(frame=20))
    rows = ideal_rows()
    sel = np.array([traj[0][k][rows] for k in range(K)])
    mean = np.array([traj[0][k].mean(axis=0) for k in range(K)])
    cov = np.array([np.cov(traj[0][k].reshape(IDEAL_N, 2 * T).T) for k in range(K)])
    np.savez(os.path.join(HERE, "ideal_ref.npz"), T=T, n=IDEAL_N, zseed=zseed,
             mean_in=np.array([mom["mean_p0p1"][0][k] for k in range(K)]),
             cov_in=np.array([mom["cov_p0p1"][0][k] for k in range(K)]),
             xcov_in=np.array([[[mom["cross_cov"][0][k][t][tau] if tau < t else np.zeros((2, 2))
                                 for tau in range(T_src)] for t in range(T_src)]
                               for k in range(K)]),
             x0=np.array(x0s), rows=rows, traj_rows=sel, traj_mean=mean, traj_cov=cov)


# ---- the generator loops themselves (rows a9, a10, a11, a3) ---------------------------------
class _XY:
    """temp_x[t][i] (v8ideal/__init__.py:2932: X[t, 0], X[t, 1]) -- a marker of the step."""

    def __init__(self, t):
        self.t = t


class _Stack:
    """cp.vstack([temp_x[t][0], temp_x[t][1]]): `n.T @ it` becomes the linear form n . x_t.
    __array_ufunc__ = None makes numpy's matmul defer to __rmatmul__."""
    __array_ufunc__ = None

    def __init__(self, t):
        self.t = t

    def __rmatmul__(self, n):
        return _Linear(self.t, np.array(n, dtype=float))


class _Linear:
    """n . x_t; a comparison with a right-hand side is the recorded constraint."""
    __array_ufunc__ = None

    def __init__(self, t, n):
        self.t, self.n = t, n

    def __ge__(self, rhs):
        return (+1, self.t, self.n, complex(rhs))

    def __le__(self, rhs):
        return (-1, self.t, self.n, complex(rhs))


def _recording_cp():
    """The slice of cvxpy the generators touch with road-boundary constraints off: vstack of
    two temp_x entries and a 2-norm of a constant vector (evaluated)."""
    import types

    def vstack(items):
        assert len(items) == 2 and items[0].t == items[1].t
        return _Stack(items[0].t)

    def norm(x, p=2):
        assert p == 2
        return np.linalg.norm(np.asarray(x), 2)
    return types.SimpleNamespace(vstack=vstack, norm=norm)


def reference_generators():
    """The reference's own compute_obstacle_constraints_GMM_Minkowski_idealprediction
    (v8ideal/__init__.py:781-964), compute_obstacle_constraints_GMM_affine (:1378-1539) and
    save_moments (:2575-2618), each taken from the file's syntax tree unchanged and executed in a
    namespace of numpy / scipy / the reference makeconstraint module and a recording `cp`.
    Outside their class body the methods' private names are not mangled, so the `self` they
    get carries the attributes `__params`, `__prediction_horizon`, `__ego_vehicle` literally;
    predict_ideal, __compute_vertices and __compute_overapproximations (pinned separately:
    ideal_ref.npz, ovehicle_l4.npz) are stubs; save_moments' pickle.dump is captured."""
    import copy
    import logging
    import types
    import scipy.linalg
    import scipy.stats
    path = os.path.join(REF_MID, "v8ideal", "__init__.py")
    ns = {"np": np, "scipy": scipy_mod(), "linalg": scipy.linalg, "norm": scipy.stats.norm,
          "makeconstraint": load_reference(), "cp": _recording_cp(), "logging": logging,
          "copy": copy, "os": SAFE_OS}
    saved = {}

    class _File:
        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

    ns_sm = dict(ns, open=lambda *a, **k: _File(),
                 pickle=types.SimpleNamespace(dump=lambda obj, f: saved.update(moments=obj)))
    mink = reference_function(path, "compute_obstacle_constraints_GMM_Minkowski_idealprediction",
                              cls="MidlevelAgent", namespace=ns)
    aff = reference_function(path, "compute_obstacle_constraints_GMM_affine",
                             cls="MidlevelAgent", namespace=ns)
    save_moments = reference_function(path, "save_moments", cls="MidlevelAgent",
                                      namespace=ns_sm)
    return mink, aff, save_moments, saved


def _agent_self(ph, save_moments, ideal=None):
    import types
    me = types.SimpleNamespace(road_boundary_constraints=False)
    setattr(me, "__params", types.SimpleNamespace(M_big=10_000, L=4))
    setattr(me, "__prediction_horizon", ph)
    setattr(me, "__ego_vehicle", types.SimpleNamespace(id=0))
    setattr(me, "__compute_vertices", lambda params, ovehicles: None)
    setattr(me, "__compute_overapproximations", lambda params, ovehicles, vertices: (None, None))
    me.predict_ideal = lambda ovehicles, T, ego_id, params: ideal
    me.save_moments = lambda *a: save_moments(me, *a)
    return me


def _grid_cells(grid, K):
    return np.array([grid[o][k] for o in range(len(K)) for k in range(K[o])], dtype=float)


def run_reference_generators(cells_per_ov, yaws_per_ov, T, ph, ref_traj, ideal=None,
                             with_affine=True):
    """Both reference generators on one planning step; returns npz-ready arrays."""
    import types
    mink, aff, save_moments, saved = reference_generators()
    K = [len(c) for c in cells_per_ov]
    O = len(K)
    ovs = [types.SimpleNamespace(n_states=K[o], pred_positions=list(cells_per_ov[o]),
                                 pred_yaws=list(yaws_per_ov[o])) for o in range(O)]
    params = types.SimpleNamespace(O=O, K=np.array(K), frame=40)
    eps_ura = np.zeros((O, max(K)))
    for o in range(O):
        eps_ura[o, :] = 0.05 / O                    # v8ideal/__init__.py:2920-2926
    temp_x = [[_XY(t), _XY(t), 1] for t in range(ph)]
    out = {}
    for kind, fn in (("mk", mink), ("aff", aff)):
        if kind == "aff" and not with_affine:
            continue
        me = _agent_self(ph, save_moments, ideal)
        saved.clear()
        res = fn(me, params, ovs, None, None, temp_x, eps_ura, None, T, ref_traj)
        cons, ovc, st_mean, st_cov = res[0], res[4], res[6], res[7]
        assert all(isinstance(c, tuple) for c in cons)
        out[f"{kind}_side"] = np.array([c[0] for c in cons], np.int64)
        out[f"{kind}_t"] = np.array([c[1] for c in cons], np.int64)
        out[f"{kind}_n"] = np.array([c[2] for c in cons]).reshape(-1, 2)
        rhs = np.array([c[3] for c in cons])
        assert np.all(rhs.imag == 0)
        out[f"{kind}_rhs"] = rhs.real
        out[f"{kind}_ovconstraint"] = np.bool_(ovc)
        out[f"{kind}_state_mean"] = np.stack([_grid_cells(g, K) for g in st_mean], 1)
        out[f"{kind}_state_cov"] = np.stack([_grid_cells(g, K) for g in st_cov], 1)
        if kind == "mk":
            if T == ph:
                out["mk_prob_lower_save"] = np.array(getattr(me, "__prob_lower_save"), float)
            mom = saved["moments"]
            C = sum(K)
            xc = np.zeros((C, T, T, 2, 2))
            c = 0
            for o in range(O):
                for k in range(K[o]):
                    for t in range(T):
                        for tau in range(t):
                            xc[c, t, tau] = mom["cross_cov"][o][k][t][tau]
                    c += 1
            out["mom_mean"] = np.array([[mom["mean_p0p1"][o][k][t] for t in range(T)]
                                        for o in range(O) for k in range(K[o])])
            out["mom_cov"] = np.array([[mom["cov_p0p1"][o][k][t] for t in range(T)]
                                       for o in range(O) for k in range(K[o])])
            out["mom_xcov"] = xc
    return out


def _fixture_inputs(cells_per_ov, T, ph, ref_traj):
    pasts = np.array([[c[0][0, 0, 0] - 4.0, c[0][0, 0, 1] - 1.0] for c in cells_per_ov])
    yaws = [[orc._step_yaws(c, pasts[o], ph) for c in cells]
            for o, cells in enumerate(cells_per_ov)]
    counts, flat = pack_cells([c for cs in cells_per_ov for c in cs])
    return pasts, yaws, dict(T=T, ph=ph, K=np.array([len(c) for c in cells_per_ov]),
                             counts=counts, positions=flat, ref_traj=ref_traj, past=pasts,
                             yaws=np.concatenate([y for ys in yaws for y in ys]))


def pin_generator_glue(rng):
    """The reference's own generator loops on five planning steps -> tests/golden/refloop_*.npz:
    the two whole-cycle fixtures' inputs (cycle_o2_t8, cycle_o1_t12), a multi-OV T = 12 step, a
    T = 40 step (780 (t, tau) pairs per cell), and one shrinking step (ph = 8, T = 7) on
    injected ideal trajectories (the T < ph switch :885-888, eps / ph with ph != T)."""
    def ego_ref(cells, T):
        ego = np.array(cells[0][0][:, 0].mean(0)) + np.array([-12.0, 3.0])
        return np.array([ego + np.array([4.0 * (t + 1), 0.5 * (t + 1)]) for t in range(T)])

    steps = []
    for name in ("cycle_o2_t8", "cycle_o1_t12"):
        g = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
        T, K = int(g["T"]), [int(k) for k in g["K"]]
        flat, cnt = g["positions"], g["counts"]
        cells, c0 = [], 0
        for n in cnt:
            cells.append(flat[c0:c0 + n])
            c0 += n
        it = iter(cells)
        steps.append(("refloop_" + name[6:], [[next(it) for _ in range(k)] for k in K], T, T,
                      np.asarray(g["ref_traj"]), None))
    for name, Ks, lo, hi, T in (("refloop_o3_t12", (2, 1, 3), 150, 420, 12),
                                ("refloop_o2_t40", (1, 2), 120, 220, 40)):
        cells = [[random_walk_cell(rng, int(rng.integers(lo, hi)), T) for _ in range(k)]
                 for k in Ks]
        steps.append((name, cells, T, T, ego_ref(cells, T), None))
    # shrinking step: sampler particles over ph = 8, ideal rollouts (T = 7) of their moments
    ph, T, Ks = 8, 7, (2, 1)
    cells = [[random_walk_cell(rng, int(rng.integers(200, 400)), ph) for _ in range(k)]
             for k in Ks]
    mom = orc.save_moments(cells, ph)
    x0s = [[mom["mean_p0p1"][o][k][0] + rng.normal(0, 0.3, 2) for k in range(Ks[o])]
           for o in range(len(Ks))]
    Zs = [[[rng.normal(size=(300, 2)) for _ in range(T)] for _ in range(Ks[o])]
          for o in range(len(Ks))]
    ideal = orc.predict_ideal(mom, list(Ks), T, 300, x0s=x0s, Zs=Zs)
    steps.append(("refloop_shrink_t7", cells, T, ph, ego_ref(cells, ph), ideal))

    for name, cells, T, ph, ref_traj, ideal_trajs in steps:
        pasts, yaws, inputs = _fixture_inputs(cells, T, ph, ref_traj)
        outs = run_reference_generators(cells, yaws, T, ph, ref_traj, ideal=ideal_trajs,
                                        with_affine=ideal_trajs is None)
        if ideal_trajs is not None:
            inputs["ideal"] = np.concatenate([ideal_trajs[o][k] for o in range(len(cells))
                                              for k in range(len(cells[o]))])
            inputs["ideal_counts"] = np.array([ideal_trajs[o][k].shape[0]
                                               for o in range(len(cells))
                                               for k in range(len(cells[o]))])
        np.savez(os.path.join(HERE, name + ".npz"), **inputs, **outs)


def main_reference_glue():
    rng = np.random.default_rng(20261016)
    pin_ovehicles_and_l4(rng)
    pin_predict_ideal(rng)
    pin_generator_glue(np.random.default_rng(20261017))
    print("reference-glue fixtures written to", HERE)


if __name__ == "__main__":
    if "--generators-only" in sys.argv:
        pin_generator_glue(np.random.default_rng(20261017))
        sys.exit(0)
    if "--glue-only" not in sys.argv:
        main()
    main_reference_glue()
