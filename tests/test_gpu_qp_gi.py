"""The Goldfarb-Idnani active-set solve of the planning QP (CCMPC_QP_METHOD=gi, one wave per
scene for n = 2T <= 32: the factor and J in registers, 16 or 32 per lane) against the interior
point + polish (=ipm) and the oracle: the QP is strictly convex, so both methods must return
its unique minimiser and the same verdict on every scene (u within 1e-7 (1 + |u|), the
objective within 1e-9 relative)."""
import numpy as np
import pytest
import torch

from ccmpc import mpc
from test_gpu_mpc import LON, _check, _oracle_solve, _params_dict, _scene_inputs

pytestmark = pytest.mark.gpu


def _solve(monkeypatch, method, cps, T, kind, order, gamma, xbar, goals, refs, rec, **kw):
    monkeypatch.setenv("CCMPC_QP_METHOD", method)
    qp = mpc.PlanningQP(cps, T, kind=kind, u_order=order, **kw)
    out = qp.solve(gamma, xbar, goals, refs, rec, u_prev=kw.get("u_prev_t"))
    return [o.cpu().numpy() for o in out]


@pytest.mark.parametrize("kind", ["halfspace", "affine"])
@pytest.mark.parametrize("order", [mpc.U_ORDER_F, mpc.U_ORDER_C])
@pytest.mark.parametrize("T", [8, 12, 16])
def test_gi_equals_ipm_on_many_scenes(gpu, monkeypatch, kind, order, T):
    """T = 8: the 16-per-lane instance (the combined GI + IPM instance for a batch's hand-overs
    is not used: the GI-only pass, then the one-wave IPM pass); T = 12 / 16: the 32-per-lane
    GI-only instance, then the four-wave IPM pass."""
    seeds = list(range(100, 148)) if T <= 12 else list(range(100, 124))
    rec, cps, o_recs, refs, goals, x0s = _scene_inputs(seeds, T, gpu, kind=kind)
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    g_t, r_t = torch.as_tensor(goals, device=gpu), torch.as_tensor(refs, device=gpu)
    k = mpc.REC_HALFSPACE if kind == "halfspace" else mpc.REC_AFFINE
    u0, X0, c0, s0, _ = _solve(monkeypatch, "ipm", cps, T, k, order, gamma, xbar, g_t, r_t, rec)
    u1, X1, c1, s1, i1 = _solve(monkeypatch, "gi", cps, T, k, order, gamma, xbar, g_t, r_t, rec)
    np.testing.assert_array_equal(s1, s0)
    ok = s0 == mpc.QP_OK
    assert ok.sum() >= 4
    if T == 8:
        assert (~ok).sum() >= 1          # both verdicts exercised
    for i in np.flatnonzero(ok):
        tol = 1e-7 * (1.0 + np.abs(u0[i]).max())
        assert np.abs(u1[i] - u0[i]).max() <= tol, (seeds[i], np.abs(u1[i] - u0[i]).max())
        assert c1[i] == pytest.approx(c0[i], rel=1e-9)
    prm = _params_dict(mpc.MPCParams.reference_defaults())
    for i in np.flatnonzero(ok)[:8 if T <= 12 else 3]:
        want = _oracle_solve(x0s[i], T, goals[i], refs[i], o_recs[i], kind, prm,
                             order="F" if order == mpc.U_ORDER_F else "C")
        assert want["feasible"]
        _check(u1[i], X1[i], float(c1[i]), want, T)


def test_gi_shrinking_horizon_with_executed_controls(gpu, monkeypatch):
    """T < T_full (u_prev in the state's constant part): the same minimiser by both methods."""
    from ccmpc import cycle, engine
    from _qp_inputs import crossing_scene as cs
    Tf, T = 8, 5
    seeds = list(range(100, 116))
    rec, cps, goals, refs, x0s = [], [], [], [], []
    for s in seeds:
        ovs, cells, K, ref, goal, x0 = cs(s, T=Tf)
        store = engine.ParticleStore.from_cells([c[:, :T] for c in cells], device=gpu)
        cyc = cycle.MinkowskiCycle(store, K, ref[:T])
        cyc.run()
        rec.append(cyc.rec)
        cps.append(len(cells))
        goals.append(goal)
        refs.append(ref[:T])
        x0s.append(x0)
    rec = torch.cat(rec, 0).contiguous()
    u_prev = torch.as_tensor(np.random.default_rng(3).normal(0, 0.3, (len(seeds), 2 * (Tf - T))),
                             device=gpu)
    xbar, gamma = mpc.ltv(np.array(x0s), Tf, lon=LON)
    g_t = torch.as_tensor(np.array(goals), device=gpu)
    r_t = torch.as_tensor(np.array(refs), device=gpu)
    res = {}
    for m in ("ipm", "gi"):
        monkeypatch.setenv("CCMPC_QP_METHOD", m)
        qp = mpc.PlanningQP(cps, T, T_full=Tf)
        res[m] = [o.cpu().numpy() for o in qp.solve(gamma, xbar, g_t, r_t, rec, u_prev=u_prev)]
    np.testing.assert_array_equal(res["gi"][3], res["ipm"][3])
    for i in np.flatnonzero(res["ipm"][3] == mpc.QP_OK):
        tol = 1e-7 * (1.0 + np.abs(res["ipm"][0][i]).max())
        assert np.abs(res["gi"][0][i] - res["ipm"][0][i]).max() <= tol


@pytest.mark.parametrize("T", [8, 12])
def test_gi_hands_over_to_the_ipm(gpu, monkeypatch, T):
    """A solve that exceeds the active-set step budget (forced here: CCMPC_QP_GI_MAX_STEPS=0)
    hands the problem to the IPM in the same launch from the setup's state: the scenes that
    needed an active-set change come back as the IPM alone returns them, byte for byte, the
    others (the unconstrained minimum is feasible) agree to round-off.  T = 12: the hand-over
    is from the 32-per-lane GI-only instance to the four-wave IPM pass."""
    from ccmpc import mpc
    seeds = list(range(40, 52))
    rec, cps, _, refs, goals, x0s = _scene_inputs(seeds, T, gpu, "halfspace")
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    goal = torch.as_tensor(goals, device=gpu)
    ref = torch.as_tensor(refs, device=gpu)

    # every infeasibility verdict through the IPM here (CCMPC_QP_GI_NOSTEP=1), so that "GI
    # finished" is exactly "GI solved it"
    monkeypatch.setenv("CCMPC_QP_GI_NOSTEP", "1")

    def run(method, steps=None):
        monkeypatch.setenv("CCMPC_QP_METHOD", method)
        if steps is None:
            monkeypatch.delenv("CCMPC_QP_GI_MAX_STEPS", raising=False)
        else:
            monkeypatch.setenv("CCMPC_QP_GI_MAX_STEPS", str(steps))
        qp = mpc.PlanningQP(cps, T, device=gpu)
        out = qp.solve(gamma, xbar, goal, ref, rec)
        return [t.cpu().numpy().copy() for t in out]

    ipm = run("ipm")
    gi = run("gi")
    gi_done = (gi[3] == mpc.QP_OK)
    handed_mid = 0
    for budget in (0, 1, 2, 3):
        forced = run("gi", budget)
        handed = 0
        for s in range(len(seeds)):
            if gi_done[s] and gi[4][s] <= budget:   # the budget never bit
                assert all(a[s].tobytes() == b[s].tobytes() for a, b in zip(forced, gi)), \
                    (budget, s)
            else:
                # handed over after `budget` active-set changes: GI wrote IPM-owned LDS slots
                # (row flags, per-step weights, the polish's R / active list); the IPM must not
                # see any of it
                assert all(a[s].tobytes() == b[s].tobytes() for a, b in zip(forced, ipm)), \
                    (budget, s)
                handed += 1
                handed_mid += budget > 0
        assert handed > 0, budget
    assert handed_mid > 0            # some hand-over came after rows had entered


def test_gi_verdict_on_near_parallel_rows(gpu, monkeypatch):
    """Every cell's half-spaces twice, the copy's normal turned by 1e-7 rad and its offset moved
    by 1e-9 (near-duplicate, near-parallel rows at every step, what several cells' tangents at
    one t can give): GI and the IPM must return the same verdict on every scene and the same
    minimiser where it exists.  GI's own 'no step exists' test rests on round-off-sensitive
    comparisons, so a marginal verdict is handed to the IPM to confirm; the test
    runs both that default and every verdict through the IPM."""
    from ccmpc import _lib
    T = 8
    seeds = list(range(100, 132))
    rec, cps, _, refs, goals, x0s = _scene_inputs(seeds, T, gpu, "halfspace")
    h = rec.cpu().numpy().reshape(rec.shape[0], -1).view(_lib.HALFSPACE_DTYPE).copy()
    dup = h.copy()
    a = 1e-7
    n0, n1 = dup["n0"].copy(), dup["n1"].copy()
    dup["n0"], dup["n1"] = np.cos(a) * n0 - np.sin(a) * n1, np.sin(a) * n0 + np.cos(a) * n1
    dup["d"] = dup["d"] + 1e-9
    blocks, c = [], 0
    for k in cps:                           # scene s: its cells, then their near copies
        blocks += [h[c:c + k], dup[c:c + k]]
        c += k
    rec2 = torch.as_tensor(np.concatenate(blocks).view(np.uint8).reshape(
        sum(cps) * 2, h.shape[1], -1), device=gpu).contiguous()
    cps2 = [2 * k for k in cps]
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    g_t, r_t = torch.as_tensor(goals, device=gpu), torch.as_tensor(refs, device=gpu)
    k = mpc.REC_HALFSPACE
    u0, _, c0, s0, _ = _solve(monkeypatch, "ipm", cps2, T, k, mpc.U_ORDER_F, gamma, xbar, g_t,
                              r_t, rec2)
    for policy in ("2", "1"):
        monkeypatch.setenv("CCMPC_QP_GI_NOSTEP", policy)
        u1, _, c1, s1, _ = _solve(monkeypatch, "gi", cps2, T, k, mpc.U_ORDER_F, gamma, xbar,
                                  g_t, r_t, rec2)
        np.testing.assert_array_equal(s1, s0)
        ok = s0 == mpc.QP_OK
        assert ok.sum() >= 4 and (~ok).sum() >= 1
        for i in np.flatnonzero(ok):
            tol = 1e-6 * (1.0 + np.abs(u0[i]).max())
            assert np.abs(u1[i] - u0[i]).max() <= tol, (seeds[i], np.abs(u1[i] - u0[i]).max())
