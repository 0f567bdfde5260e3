"""GPU parity of the planning QP (ccmpc_mpc_ltv, ccmpc_mpc_qp) against oracle/mpc_oracle.py.

Parity bar: the QP's minimiser is unique (strictly convex objective), so the GPU solution is
compared with the oracle's KKT-certified one: |du|_inf <= 1e-6 (1 + |u|_inf), objective within
1e-8 relative, and the GPU point itself satisfies the KKT conditions; infeasible problems must
be reported (the reference's CPLEX failure path, v8ideal/__init__.py:3099-3110)."""
import numpy as np
import pytest
import torch

from ccmpc import cycle, engine, mpc
from oracle import ccmpc_oracle as orc
from oracle import mpc_oracle as mo
from _qp_inputs import crossing_scene, pick_seeds

pytestmark = pytest.mark.gpu

LON = 3.7


def _feasible(n=8):
    return pick_seeds("binding", n)


def _infeasible(n=2):
    return pick_seeds("infeasible", n)


def _params_dict(prm):
    return prm.as_dict()


def _scene_inputs(seeds, T, gpu, kind="halfspace"):
    """Device records (one block over all scenes), per-scene oracle records and QP inputs."""
    recs, cells_per_scene, o_recs, refs, goals, x0s = [], [], [], [], [], []
    for s in seeds:
        ovs, cells, K, ref, goal, x0 = crossing_scene(s, T=T)
        store = engine.ParticleStore.from_cells(cells, device=gpu)
        if kind == "halfspace":
            cyc = cycle.MinkowskiCycle(store, K, ref)
            cyc.run()
            o_recs.append(orc.minkowski_generator(ovs, T, T, ref, with_l4=False)["records"])
        else:
            cyc = cycle.AffineCycle(store, K, ref)
            cyc.run()
            o_recs.append(orc.affine_generator(ovs, T, T, ref, with_l4=False)["records"])
        recs.append(cyc.rec)
        cells_per_scene.append(len(cells))
        refs.append(ref)
        goals.append(goal)
        x0s.append(x0)
    rec = torch.cat(recs, 0).contiguous()
    return rec, cells_per_scene, o_recs, np.array(refs), np.array(goals), np.array(x0s)


def _oracle_solve(x0, T, goal, ref, o_rec, kind, prm, order="F", Tf=None, u_prev=None):
    Tf = Tf or T
    xbar, _, G, _, _ = mo.VehicleModel(Tf, 0.5, 0.5 * LON, LON).get_optimization_ltv(
        x0, np.zeros(2))
    return mo.solve_step(G, xbar, T, Tf, goal, ref, o_rec, kind, prm, u_prev=u_prev,
                         order=order)


def _check(u, X, cost, want, T):
    """The GPU point must be THE minimiser: the problem is strictly convex, so a point that
    meets the KKT conditions of the oracle's own (H, f, G, h) is the unique optimum whatever
    solver found it.  Where the oracle's SLSQP + active-set polish converged (its own point is
    KKT-certified) the two points must also agree; where it stalled (a few T = 12 scenes) the
    certificate decides."""
    prim, stat, comp, _ = mo.kkt_residuals(want["H"], want["f"], want["G"], want["h"], u)
    assert prim <= 1e-8 and stat <= 1e-5 and comp <= 1e-6, (prim, stat, comp)
    Xu = (want["Gf"] @ u + want["c"]).reshape(T, 4)
    np.testing.assert_allclose(X, Xu, rtol=0, atol=1e-8 * (1 + np.abs(Xu).max()))
    o_prim, o_stat, _, _ = mo.kkt_residuals(want["H"], want["f"], want["G"], want["h"],
                                            want["u"], want["lam"])
    if o_prim <= 1e-8 and o_stat <= 1e-6:
        tol = 1e-6 * (1.0 + np.max(np.abs(want["u"])))
        assert np.max(np.abs(u - want["u"])) <= tol, np.max(np.abs(u - want["u"]))
        assert abs(cost - want["cost"]) <= 1e-8 * abs(want["cost"])
        np.testing.assert_allclose(X, want["X"], rtol=0,
                                   atol=1e-6 * (1 + np.abs(want["X"]).max()))


@pytest.mark.parametrize("T", [8, 12, 40])
def test_ltv_kernel_matches_reference_model(gpu, T):
    rng = np.random.default_rng(T)
    x0 = np.column_stack((rng.uniform(-200, 200, 6), rng.uniform(-200, 200, 6),
                          rng.uniform(-np.pi, np.pi, 6), rng.uniform(0, 12, 6)))
    xbar, gamma = mpc.ltv(x0, T, Ts=0.5, lon=LON)
    xbar, gamma = xbar.cpu().numpy(), gamma.cpu().numpy()
    for s in range(len(x0)):
        xb, _, G, _, _ = mo.VehicleModel(T, 0.5, 0.5 * LON, LON).get_optimization_ltv(
            x0[s], np.zeros(2))
        np.testing.assert_allclose(xbar[s], xb, rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(gamma[s], G, rtol=0, atol=1e-11 * max(1.0, np.abs(G).max()))


@pytest.mark.parametrize("order", [mpc.U_ORDER_F, mpc.U_ORDER_C])
def test_qp_batch_matches_oracle(gpu, order):
    T = 8
    rec, cps, o_recs, refs, goals, x0s = _scene_inputs(_feasible(), T, gpu)
    prm = mpc.MPCParams.reference_defaults()
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    qp = mpc.PlanningQP(cps, T, params=prm, u_order=order)
    u, X, cost, status, iters = qp.solve(gamma, xbar, torch.as_tensor(goals, device=gpu),
                                         torch.as_tensor(refs, device=gpu), rec)
    u, X, cost = u.cpu().numpy(), X.cpu().numpy(), cost.cpu().numpy()
    status, iters = status.cpu().numpy(), iters.cpu().numpy()
    n_ok = 0
    for i, s in enumerate(_feasible()):
        want = _oracle_solve(x0s[i], T, goals[i], refs[i], o_recs[i], "halfspace",
                             _params_dict(prm), order="F" if order == mpc.U_ORDER_F else "C")
        if not want["feasible"]:     # (the 'C' pairing is a different problem)
            assert status[i] == mpc.QP_MAXITER, (s, status[i])
            continue
        assert status[i] == mpc.QP_OK and iters[i] < 60, (s, status[i], iters[i])
        _check(u[i], X[i], cost[i], want, T)
        n_ok += 1
    assert n_ok >= 4


def test_qp_reports_infeasible_scenes(gpu):
    T = 8
    seeds = _feasible(1) + _infeasible()
    rec, cps, o_recs, refs, goals, x0s = _scene_inputs(seeds, T, gpu)
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    qp = mpc.PlanningQP(cps, T)
    _, _, _, status, _ = qp.solve(gamma, xbar, torch.as_tensor(goals, device=gpu),
                                  torch.as_tensor(refs, device=gpu), rec)
    status = status.cpu().numpy()
    assert status[0] == mpc.QP_OK
    assert np.all(status[1:] == mpc.QP_MAXITER), status


def test_qp_batch_equals_single_scene_solves(gpu):
    T = 8
    seeds = _feasible(4)
    rec, cps, o_recs, refs, goals, x0s = _scene_inputs(seeds, T, gpu)
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    g_t, r_t = torch.as_tensor(goals, device=gpu), torch.as_tensor(refs, device=gpu)
    batch = mpc.PlanningQP(cps, T).solve(gamma, xbar, g_t, r_t, rec)[0].cpu().numpy()
    c0 = 0
    for i in range(len(seeds)):
        one = mpc.PlanningQP([cps[i]], T).solve(gamma[i:i + 1], xbar[i:i + 1], g_t[i:i + 1],
                                                r_t[i:i + 1], rec[c0:c0 + cps[i]])[0]
        c0 += cps[i]
        assert np.array_equal(one.cpu().numpy()[0], batch[i])


def test_qp_shrinking_step_with_executed_controls(gpu):
    """T < T_full: the first step's model, sliced, plus Gamma_p u_prev (:2858-2891)."""
    Tf, T = 8, 5
    seeds = _feasible(3)
    _, _, _, refs, goals, x0s = _scene_inputs(seeds, Tf, gpu)
    rec, cps, o_recs = [], [], []
    for s in seeds:  # records of a T-step horizon: the clouds' first T steps
        ovs, cells, K, ref, goal, x0 = crossing_scene(s, T=Tf)
        cells = [c[:, :T] for c in cells]
        store = engine.ParticleStore.from_cells(cells, device=gpu)
        cyc = cycle.MinkowskiCycle(store, K, ref[:T])
        cyc.run()
        rec.append(cyc.rec)
        cps.append(len(cells))
        ovs_t = [orc.OVehicle(T, ov.past, ov.latent_pmf, [c[:, :T] for c in ov.pred_positions],
                              [y[:, :T] for y in ov.pred_yaws], ov.init_center, ov.bbox)
                 for ov in ovs]
        o_recs.append(orc.minkowski_generator(ovs_t, T, T, ref[:T], with_l4=False)["records"])
    rec = torch.cat(rec, 0).contiguous()
    rng = np.random.default_rng(7)
    u_prev = rng.normal(0, 0.3, (len(seeds), 2 * (Tf - T)))
    xbar, gamma = mpc.ltv(x0s, Tf, lon=LON)
    qp = mpc.PlanningQP(cps, T, T_full=Tf)
    u, X, cost, status, _ = qp.solve(gamma, xbar, torch.as_tensor(goals, device=gpu),
                                     torch.as_tensor(refs[:, :T], device=gpu), rec,
                                     u_prev=torch.as_tensor(u_prev, device=gpu))
    status = status.cpu().numpy()
    prm = _params_dict(mpc.MPCParams.reference_defaults())
    for i in range(len(seeds)):
        want = _oracle_solve(x0s[i], T, goals[i], refs[i, :T], o_recs[i], "halfspace", prm,
                             Tf=Tf, u_prev=u_prev[i])
        if not want["feasible"]:
            assert status[i] == mpc.QP_MAXITER
            continue
        assert status[i] == mpc.QP_OK
        _check(u[i].cpu().numpy(), X[i].cpu().numpy(), float(cost[i]), want, T)


def test_qp_affine_records(gpu):
    T = 8
    seeds = _feasible(4)
    rec, cps, o_recs, refs, goals, x0s = _scene_inputs(seeds, T, gpu, kind="affine")
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    qp = mpc.PlanningQP(cps, T, kind=mpc.REC_AFFINE)
    u, X, cost, status, _ = qp.solve(gamma, xbar, torch.as_tensor(goals, device=gpu),
                                     torch.as_tensor(refs, device=gpu), rec)
    status = status.cpu().numpy()
    prm = _params_dict(mpc.MPCParams.reference_defaults())
    for i in range(len(seeds)):
        want = _oracle_solve(x0s[i], T, goals[i], refs[i], o_recs[i], "affine", prm)
        if not want["feasible"]:
            assert status[i] == mpc.QP_MAXITER
            continue
        assert status[i] == mpc.QP_OK, status
        _check(u[i].cpu().numpy(), X[i].cpu().numpy(), float(cost[i]), want, T)


def test_qp_leaves_out_failed_records_and_flags_them(gpu):
    T = 8
    rec, cps, o_recs, refs, goals, x0s = _scene_inputs(_feasible(4)[3:], T, gpu)
    h = engine.halfspaces(rec).reshape(-1)
    want_rows = list(o_recs[0])
    # fail the first binding record of the oracle solution: it must drop out of the QP
    prm = _params_dict(mpc.MPCParams.reference_defaults())
    full = _oracle_solve(x0s[0], T, goals[0], refs[0], want_rows, "halfspace", prm)
    first_obstacle = [a - 6 * T for a in full["active"] if a >= 6 * T][0]
    bad = torch.zeros(1, dtype=torch.int32)
    bad[0] = -11
    flat = rec.view(-1, 128)
    flat[first_obstacle, 120:124] = bad.view(torch.uint8).to(gpu)
    del want_rows[first_obstacle]
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    u, X, cost, status, _ = mpc.PlanningQP(cps, T).solve(
        gamma, xbar, torch.as_tensor(goals, device=gpu), torch.as_tensor(refs, device=gpu), rec)
    assert int(status[0]) == mpc.QP_OK | mpc.QP_SKIPPED_ROWS
    want = _oracle_solve(x0s[0], T, goals[0], refs[0], want_rows, "halfspace", prm)
    _check(u[0].cpu().numpy(), X[0].cpu().numpy(), float(cost[0]), want, T)
    assert h["status"][first_obstacle] == 0  # (the host copy taken before the edit)


def test_qp_feasibility_and_solution_agree_with_oracle_on_many_scenes(gpu):
    """32 more crossing scenes in one launch: the GPU solves exactly the scenes the oracle finds
    feasible (HiGHS phase 1), to the oracle's KKT-certified minimiser, and reports the rest."""
    T = 8
    seeds = list(range(100, 132))
    rec, cps, o_recs, refs, goals, x0s = _scene_inputs(seeds, T, gpu)
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    qp = mpc.PlanningQP(cps, T)
    u, X, cost, status, _ = qp.solve(gamma, xbar, torch.as_tensor(goals, device=gpu),
                                     torch.as_tensor(refs, device=gpu), rec)
    u, X, cost, status = u.cpu().numpy(), X.cpu().numpy(), cost.cpu().numpy(), status.cpu().numpy()
    prm = _params_dict(mpc.MPCParams.reference_defaults())
    n_feas = 0
    for i, s in enumerate(seeds):
        want = _oracle_solve(x0s[i], T, goals[i], refs[i], o_recs[i], "halfspace", prm)
        if not want["feasible"]:
            assert status[i] == mpc.QP_MAXITER, (s, status[i])
            continue
        n_feas += 1
        assert status[i] == mpc.QP_OK, (s, status[i])
        _check(u[i], X[i], cost[i], want, T)
    assert 1 <= n_feas <= 31   # both outcomes are exercised


@pytest.mark.parametrize("T", [12, 24])
def test_qp_longer_horizons_lds_factor(gpu, T):
    """T > 8 (n = 2T > 16): the IPM's Cholesky in LDS instead of registers, then the polish;
    ph = 12 is BASELINE configs[3]'s horizon."""
    seeds = list(range(200, 216))
    rec, cps, o_recs, refs, goals, x0s = _scene_inputs(seeds, T, gpu)
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    qp = mpc.PlanningQP(cps, T)
    u, X, cost, status, _ = qp.solve(gamma, xbar, torch.as_tensor(goals, device=gpu),
                                     torch.as_tensor(refs, device=gpu), rec)
    u, X, cost, status = u.cpu().numpy(), X.cpu().numpy(), cost.cpu().numpy(), status.cpu().numpy()
    prm = _params_dict(mpc.MPCParams.reference_defaults())
    n_feas = 0
    for i, s in enumerate(seeds):
        want = _oracle_solve(x0s[i], T, goals[i], refs[i], o_recs[i], "halfspace", prm)
        if not want["feasible"]:
            assert status[i] == mpc.QP_MAXITER, (s, status[i])
            continue
        n_feas += 1
        assert status[i] == mpc.QP_OK, (s, status[i])
        _check(u[i], X[i], cost[i], want, T)
    assert n_feas >= 1


def test_qp_refuses_malformed_inputs(gpu):
    """Raw pointers go to the kernel: wrong dtype, shape or record block must raise on the
    host, never launch."""
    T = 8
    rec, cps, o_recs, refs, goals, x0s = _scene_inputs(_feasible(2), T, gpu)
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    g_t, r_t = torch.as_tensor(goals, device=gpu), torch.as_tensor(refs, device=gpu)
    qp = mpc.PlanningQP(cps, T)
    with pytest.raises(ValueError):
        qp.solve(gamma.float(), xbar, g_t, r_t, rec)
    with pytest.raises(ValueError):
        qp.solve(gamma[:, :-4], xbar, g_t, r_t, rec)
    with pytest.raises(ValueError):
        qp.solve(gamma, xbar, g_t, r_t, rec[:1])
    with pytest.raises(ValueError):
        mpc.PlanningQP(cps, 5, T_full=8).solve(gamma, xbar, g_t, r_t[:, :5], rec)
    qp.solve(gamma, xbar, g_t, r_t, rec)          # the well-formed call still runs
    assert np.all(qp.status.cpu().numpy() >= 0)


@pytest.mark.parametrize("T", [8, 5])
def test_planning_qp_step_equals_the_direct_solve(gpu, T):
    """mpc.PlanningQPStep (what solve_planning_qp runs: inputs up in one pinned pack, LTV on the
    device at T == T_full, outputs back in one copy + a polled signal) gives the bytes of the
    plain PlanningQP.solve on the same inputs, per scene, for the full and a shrinking horizon."""
    Tf = 8
    for s in _feasible(2) + _infeasible(1):
        ovs, cells, K, ref, goal, x0 = crossing_scene(s, T=Tf)
        cells_t = [c[:, :T] for c in cells]
        store = engine.ParticleStore.from_cells(cells_t, device=gpu)
        cyc = cycle.MinkowskiCycle(store, K, ref[:T])
        cyc.run()
        u_prev = np.linspace(-0.2, 0.3, 2 * (Tf - T)) if T < Tf else None
        xbar, gamma = mpc.ltv(x0[None], Tf, lon=LON)
        qp = mpc.PlanningQP([len(cells)], T, T_full=Tf, device=gpu)
        u, X, cost, st, it = qp.solve(
            gamma, xbar, torch.as_tensor(goal[None], device=gpu),
            torch.as_tensor(ref[None, :T], device=gpu), cyc.rec,
            u_prev=None if u_prev is None else torch.as_tensor(u_prev[None], device=gpu))
        run = mpc.PlanningQPStep(len(cells), T, Tf, device=gpu)
        xb2 = torch.empty_like(xbar)
        ga2 = torch.empty_like(gamma)
        if T < Tf:      # the shrinking step reuses the full step's model
            xb2.copy_(xbar)
            ga2.copy_(gamma)
        res = run.solve(x0, goal, ref, cyc.rec, xb2, ga2, u_prev=u_prev, ltv=T == Tf,
                        lon=LON)
        assert res["status"] == int(st[0]) and res["iters"] == int(it[0])
        assert res["u"].tobytes() == u[0].cpu().numpy().tobytes()
        assert res["X_star"].tobytes() == X[0].cpu().numpy().tobytes()
        assert res["cost"] == float(cost[0])
        np.testing.assert_array_equal(res["U_star"], qp.U(u)[0].cpu().numpy())


def _solve_with_env(monkeypatch, value, seeds, T, gpu, rec_in=None):
    monkeypatch.setenv("CCMPC_QP_METHOD", "ipm")      # the interior point's own path
    if value is None:
        monkeypatch.delenv("CCMPC_QP_EARLY_POLISH", raising=False)
    else:
        monkeypatch.setenv("CCMPC_QP_EARLY_POLISH", value)
    rec, cps, o_recs, refs, goals, x0s = rec_in or _scene_inputs(seeds, T, gpu)
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    out = mpc.PlanningQP(cps, T).solve(gamma, xbar, torch.as_tensor(goals, device=gpu),
                                       torch.as_tensor(refs, device=gpu), rec)
    return [o.cpu().numpy().copy() for o in out], (rec, cps, o_recs, refs, goals, x0s)


@pytest.mark.parametrize("T", [8, 12])
def test_failed_early_polish_leaves_the_ipm_untouched(gpu, monkeypatch, T):
    """The early polish factors H in the normal matrix's storage.  A failed attempt must rebuild
    the barrier-weighted matrix before the IPM's own factor: with the attempt forced
    to fail (CCMPC_QP_EARLY_POLISH = -x: attempted at x, its answer discarded) every scene's
    status, iteration count and u are the bytes of a solve with no early attempt (= 0), at an
    early threshold (1e-1) where the active set is not yet settled and at the default one."""
    seeds = list(range(100, 124)) if T == 8 else list(range(200, 212))
    none, inp = _solve_with_env(monkeypatch, "0", seeds, T, gpu)
    for x in ("-1e-1", "-1e-2", "-1e-4"):
        forced, _ = _solve_with_env(monkeypatch, x, seeds, T, gpu, inp)
        for a, b in zip(none, forced):
            assert a.tobytes() == b.tobytes(), x
    # a real early attempt at 1e-1 either ends the solve sooner with a verified answer or fails
    # and leaves the IPM's path unchanged; either way the same minimiser and status
    early, _ = _solve_with_env(monkeypatch, "1e-1", seeds, T, gpu, inp)
    dflt, _ = _solve_with_env(monkeypatch, None, seeds, T, gpu, inp)
    for got in (early, dflt):
        assert np.array_equal(got[3], none[3])
        assert np.all(got[4] <= none[4])
        ok = none[3] == mpc.QP_OK
        scale = 1.0 + np.abs(none[0][ok]).max(axis=1, keepdims=True)
        assert np.all(np.abs(got[0][ok] - none[0][ok]) <= 1e-9 * scale)
    assert np.any(none[3] == mpc.QP_OK) and np.any(none[3] == mpc.QP_MAXITER)


def test_qp_at_the_longest_horizon(gpu):
    """T = 40 (the C5 horizon, the ABI's maximum): the LDS image must fit (the one-wave H_ctrl
    table is reserved only for n <= 16), and every solved scene is a KKT point of
    the oracle's own (H, f, G, h)."""
    T = 40
    seeds = [300, 301, 302]
    rec, cps, o_recs, refs, goals, x0s = _scene_inputs(seeds, T, gpu)
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    u, X, cost, status, iters = mpc.PlanningQP(cps, T).solve(
        gamma, xbar, torch.as_tensor(goals, device=gpu), torch.as_tensor(refs, device=gpu), rec)
    u, status = u.cpu().numpy(), status.cpu().numpy()
    prm = _params_dict(mpc.MPCParams.reference_defaults())
    n_ok = 0
    for i in range(len(seeds)):
        Gf, c = mo.state_map(gamma[i].cpu().numpy(), xbar[i].cpu().numpy(), T, T)
        rows = mo.obstacle_rows(o_recs[i], "halfspace", T)
        H, f, _, G, h = mo.assemble_qp(Gf, c, T, goals[i], refs[i], rows, prm)
        feasible = mo.is_feasible(G, h)
        if not feasible:
            assert status[i] == mpc.QP_MAXITER, (seeds[i], status[i])
            continue
        assert status[i] == mpc.QP_OK, (seeds[i], status[i])
        prim, stat, comp, _ = mo.kkt_residuals(H, f, G, h, u[i])
        assert prim <= 1e-8 and stat <= 1e-5 and comp <= 1e-6, (prim, stat, comp)
        n_ok += 1
    assert n_ok >= 1


@pytest.mark.parametrize("kind", ["halfspace", "affine"])
def test_qp_on_compact_records_equals_the_full_records(gpu, kind):
    """The multi-GPU exchange moves ccmpc_gather_rec (32 bytes: n, rhs, side, status, t_tau)
    instead of the 128-byte records: the packed fields equal the records' own, and the QP solved
    in place on the packed block (REC_*_COMPACT) gives the same bytes as on the full records."""
    from ccmpc import _lib, dist as cdist
    T = 8
    seeds = _feasible(4) + _infeasible(1)
    rec, cps, o_recs, refs, goals, x0s = _scene_inputs(seeds, T, gpu, kind=kind)
    k_full = mpc.REC_HALFSPACE if kind == "halfspace" else mpc.REC_AFFINE
    k_comp = mpc.REC_HALFSPACE_COMPACT if kind == "halfspace" else mpc.REC_AFFINE_COMPACT
    # poison one record's status: the flag must travel too
    flat = rec.view(-1, 128)
    flat[3, 120:124] = torch.tensor([-11], dtype=torch.int32).view(torch.uint8).to(gpu)
    crec = cdist.compact_records(rec, k_full)
    assert crec.shape == rec.shape[:2] + (32,)
    full = rec.cpu().numpy().reshape(-1, 128).view(
        _lib.HALFSPACE_DTYPE if kind == "halfspace" else _lib.AFFINE_DTYPE).reshape(-1)
    comp = crec.cpu().numpy().reshape(-1, 32).view(np.dtype(
        [("n0", "<f8"), ("n1", "<f8"), ("rhs", "<f8"), ("side", "<i2"), ("status", "<i2"),
         ("t_tau", "<i4")])).reshape(-1)
    assert np.array_equal(comp["n0"], full["n0"]) and np.array_equal(comp["n1"], full["n1"])
    assert np.array_equal(comp["rhs"], full["d"] if kind == "halfspace" else full["rhs"])
    assert np.array_equal(comp["side"], full["side"])
    assert np.array_equal(comp["status"], full["status"]) and comp["status"][3] == -11
    assert np.array_equal(comp["t_tau"], full["t_tau"] if kind == "halfspace" else full["t"])
    xbar, gamma = mpc.ltv(x0s, T, lon=LON)
    g_t, r_t = torch.as_tensor(goals, device=gpu), torch.as_tensor(refs, device=gpu)
    a = [x.cpu().numpy() for x in mpc.PlanningQP(cps, T, kind=k_full).solve(
        gamma, xbar, g_t, r_t, rec)]
    b = [x.cpu().numpy() for x in mpc.PlanningQP(cps, T, kind=k_comp).solve(
        gamma, xbar, g_t, r_t, crec)]
    for x, y in zip(a, b):
        assert x.tobytes() == y.tobytes()
    assert (a[3] & mpc.QP_SKIPPED_ROWS).any()
    with pytest.raises(ValueError):                  # a full block under a compact kind
        mpc.PlanningQP(cps, T, kind=k_comp).solve(gamma, xbar, g_t, r_t, rec)


@pytest.mark.parametrize("T,kind", [(8, "halfspace"), (6, "halfspace"), (8, "affine")])
def test_fused_ltv_equals_ltv_then_qp(gpu, T, kind):
    """ccmpc_mpc_qp_ltv (the LTV rebuild inside the QP's launch, what the planning frame runs at
    Tsh == ph) writes ccmpc_mpc_ltv's model bit for bit and solves to the bytes of ccmpc_mpc_ltv
    followed by ccmpc_mpc_qp -- a batch of scenes, the full and a shrinking horizon."""
    Tf = 8
    seeds = _feasible(3) + _infeasible(1)
    rec, cps, _, refs, goals, x0s = _scene_inputs(seeds, Tf, gpu, kind)
    if T < Tf:                      # the first T steps' records of each cell
        P = Tf * (Tf - 1) // 2 if kind == "halfspace" else Tf
        Pt = T * (T - 1) // 2 if kind == "halfspace" else T
        rec = rec.reshape(rec.shape[0], P, -1)[:, :Pt].contiguous()
    S = len(seeds)
    k = mpc.REC_HALFSPACE if kind == "halfspace" else mpc.REC_AFFINE
    x0_d = torch.as_tensor(x0s, device=gpu)
    goal = torch.as_tensor(goals, device=gpu)
    ref = torch.as_tensor(refs[:, :T], device=gpu).contiguous()
    up = (torch.as_tensor(np.tile(np.linspace(-0.2, 0.3, 2 * (Tf - T)), (S, 1)), device=gpu)
          if T < Tf else None)
    xbar, gamma = mpc.ltv(x0s, Tf, Ts=0.5, lon=LON)
    qa = mpc.PlanningQP(cps, T, T_full=Tf, kind=k, device=gpu)
    ua, Xa, ca, sa, ia = (t.clone() for t in qa.solve(gamma, xbar, goal, ref, rec, u_prev=up))
    xb2 = torch.full_like(xbar, float("nan"))
    ga2 = torch.full_like(gamma, float("nan"))
    qb = mpc.PlanningQP(cps, T, T_full=Tf, kind=k, device=gpu)
    ub, Xb, cb, sb, ib = qb.solve(ga2, xb2, goal, ref, rec, u_prev=up, ltv=(x0_d, 0.5, LON))
    torch.cuda.synchronize(gpu)
    assert torch.equal(xb2, xbar) and torch.equal(ga2, gamma)
    for a, b in ((ua, ub), (Xa, Xb), (ca, cb), (sa, sb), (ia, ib)):
        assert a.cpu().numpy().tobytes() == b.cpu().numpy().tobytes()
