"""No kernel reads LDS it did not write: LDS keeps whatever the previous workgroup on that CU
left there, so such a read makes results depend on what ran before (a stale-LDS read in the
QP's polish showed up as a 1e-10 difference only when other tests had run first).  Each check
fills every CU's LDS with NaN, then with zeros, then with a huge value (ccmpc_poison_lds), runs
the kernels after each fill and requires the same bytes."""
import numpy as np
import pytest
import torch

from ccmpc import _lib, cycle, engine, mpc
from _qp_inputs import crossing_scene, pick_seeds

pytestmark = pytest.mark.gpu

FILLS = (float("nan"), 0.0, 1e300)


def _poison(v):
    _lib.check(_lib.load().ccmpc_poison_lds(v, engine._stream()), "ccmpc_poison_lds")


def _same_under_fills(run):
    """run() -> list of arrays (host copies), after each fill."""
    outs = []
    for v in FILLS:
        _poison(v)
        torch.cuda.synchronize()
        outs.append([a.numpy() if torch.is_tensor(a) else np.asarray(a) for a in run()])
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert a.tobytes() == b.tobytes()
    return outs[0]


@pytest.mark.parametrize("method", ["gi", "ipm"])
@pytest.mark.parametrize("T,kind", [(8, "halfspace"), (8, "affine"), (12, "halfspace")])
def test_planning_qp_ignores_stale_lds(gpu, monkeypatch, T, kind, method):
    monkeypatch.setenv("CCMPC_QP_METHOD", method)      # (n > 16: the interior point either way)
    # binding and infeasible scenes, and one whose obstacles pass far off the path (few or no
    # active rows at the optimum: the polish's empty-active-set case)
    scenes = [(s, 8.0) for s in pick_seeds("binding", 3, T) + pick_seeds("infeasible", 1, T)]
    scenes.append((pick_seeds("binding", 1, T)[0], 80.0))
    recs, cps, refs, goals, x0s = [], [], [], [], []
    for s, lateral in scenes:
        ovs, cells, K, ref, goal, x0 = crossing_scene(s, T=T, lateral=lateral)
        store = engine.ParticleStore.from_cells(cells, device=gpu)
        cyc = (cycle.MinkowskiCycle if kind == "halfspace" else cycle.AffineCycle)(store, K, ref)
        cyc.run()
        recs.append(cyc.rec)
        cps.append(len(cells))
        refs.append(ref)
        goals.append(goal)
        x0s.append(x0)
    rec = torch.cat(recs, 0).contiguous()
    xbar, gamma = mpc.ltv(np.array(x0s), T, lon=3.7)
    qp = mpc.PlanningQP(cps, T, kind=mpc.REC_HALFSPACE if kind == "halfspace"
                        else mpc.REC_AFFINE, device=gpu)
    g = torch.as_tensor(np.array(goals), device=gpu)
    r = torch.as_tensor(np.array(refs), device=gpu)

    def run():
        u, X, cost, st, it = qp.solve(gamma, xbar, g, r, rec)
        return [u.cpu(), X.cpu(), cost.cpu(), st.cpu(), it.cpu()]
    out = _same_under_fills(run)
    assert (out[3] == 0).sum() >= 3            # the binding and far scenes solved


def test_constraint_cycle_ignores_stale_lds(gpu):
    ovs, cells, K, ref, goal, x0 = crossing_scene(pick_seeds("binding", 1)[0], T=8, N=5000)
    store = engine.ParticleStore.from_cells(cells, device=gpu)
    cyc = cycle.MinkowskiCycle(store, K, ref)

    def run():
        cyc.run()
        return [cyc.rec.cpu(), cyc.mean.cpu(), cyc.cov.cpu()]
    _same_under_fills(run)


def test_planning_step_ignores_stale_lds(gpu):
    from ccmpc import episode, planner
    O, N, ph = 3, 3000, 8
    init, pmf, gmm = episode.synthetic_gmm(O, T=ph, seed=99)
    minpos = np.array([150.0, -120.0])
    pasts = [np.array([[minpos[0] + init[o, 0] - 2.0, minpos[1] + init[o, 1]]])
             for o in range(O)]
    K = [int(np.count_nonzero(pmf[o] > 0.1)) for o in range(O)]
    eps = np.full((O, max(K)), 0.05 / O)
    ref = np.array([[165.0 + 4.0 * (t + 1), -72.0 + 0.5 * (t + 1)] for t in range(ph)])
    agent = planner.MidlevelAgent(prediction_horizon=ph, device=gpu)
    params = episode.Params(O, K, 0)

    def run():
        ovs, out = agent.predict_and_constrain(params, dict(init_state=init, latent_pmf=pmf,
                                                            gmm=gmm, N=N, seed=5), eps, ph,
                                               ref, minpos, pasts)
        return [np.array(agent.last_records).view(np.uint8)] + [
            np.array(p) for ov in ovs for p in ov.pred_positions]
    _same_under_fills(run)
