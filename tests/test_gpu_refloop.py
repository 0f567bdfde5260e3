"""The drop-in generators on the GPU against the reference's OWN generator loops
(tests/golden/refloop_*.npz: compute_obstacle_constraints_GMM_Minkowski_idealprediction
v8ideal/__init__.py:781-964, compute_obstacle_constraints_GMM_affine :1378-1539 and save_moments
:2575-2618 executed unchanged by make_golden.py with a recording cvxpy):

* constraint order, step t and side (>= / <=) bit-exact; n and the right-hand side to 1e-9;
* the 9-tuple's ovStateMean/Cov_tau_1 (:864-875) and OVconstraint (:831-851);
* prob_lower_save (:947, :961-962) and the saved moments (mean, cov, cross_cov);
* at T = 12 with three OVs, at T = 40 (780 pairs per cell), and one shrinking step (ph = 8,
  T = 7) on injected ideal trajectories -- the Tpred = T switch (:885-888) with eps / ph.
"""
import numpy as np
import pytest
import torch

from _cycle_inputs import REFLOOP, refloop_inputs

pytestmark = pytest.mark.gpu


def _check_constraints(cons, g, kind):
    assert len(cons) == len(g[f"{kind}_t"])
    np.testing.assert_array_equal([c.t for c in cons], g[f"{kind}_t"])
    np.testing.assert_array_equal([c.side for c in cons], g[f"{kind}_side"])
    n = np.array([c.n for c in cons])
    rhs = np.array([c.rhs for c in cons])
    scale = np.maximum(np.abs(g[f"{kind}_n"]), 1.0)
    assert np.max(np.abs(n - g[f"{kind}_n"]) / scale) < 1e-9
    np.testing.assert_allclose(rhs, g[f"{kind}_rhs"], rtol=1e-9, atol=1e-9)


def _state(out, K):
    cells = [(o, k) for o in range(len(K)) for k in range(K[o])]
    sm = np.array([[out[6][j][o][k] for j in range(3)] for o, k in cells], float)
    sc = np.array([[out[7][j][o][k] for j in range(3)] for o, k in cells], float)
    return sm, sc


@pytest.mark.parametrize("name", [n for n in REFLOOP if "shrink" not in n])
def test_drop_in_generators_match_reference_loops(gpu, golden, name):
    from ccmpc import episode, ovehicle, planner
    g = golden(name)
    K, T, ph, cells, yaws, _ = refloop_inputs(g)
    agent = planner.MidlevelAgent(prediction_horizon=ph, device=gpu)
    pasts = [np.asarray(p).reshape(1, 2) for p in g["past"]]
    ovs = ovehicle.scene_from_positions(cells, pasts, device=gpu)
    params = episode.Params(len(K), K, 40)
    eps_ura = np.full((len(K), max(K)), 0.05 / len(K))
    out = agent.compute_obstacle_constraints_GMM_Minkowski_idealprediction(
        params, ovs, None, None, None, eps_ura, None, T, g["ref_traj"])
    _check_constraints(out[0], g, "mk")
    assert out[4] == bool(g["mk_ovconstraint"])
    sm, sc = _state(out, K)
    np.testing.assert_allclose(sm, g["mk_state_mean"], rtol=1e-12)
    np.testing.assert_allclose(sc, g["mk_state_cov"], rtol=1e-9)
    np.testing.assert_allclose(np.array(agent.prob_lower_save, float), g["mk_prob_lower_save"],
                               rtol=1e-8, atol=1e-13)
    mom = agent.saved_moments(40)
    for c, (o, k) in enumerate([(o, k) for o in range(len(K)) for k in range(K[o])]):
        for t in range(T):
            np.testing.assert_allclose(mom["mean_p0p1"][o][k][t], g["mom_mean"][c, t],
                                       rtol=1e-13)
            np.testing.assert_allclose(mom["cov_p0p1"][o][k][t], g["mom_cov"][c, t],
                                       rtol=1e-10, atol=1e-12)
            for tau in range(t):
                np.testing.assert_allclose(mom["cross_cov"][o][k][t][tau],
                                           g["mom_xcov"][c, t, tau], rtol=1e-10, atol=1e-12)
    out_a = agent.compute_obstacle_constraints_GMM_affine(
        params, ovs, None, None, None, eps_ura, None, T, g["ref_traj"])
    _check_constraints(out_a[0], g, "aff")
    sm, sc = _state(out_a, K)
    np.testing.assert_allclose(sm, g["aff_state_mean"], rtol=1e-12)
    np.testing.assert_allclose(sc, g["aff_state_cov"], rtol=1e-9)


def test_shrinking_step_matches_reference_loop(gpu, golden):
    """ph = 8, T = 7: the reference's generator on injected ideal trajectories (its
    predict_ideal stubbed to return them).  The constraints come from the ideal clouds with
    Tpred = T and eps = eps_ura / ph; the state statistics from the sampler particles (Tpred =
    ph); the saved moments from the ideal clouds.  On the GPU: the one-launch cycle over an
    f64 store of the same ideal clouds with ph = 8, and the scene's moments / L4."""
    from ccmpc import cycle, engine, ovehicle, planner
    from ccmpc.planner import HalfSpaceList
    g = golden("refloop_shrink_t7")
    K, T, ph, cells, yaws, ideal = refloop_inputs(g)
    assert T < ph
    store = engine.ParticleStore.from_cells(ideal, device=gpu)
    cyc = cycle.MinkowskiCycle(store, K, g["ref_traj"][:T], ph=ph)
    cyc.run()
    cell_of = [(o, k) for o in range(len(K)) for k in range(K[o])]
    cons = HalfSpaceList(cyc.records(), cell_of, T * (T - 1) // 2)
    _check_constraints(list(cons), g, "mk")
    np.testing.assert_allclose(cyc.mean.cpu().numpy(), g["mom_mean"], rtol=1e-13)
    cov = cyc.cov.cpu().numpy()
    for t in range(T):
        np.testing.assert_allclose(cov[:, 2 * t:2 * t + 2, 2 * t:2 * t + 2], g["mom_cov"][:, t],
                                   rtol=1e-10, atol=1e-12)
        for tau in range(t):
            np.testing.assert_allclose(cov[:, 2 * t:2 * t + 2, 2 * tau:2 * tau + 2],
                                       g["mom_xcov"][:, t, tau], rtol=1e-10, atol=1e-12)
    # ovStateMean/Cov_tau_1 of the shrinking step: the sampler particles' t = 0 statistics
    agent = planner.MidlevelAgent(prediction_horizon=ph, device=gpu)
    ovs = ovehicle.scene_from_positions(cells, [np.asarray(p).reshape(1, 2) for p in g["past"]],
                                        device=gpu)
    scene = ovs[0].scene
    m, c = engine.moments(scene.store)
    sm, sc = agent._state_stats(scene, m[:, 0, :].cpu().numpy(), c[:, 0:2, 0:2].cpu().numpy())
    got_m = np.array([[sm[j][o][k] for j in range(3)] for o, k in cell_of], float)
    got_c = np.array([[sc[j][o][k] for j in range(3)] for o, k in cell_of], float)
    np.testing.assert_allclose(got_m, g["mk_state_mean"], rtol=1e-12)
    np.testing.assert_allclose(got_c, g["mk_state_cov"], rtol=1e-9)
    assert not torch.isnan(cyc.mean).any()
