"""The `_cov` data_save format (v8ideal/__init__.py:2979-2993, save_data :2559-2567) as
npz-safe arrays: flatten -> file -> meanNtangent object grids, on the host only."""
import numpy as np

from ccmpc import planner


def _mean_tangent(K, T, rng):
    O, maxK = len(K), max(K)
    grids = [planner._object_grid(O, maxK, T) for _ in range(4)]
    for o, k_o in enumerate(K):
        for k in range(k_o):
            for t in range(T):
                grids[0][o][k][t] = rng.normal(size=2)
                grids[1][o][k][t] = float(rng.normal())
                a = rng.normal(size=(2, 2))
                grids[2][o][k][t] = a @ a.T
                grids[3][o][k][t] = int(rng.integers(-1, 2))
    return grids[0], grids[1], grids[2], 0, grids[3]


def test_data_arrays_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    K, T = [3, 1, 2], 5
    mnt = _mean_tangent(K, T, rng)
    st = tuple(planner._object_grid(len(K), max(K)) for _ in range(3))
    for g in st:
        for o, k_o in enumerate(K):
            for k in range(k_o):
                g[o][k] = float(rng.normal())
    d = {"direct": planner._object_grid(len(K)), "MeanCov": True, "OVconstraint": False,
         "ovStateMean_tau_1": st, "ovStateCov_tau_1": st, "shrinking": True,
         "meanNtangent": mnt, "x_init": np.arange(4.0), "solve_time": 0.01}
    arrs = planner._data_arrays(d, K)
    np.savez(tmp_path / "f.npz", **arrs)
    back = planner._mean_tangent_from_arrays(np.load(tmp_path / "f.npz", allow_pickle=False))
    for o, k_o in enumerate(K):
        for k in range(k_o):
            for t in range(T):
                np.testing.assert_array_equal(back[0][o][k][t], mnt[0][o][k][t])
                assert back[1][o][k][t] == mnt[1][o][k][t]
                np.testing.assert_array_equal(back[2][o][k][t], mnt[2][o][k][t])
                assert back[4][o][k][t] == mnt[4][o][k][t]
                assert isinstance(back[4][o][k][t], int)
        for k in range(k_o, max(K)):          # unused modes stay empty, as in the reference
            assert back[0][o][k][0] is None
    assert arrs["ovStateMean_tau_1"].shape == (sum(K), 3)
    assert float(arrs["solve_time"]) == 0.01
