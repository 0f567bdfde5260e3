"""Host-side risk allocation constants (v8ideal/__init__.py:2920-2926, :910-913, :1481-1482).

These are per-cell scalars computed once per planning step with the same scipy calls the
reference makes inside its inner loop; the kernels receive them as data.
"""
import functools

import numpy as np
import scipy.stats

EPS_TOTAL = 0.05      # v8ideal/__init__.py:2920
TARGET_P = 0.9999     # v8ideal/__init__.py:912
R_COLLISION = 3.4     # v8ideal/__init__.py:795


def eps_ura(K, eps=EPS_TOTAL):
    """eps_ura[i, k] = eps / O for every mode of every OV (not divided by K)."""
    K = [int(k) for k in K]
    O = len(K)
    out = np.zeros((O, max(K) if O else 0))
    for i, k in enumerate(K):
        out[i, :k] = eps / O
    return out


@functools.lru_cache(maxsize=4096)
def _chi2_ppf2(p):
    """scipy.stats.chi2.ppf(p, df=2), memoised: the reference's value, computed once per
    distinct probability (a planning episode reuses a handful)."""
    return float(scipy.stats.chi2.ppf(p, df=2))


@functools.lru_cache(maxsize=4096)
def _norm_ppf(p):
    return float(scipy.stats.norm.ppf(p))


def cell_risk(eps_ura_mat, K, ph, target_p=TARGET_P):
    """(n_cells, 3) = chi2.ppf(1-eps_ijt, 2), chi2.ppf(target_p, 2), norm.ppf(1-eps_ijt) with
    eps_ijt = eps_ura[ov, k] / ph, cells in (ov, k) order."""
    chi_p = _chi2_ppf2(float(target_p))
    rows = []
    for o, k_o in enumerate(K):
        for k in range(int(k_o)):
            e = float(eps_ura_mat[o, k]) / ph
            rows.append((_chi2_ppf2(1 - e), chi_p, _norm_ppf(1 - e)))
    return np.asarray(rows, dtype=np.float64).reshape(-1, 3)


def scenes_cell_risk(scene_K, ph, target_p=TARGET_P):
    """cell_risk of several independent planning steps batched into one cycle: each scene
    allocates its own risk, eps_ura = 0.05 / O_scene (v8ideal/__init__.py:2920-2926)."""
    parts = [cell_risk(eps_ura(K), K, ph, target_p) for K in scene_K]
    return np.concatenate(parts, 0) if parts else np.zeros((0, 3))


def cell_gamma(eps_ura_mat, K, ph):
    """(n_cells,) = norm.ppf(1 - eps_ura[ov, k] / ph) for the GMM-affine generator."""
    return cell_risk(eps_ura_mat, K, ph)[:, 2].copy()
