// Half-space assembly: Minkowski/MVOE (v8ideal/__init__.py:893-947) and GMM-affine
// (v8ideal/__init__.py:1470-1515), both fed by ccmpc_moments output.
//
// One lane per (cell, t, tau) pair for the Minkowski generator: the work per pair is scalar
// float64 arithmetic on 2x2 matrices plus the MVOE fixed point (median ~10 iterations), so the
// kernel is latency-bound and tiny next to the moment reduction.  One wave per (cell, t): its
// lanes tau < t are the row's pairs, all in flight at once (one chain deep, at any T), and the
// per-t minimum of the lower bound is a wave reduction.  (One workgroup per cell ran T = 40's
// 780 pairs in four rounds of chains.)
//
// Every step follows the reference's operation order (which matrix is formed first, the
// strict '<' tie-break, the side test n.mean <= d) so that the integer outputs (which, side)
// match bit-for-bit and the floating outputs match to rounding.
#include "constraints.hpp"

namespace ccmpc {

__global__ __launch_bounds__(64) void minkowski_rows_kernel(const double *__restrict__ mean,
                                                            const double *__restrict__ cov, int T,
                                                            MinkParams mp) {
  const int cell = blockIdx.x, t = blockIdx.y, tau = threadIdx.x;
  const int rows = 2 * T;
  const int rsel = mp.cell_ref ? mp.cell_ref[cell] : 0;
  const double *ref = mp.ref_traj + static_cast<int64_t>(rsel) * rows;
  const double *C = cov + static_cast<int64_t>(cell) * rows * rows;
  const double *mu = mean + static_cast<int64_t>(cell) * rows;
  double lb = 1.0;
  if (tau < t) {
    const int p = t * (t - 1) / 2 + tau;
    ccmpc_halfspace *rec = mp.out_rec + static_cast<int64_t>(cell) * (T * (T - 1) / 2) + p;
    const double *risk = mp.cell_risk + 3 * cell;
    lb = pair_lower_bound(pair_moments(C, rows, t, tau), risk[2]);
    rec->lower_bound = lb;
    minkowski_pair(C, mu, ref, rows, t, tau, risk[0], risk[1], mp.R, mp.tol, mp.maxiter, rec);
  }
  // prob_lower[t] = fmin over the row from 1.0 (:946; fmin ignores NaN in any order, and the
  // lanes tau >= t hold the 1.0 start)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lb = fmin(lb, __shfl_xor(lb, o, 64));
  if (tau == 0) mp.out_prob_lower[static_cast<int64_t>(cell) * T + t] = lb;
}

__global__ __launch_bounds__(64) void affine_kernel(
    const double *__restrict__ mean, const double *__restrict__ cov, int T, int n_cells,
    const double *__restrict__ ref_traj, const int32_t *__restrict__ cell_ref,
    const double *__restrict__ cell_gamma, double R, ccmpc_affine_rec *__restrict__ out) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(n_cells) * T) return;
  const int cell = static_cast<int>(idx / T), t = static_cast<int>(idx % T);
  const int rows = 2 * T;
  const double *C = cov + static_cast<int64_t>(cell) * rows * rows;
  const double *mu = mean + static_cast<int64_t>(cell) * rows;
  const int rsel = cell_ref ? cell_ref[cell] : 0;
  const double *ref = ref_traj + static_cast<int64_t>(rsel) * rows;
  const double gamma = cell_gamma[cell];
  ccmpc_affine_rec h;
  h.status = 0;
  h.t = t;
  const M2 c = block(C, rows, t, t);
  // sqrtm of a 2x2 SPD matrix: (A + sqrt(det) I) / sqrt(tr + 2 sqrt(det))   (:1494)
  const double det = c.a * c.d - c.b * c.c;
  double s00 = NAN, s01 = NAN, s11 = NAN;
  if (det >= 0.0 && c.a + c.d > 0.0) {
    const double sd = sqrt(det);
    const double inv_tau = 1.0 / sqrt(c.a + c.d + 2.0 * sd);
    s00 = (c.a + sd) * inv_tau;
    s01 = c.b * inv_tau;
    s11 = (c.d + sd) * inv_tau;
  } else {
    h.status = CCMPC_REC_NOT_PSD;
  }
  const double m0 = mu[2 * t], m1 = mu[2 * t + 1];
  const double a0 = ref[2 * t], a1 = ref[2 * t + 1];
  const double m = -(a0 - m0) / (a1 - m1);
  // || sqrtm(cov) [m, -1]^T ||_2
  const double v0 = s00 * m - s01, v1 = s01 * m - s11;
  const double margin = gamma * sqrt(v0 * v0 + v1 * v1);
  const double n0 = -m, n1 = 1.0;
  double d = NAN, rhs = NAN;
  int which = 0, side = 0;
  if (!isfinite(m)) {
    if (h.status == 0) h.status = CCMPC_REC_NONFINITE;
  } else {
    // choose_closest_tangent(mean, I, R, m, ref) (:1502)
    const double q = n0 * n0 + n1 * n1;
    const double proj = n0 * m0 + n1 * m1;
    const double delta = R * sqrt(q);
    const double d1 = proj + delta, d2 = proj - delta;
    const double nrm = sqrt(n0 * n0 + n1 * n1);
    const double na = n0 * a0 + n1 * a1;
    const double dist0 = fabs(na - d1) / nrm, dist1 = fabs(na - d2) / nrm;
    which = (dist1 < dist0) ? 1 : 0;
    d = which ? d2 : d1;
    side = (proj <= d) ? 1 : -1;
    rhs = side > 0 ? d + margin : d - margin;
  }
  h.n0 = n0;
  h.n1 = n1;
  h.d = d;
  h.margin = margin;
  h.rhs = rhs;
  h.mean0 = m0;
  h.mean1 = m1;
  h.c00 = c.a;
  h.c01 = c.b;
  h.c11 = c.d;
  h.s00 = s00;
  h.s01 = s01;
  h.s11 = s11;
  h.m = m;
  h.which = which;
  h.side = side;
  out[idx] = h;
}

// compute_obstacle_constraints_GMM_affine_scale_ideal (v8ideal/__init__.py:2074-2456) per cell:
// scale(t) = max(1, max_{tau<t} compute_scale(predict_moments(t, tau), Gamma, chi_p))
// (makeconstraint.py:259-280), cov = scale C_tt, and a slope-m tangent of the radius-R circle
// around the mean with margin Gamma sqrt(|cov|_F) |[m, -1]|.  Threads first cover the cell's
// (t, tau) pairs (per-t max in LDS, scale >= 1 so an int compare of the bits is an exact max),
// then one thread per t builds the record.
__global__ __launch_bounds__(256) void affine_scale_kernel(
    const double *__restrict__ mean, const double *__restrict__ cov, int T,
    const double *__restrict__ ref_traj, const int32_t *__restrict__ cell_ref,
    const double *__restrict__ cell_risk, double R, int scaled,
    const double *__restrict__ tangent_in, const int32_t *__restrict__ const_idx_in,
    ccmpc_affine_rec *__restrict__ out) {
  __shared__ unsigned long long scale_bits[40];
  const int cell = blockIdx.x, rows = 2 * T;
  const double *C = cov + static_cast<int64_t>(cell) * rows * rows;
  const double *mu = mean + static_cast<int64_t>(cell) * rows;
  const double chi_p = cell_risk[3 * cell + 1], gamma = cell_risk[3 * cell + 2];
  const double one = 1.0;
  for (int t = threadIdx.x; t < T; t += blockDim.x)
    scale_bits[t] = static_cast<unsigned long long>(__double_as_longlong(one));
  __syncthreads();
  const int P = scaled ? T * (T - 1) / 2 : 0;  // _affine_robust: scale = 1 (:1766)
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    int t, tau;
    pair_of(p, t, tau);
    const double sc = pair_scale(pair_moments(C, rows, t, tau), chi_p, gamma);
    // positive doubles order like their bit patterns; NaN (all-ones exponent) also wins, as
    // np.max propagates it
    atomicMax(&scale_bits[t], static_cast<unsigned long long>(__double_as_longlong(sc)));
  }
  __syncthreads();
  const int rsel = cell_ref ? cell_ref[cell] : 0;
  const double *ref = ref_traj + static_cast<int64_t>(rsel) * rows;
  for (int t = threadIdx.x; t < T; t += blockDim.x) {
    ccmpc_affine_rec h;
    h.status = 0;
    h.t = t;
    const double sf = __longlong_as_double(static_cast<long long>(scale_bits[t]));
    const M2 c = block(C, rows, t, t);
    const M2 cs = scale(c, sf);
    const double cov_fro_sqrt = sqrt(fro(cs));
    const double m0 = mu[2 * t], m1 = mu[2 * t + 1];
    const double a0 = ref[2 * t], a1 = ref[2 * t + 1];
    const int64_t slot = static_cast<int64_t>(cell) * T + t;
    const double m = tangent_in ? tangent_in[slot] : -(a0 - m0) / (a1 - m1);
    const int ci = (tangent_in && const_idx_in) ? const_idx_in[slot] : CCMPC_TANGENT_CHOOSE;
    const double margin = gamma * cov_fro_sqrt * sqrt(m * m + 1.0);  // |[m, -1]|_2
    const double n0 = -m, n1 = 1.0;
    double d = NAN, rhs = NAN;
    int which = 0, side = 0;
    if (!isfinite(m) || !isfinite(sf)) {
      h.status = CCMPC_REC_NONFINITE;
    } else {
      // choose_closest_tangent(mean, I, R, m, ref, const_idx) (makeconstraint.py:176-207)
      const double proj = n0 * m0 + n1 * m1;
      const double delta = R * sqrt(n0 * n0 + n1 * n1);
      const double d1 = proj + delta, d2 = proj - delta;
      int pick;
      if (ci == CCMPC_TANGENT_CHOOSE) {
        const double nrm = sqrt(n0 * n0 + n1 * n1);
        const double na = n0 * a0 + n1 * a1;
        const double dist0 = fabs(na - d1) / nrm, dist1 = fabs(na - d2) / nrm;
        pick = (dist1 < dist0) ? 1 : 0;
        which = pick;
      } else {
        pick = ci < 0 ? ci + 2 : ci;  // Python indexing of the 2-candidate list
        which = ci;                   // the reference returns the index it was given
      }
      d = pick ? d2 : d1;
      side = (proj <= d) ? 1 : -1;     // (:2379) n.mean <= d  ->  n.x >= d + margin
      rhs = side > 0 ? d + margin : d - margin;
    }
    h.n0 = n0;
    h.n1 = n1;
    h.d = d;
    h.margin = margin;
    h.rhs = rhs;
    h.mean0 = m0;
    h.mean1 = m1;
    h.c00 = c.a;  // the original (unscaled) cov is what the generator saves (:2425)
    h.c01 = c.b;
    h.c11 = c.d;
    h.s00 = sf;
    h.s01 = cov_fro_sqrt;
    h.s11 = 0.0;
    h.m = m;
    h.which = which;
    h.side = side;
    out[slot] = h;
  }
}

void launch_minkowski_rows(const double *mean, const double *cov, int T, int n_cells,
                           const MinkParams &mp, hipStream_t s) {
  hipLaunchKernelGGL(minkowski_rows_kernel,
                     dim3(static_cast<unsigned>(n_cells), static_cast<unsigned>(T)), dim3(64), 0,
                     s, mean, cov, T, mp);
}

}  // namespace ccmpc

using namespace ccmpc;

extern "C" int ccmpc_minkowski(const double *mean, const double *cov, int64_t T, int64_t n_cells,
                               const double *ref_traj, const int32_t *cell_ref,
                               const double *cell_risk, double R, double tol, int32_t maxiter,
                               ccmpc_halfspace *out_rec, double *out_prob_lower,
                               ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T >= 1 && T <= 40, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_cells >= 0 && n_cells < (1 << 30), "bad n_cells");
  if (n_cells == 0) return CCMPC_OK;
  CCMPC_REQUIRE(mean && cov && ref_traj && cell_risk && out_rec && out_prob_lower, "null pointer");
  CCMPC_REQUIRE(maxiter >= 1, "maxiter must be >= 1");
  const MinkParams mp{ref_traj, cell_ref, cell_risk, R, tol, maxiter, out_rec, out_prob_lower};
  launch_minkowski_rows(mean, cov, static_cast<int>(T), static_cast<int>(n_cells), mp,
                        as_stream(stream));
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}

extern "C" int ccmpc_affine(const double *mean, const double *cov, int64_t T, int64_t n_cells,
                            const double *ref_traj, const int32_t *cell_ref,
                            const double *cell_gamma, double R, ccmpc_affine_rec *out_rec,
                            ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T >= 1 && T <= 40, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_cells >= 0 && n_cells < (1 << 30), "bad n_cells");
  if (n_cells == 0) return CCMPC_OK;
  CCMPC_REQUIRE(mean && cov && ref_traj && cell_gamma && out_rec, "null pointer");
  const int64_t total = n_cells * T;
  const unsigned blocks = static_cast<unsigned>((total + 63) / 64);
  hipLaunchKernelGGL(affine_kernel, dim3(blocks), dim3(64), 0, as_stream(stream), mean, cov,
                     static_cast<int>(T), static_cast<int>(n_cells), ref_traj, cell_ref,
                     cell_gamma, R, out_rec);
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}

extern "C" int ccmpc_affine_scale(const double *mean, const double *cov, int64_t T,
                                  int64_t n_cells, const double *ref_traj,
                                  const int32_t *cell_ref, const double *cell_risk, double R,
                                  int32_t scaled, const double *tangent_in,
                                  const int32_t *const_idx_in, ccmpc_affine_rec *out_rec,
                                  ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T >= 1 && T <= 40, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_cells >= 0 && n_cells < (1 << 30), "bad n_cells");
  if (n_cells == 0) return CCMPC_OK;
  CCMPC_REQUIRE(mean && cov && ref_traj && cell_risk && out_rec, "null pointer");
  hipLaunchKernelGGL(affine_scale_kernel, dim3(static_cast<unsigned>(n_cells)), dim3(256), 0,
                     as_stream(stream), mean, cov, static_cast<int>(T), ref_traj, cell_ref,
                     cell_risk, R, static_cast<int>(scaled != 0), tangent_in, const_idx_in,
                     out_rec);
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}
