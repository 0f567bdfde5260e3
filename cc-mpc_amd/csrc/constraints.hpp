// Per-record math of the half-space generators, shared by the standalone kernels
// (constraints.hip) and the fused moments -> half-space kernels (moments.hip, rollout.hip).
//
// Every step follows the reference's operation order (which matrix is formed first, the
// strict '<' tie-break, the side test n.mean <= d) so that the integer outputs (which, side)
// match bit-for-bit and the floating outputs match to rounding.
#pragma once
#include "ccmpc_common.hpp"

namespace ccmpc {


struct M2 {
  double a, b, c, d;  // [[a, b], [c, d]]
};

__device__ __forceinline__ M2 mul(const M2 &x, const M2 &y) {
  return {x.a * y.a + x.b * y.c, x.a * y.b + x.b * y.d, x.c * y.a + x.d * y.c,
          x.c * y.b + x.d * y.d};
}
__device__ __forceinline__ M2 scale(const M2 &x, double s) {
  return {x.a * s, x.b * s, x.c * s, x.d * s};
}
__device__ __forceinline__ M2 sub(const M2 &x, const M2 &y) {
  return {x.a - y.a, x.b - y.b, x.c - y.c, x.d - y.d};
}
__device__ __forceinline__ M2 add(const M2 &x, const M2 &y) {
  return {x.a + y.a, x.b + y.b, x.c + y.c, x.d + y.d};
}
__device__ __forceinline__ M2 transpose(const M2 &x) { return {x.a, x.c, x.b, x.d}; }

// Latency-lean f64 reciprocal and square root for the MVOE chain (a serial dependency chain per
// record, so each IEEE div / sqrt fix-up sequence is pure latency): hardware estimate + Newton /
// Goldschmidt refinement, <= ~2 ulp on the well-scaled values here (covariances, beta ~ 1),
// against the 1e-5 relative Frobenius parity bar on Q.  The tangent choice and side test keep
// IEEE division, so which / side stay decided exactly as the reference decides them.
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  r = fma(fma(-x, r, 1.0), r, r);
  return r;
}

__device__ __forceinline__ double div_nr(double a, double b) {
  const double r = rcp_nr(b);
  const double q = a * r;
  return fma(fma(-b, q, a), r, q);  // one residual correction
}

__device__ __forceinline__ double sqrt_gs(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-g, h, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  const double d = fma(-g, g, x);
  return x > 0.0 ? fma(d, h, g) : (x == 0.0 ? 0.0 : NAN);
}

// Inverse by LU with partial pivoting, as LAPACK getrf/getri does it for 2x2.  Branch-free:
// the pivot row is selected, not branched on (lanes of a wave pick different pivots, and a
// branch would run both LU paths back to back); the arithmetic per pivot choice is unchanged.
__device__ __forceinline__ bool inv2(const M2 &m, M2 &out) {
  const bool piv = fabs(m.c) > fabs(m.a);
  const double p0 = piv ? m.c : m.a, p1 = piv ? m.d : m.b;  // pivot row of P m
  const double q0 = piv ? m.a : m.c, q1 = piv ? m.b : m.d;  // other row
  const double i11 = rcp_nr(p0);
  const double l = q0 * i11;
  const double u22 = q1 - l * p1;
  const double i22 = rcp_nr(u22);
  const double i12 = -p1 * i11 * i22;
  // inv(U) = [[i11, i12], [0, i22]]; inv(L) = [[1, 0], [-l, 1]]; inv(P m) = inv(U) inv(L)
  const double x11 = i11 - i12 * l, x12 = i12, x21 = -i22 * l, x22 = i22;
  out = piv ? M2{x12, x11, x22, x21} : M2{x11, x12, x21, x22};  // inv(m) = inv(P m) P
  return p0 != 0.0 && u22 != 0.0;
}

// solve(S1, S2) = S1^{-1} S2 by the same LU (scipy.linalg.solve -> gesv)
__device__ __forceinline__ bool solve2(const M2 &s1, const M2 &s2, M2 &out) {
  M2 inv;
  if (!inv2(s1, inv)) return false;
  out = mul(inv, s2);
  return true;
}

// makeconstraint.py:7-38
__device__ bool compute_mvoe(const M2 &S1, const M2 &S2, double tol, int maxiter, double &beta,
                             M2 &Q) {
  M2 M;
  if (!solve2(S1, S2, M)) return false;
  const double half_tr = 0.5 * (M.a + M.d);
  const double hd = 0.5 * (M.a - M.d);
  const double disc = hd * hd + M.b * M.c;
  // complex pair (disc < 0): .real keeps the real part of both
  const double sd = disc >= 0.0 ? sqrt_gs(disc) : 0.0;
  const double l1 = half_tr + sd, l2 = half_tr - sd;
  // beta' = sqrt(sum 1/w / sum l/w), w = 1 + beta l  ==  sqrt(N / D) with N = w1 + w2 =
  // 2 + s beta and D = l1 w2 + l2 w1 = s + 2 p beta (s = l1 + l2, p = l1 l2)  ==  N rsqrt(N D):
  // the same fixed point, each step one product, one hardware rsqrt and one Goldschmidt step
  // (7 dependent f64 operations, against 17 for an IEEE division + square root; the iteration
  // is a serial chain per record, so its latency is the tail's critical path).  Rounding
  // differs from the reference's order by a few ulp per step; the contraction damps it.
  const double s = l1 + l2, p2 = 2.0 * (l1 * l2);
  double b = 1.0;
  for (int it = 0; it < maxiter; ++it) {
    const double N = fma(s, b, 2.0), D = fma(p2, b, s);
    const double x = N * D;
    const double y = __builtin_amdgcn_rsq(x);
    const double g = x * y, h = 0.5 * y;
    const double r = fma(-g, h, 0.5);
    const double bn = (2.0 * N) * fma(h, r, h);
    const bool done = fabs(bn - b) < tol;
    b = bn;
    if (done) break;
  }
  beta = b;
  Q = add(scale(S1, 1.0 + rcp_nr(b)), scale(S2, 1.0 + b));
  return true;
}

__device__ __forceinline__ double fro(const M2 &m) {
  return sqrt(m.a * m.a + m.b * m.b + m.c * m.c + m.d * m.d);
}

__device__ __forceinline__ M2 block(const double *cov, int rows, int i, int j) {
  const double *p = cov + (2 * i) * rows + 2 * j;
  return {p[0], p[1], p[rows], p[rows + 1]};
}

__device__ __forceinline__ void pair_of(int p, int &t, int &tau) {
  int tt = static_cast<int>((1.0f + sqrtf(1.0f + 8.0f * static_cast<float>(p))) * 0.5f);
  while (tt * (tt - 1) / 2 > p) --tt;
  while ((tt + 1) * tt / 2 <= p) ++tt;
  t = tt;
  tau = p - tt * (tt - 1) / 2;
}


// 16-byte store of two adjacent record fields (records are 128-byte aligned).
static_assert(sizeof(ccmpc_halfspace) == 128, "record size");
static_assert(offsetof(ccmpc_halfspace, d) == 16 && offsetof(ccmpc_halfspace, q01) == 32 &&
                  offsetof(ccmpc_halfspace, r00) == 48 && offsetof(ccmpc_halfspace, r11) == 64 &&
                  offsetof(ccmpc_halfspace, mean0) == 96 && offsetof(ccmpc_halfspace, which) == 112,
              "16-byte field pairs of ccmpc_halfspace");
__device__ __forceinline__ void store_pair(double *p, double a, double b) {
  *reinterpret_cast<double2 *>(p) = make_double2(a, b);
}

struct MinkParams {
  const double *ref_traj;    // [n_ref][T][2]
  const int32_t *cell_ref;   // [n_cells] or NULL
  const double *cell_risk;   // [n_cells][3] chi_r, chi_p, gamma
  double R, tol;
  int maxiter;
  ccmpc_halfspace *out_rec;  // [n_cells][P]
  double *out_prob_lower;    // [n_cells][T]
};

// predict_moments (makeconstraint.py:41-70) from blocks of the 2T x 2T covariance:
// cov_mu = C_t,tau C_tau^-1 C_tau,t and cov_infer = C_t - cov_mu.
struct PairMoments {
  M2 c_t, cov_mu, cov_infer;
  bool ok;
};

__device__ __forceinline__ PairMoments pair_moments(const double *C, int rows, int t, int tau) {
  PairMoments pm;
  pm.c_t = block(C, rows, t, t);
  const M2 c_x = block(C, rows, t, tau);
  const M2 c_xT = block(C, rows, tau, t);
  M2 inv_tau;
  pm.ok = inv2(block(C, rows, tau, tau), inv_tau);
  pm.cov_mu = mul(mul(c_x, inv_tau), c_xT);
  pm.cov_infer = sub(pm.c_t, pm.cov_mu);
  return pm;
}

// compute_lower_bound (makeconstraint.py:282-303):
// alpha = sqrt|cov_infer|_F / sqrt|C_t|_F, beta likewise with cov_mu, p = chi2_2 cdf
// ((Gamma (1 - alpha) / beta)^2) = 1 - exp(-x / 2).
__device__ __forceinline__ double pair_lower_bound(const PairMoments &pm, double gamma) {
  const double root_t = sqrt(fro(pm.c_t));
  const double al = sqrt(fro(pm.cov_infer)) / root_t;
  const double be = sqrt(fro(pm.cov_mu)) / root_t;
  const double x = gamma * (1.0 - al) / be;
  return -expm1(-0.5 * (x * x));
}

// compute_scale (makeconstraint.py:259-280): (sqrt(chi_p) beta / Gamma + alpha)^2.
__device__ __forceinline__ double pair_scale(const PairMoments &pm, double chi_p, double gamma) {
  const double root_t = sqrt(fro(pm.c_t));
  const double alpha = sqrt(fro(pm.cov_infer)) / root_t;
  const double beta = sqrt(fro(pm.cov_mu)) / root_t;
  const double x = sqrt(chi_p) * beta / gamma + alpha;
  return x * x;
}

// tangent_lines_of_slope_m + choose_closest_tangent (makeconstraint.py:134-207) for the normal
// n = [n0, n1] = [-m, 1] of a finite slope m, with the quantities that depend only on the mean
// and the point a precomputed by the caller: proj = n.mu, nrm = |n|, na = n.a.  Picks the
// candidate d = proj +- c sqrt(n^T S n) nearer to a under the reference's strict '<' (ties and
// NaN distances keep index 0).  Returns 0, or CCMPC_REC_NO_TANGENT where the reference returns
// its None tuple (n^T S n <= 0; a NaN n^T S n gives NaN candidates, decided by the caller's
// finiteness check).
__device__ __forceinline__ int closest_tangent(const M2 &S, double c, double n0, double n1,
                                               double proj, double nrm, double na, double &d,
                                               int &which) {
  const double sn0 = S.a * n0 + S.b * n1, sn1 = S.c * n0 + S.d * n1;
  const double q = n0 * sn0 + n1 * sn1;
  if (q <= 0.0) {
    d = NAN;
    which = 0;
    return CCMPC_REC_NO_TANGENT;
  }
  const double delta = c * sqrt(q);
  const double d1 = proj + delta, d2 = proj - delta;
  const double dist0 = fabs(na - d1) / nrm, dist1 = fabs(na - d2) / nrm;
  which = (dist1 < dist0) ? 1 : 0;
  d = which ? d2 : d1;
  return 0;
}

// One (cell, t, tau) record except its lower bound, from the cell's 2T x 2T covariance C (row
// stride `rows`) and mean mu (v8ideal/__init__.py:893-943), written straight to `out`.
__device__ void minkowski_pair(const double *C, const double *mu, const double *ref, int rows,
                               int t, int tau, double chi_r, double chi_p, double R, double tol,
                               int maxiter, ccmpc_halfspace *out) {
  // the tangent's slope and everything that depends only on the mean and the reference
  // point: computed ahead of the MVOE fixed points (straight-line code the scheduler overlaps
  // with the pair-moment chain; after the data-dependent loops it would be pure latency)
  const double m0 = mu[2 * t], m1 = mu[2 * t + 1];
  const double a0 = ref[2 * t], a1 = ref[2 * t + 1];
  const double m = -(a0 - m0) / (a1 - m1);
  const double n0 = -m, n1 = 1.0;
  const double proj = n0 * m0 + n1 * m1;
  const double nrm = sqrt(n0 * n0 + n1 * n1);
  const double na = n0 * a0 + n1 * a1;
  // the record goes out in 16-byte pairs (the lower bound at byte 88 belongs to another
  // thread), the fields known early ahead of the chain, so few stores follow its end
  store_pair(&out->n0, n0, n1);
  store_pair(&out->mean0, m0, m1);
  const PairMoments pm = pair_moments(C, rows, t, tau);
  int status = 0;
  // two MVOE calls (:915, :917-918)
  double b1 = NAN, b2 = NAN;
  M2 Q = {NAN, NAN, NAN, NAN}, QR = {NAN, NAN, NAN, NAN};
  bool ok = pm.ok;
  ok = ok && compute_mvoe(scale(pm.cov_infer, chi_r), scale(pm.cov_mu, chi_p), tol, maxiter, b1,
                          Q);
  store_pair(&out->q01, Q.b, Q.d);
  ok = ok && compute_mvoe(Q, M2{R * R, 0.0, 0.0, R * R}, tol, maxiter, b2, QR);
  if (!ok) status = CCMPC_REC_SINGULAR;
  store_pair(&out->r00, QR.a, QR.b);
  store_pair(&out->r11, QR.d, b1);
  out->beta2 = b2;
  // slope-m tangent of the QR ellipse closest to the reference point (:920-924)
  double d = NAN;
  int which = 0, side = 0;
  if (!isfinite(m)) {
    if (status == 0) status = CCMPC_REC_NONFINITE;
  } else {
    const int ts = closest_tangent(QR, 1.0, n0, n1, proj, nrm, na, d, which);
    if (ts != 0) {
      if (status == 0) status = ts;
    } else if (isfinite(d)) {
      side = (n0 * m0 + n1 * m1 <= d) ? 1 : -1;  // (:926) n.mean <= d  ->  n.x >= d
    }
  }
  if (status == 0 && !(isfinite(d) && isfinite(Q.a) && isfinite(QR.a) && isfinite(m0)))
    status = CCMPC_REC_NONFINITE;
  store_pair(&out->d, d, Q.a);
  *reinterpret_cast<int4 *>(&out->which) = make_int4(which, side, status, (t << 16) | tau);
}

// All pairs of one cell by the threads [0, nthreads) of the calling group, with the cell's
// reference trajectory `ref` ([T][2]) and risk constants already at hand; lb_s has room for
// T(T-1)/2 doubles.  The record of a pair is a serial chain (two MVOE fixed points, then the
// tangent) on one lane; its lower bound does not depend on that chain, so with >= 2 waves the
// lower bounds run on the upper half of the group -- other waves, i.e. truly concurrently --
// and write their record field themselves.  Up to 128 pairs that lower-bound wave also takes
// the per-t minimum (no workgroup barrier: callers must not rely on one after this call); past
// that, the barrier needed before the per-t minimum is included.
__device__ void minkowski_cell(const double *C, const double *mu, int T, int cell,
                               const double *ref, double chi_r, double chi_p, double gamma,
                               const MinkParams &mp, double *lb_s, int tid, int nthreads) {
  const int rows = 2 * T;
  const int P = T * (T - 1) / 2;
  ccmpc_halfspace *rec = mp.out_rec + static_cast<int64_t>(cell) * P;
  // lower bounds on the other half of the group (other waves: truly concurrent with the MVOE
  // chains) while the records fit half the threads; beyond that every thread takes whole pairs
  // (a record's chain is the tail's critical path, so fewer rounds of chains win: T = 40's 780
  // pairs on 512 threads take 2 rounds instead of 4)
  const int half = (nthreads >= 128 && P <= nthreads / 2) ? nthreads / 2 : 0;
  if (half && P <= 2 * 64) {
    // One lower-bound wave (threads [half, half + 64), up to two pairs per lane) also takes the
    // per-t minimum from its own LDS writes, so nobody waits on a workgroup barrier: the record
    // waves end with their chains (the barrier and the minimum after it used to follow the
    // longest chain).  fmin ignores NaN as the reference's min(prob_lower, x) does, in any order.
    if (tid < half) {
      if (tid < P) {
        int t, tau;
        pair_of(tid, t, tau);
        minkowski_pair(C, mu, ref, rows, t, tau, chi_r, chi_p, mp.R, mp.tol, mp.maxiter, rec + tid);
      }
      return;
    }
    const int lane = tid - half;
    if (lane >= 64) return;
    for (int p = lane; p < P; p += 64) {
      int t, tau;
      pair_of(p, t, tau);
      const double lb = pair_lower_bound(pair_moments(C, rows, t, tau), gamma);
      lb_s[p] = lb;
      rec[p].lower_bound = lb;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS writes, in order
    if (lane < T) {
      double v = 1.0;
      for (int tau = 0; tau < lane; ++tau) v = fmin(v, lb_s[lane * (lane - 1) / 2 + tau]);
      mp.out_prob_lower[static_cast<int64_t>(cell) * T + lane] = v;
    }
    return;
  }
  const bool lb_side = half && tid >= half;
  const int base = lb_side ? tid - half : tid, stride = half ? half : nthreads;
  for (int p = base; p < P; p += stride) {
    int t, tau;
    pair_of(p, t, tau);
    if (lb_side || !half) {
      const double lb = pair_lower_bound(pair_moments(C, rows, t, tau), gamma);
      lb_s[p] = lb;
      rec[p].lower_bound = lb;
    }
    if (!lb_side)
      minkowski_pair(C, mu, ref, rows, t, tau, chi_r, chi_p, mp.R, mp.tol, mp.maxiter, rec + p);
  }
  __syncthreads();
  for (int t = tid; t < T; t += nthreads) {
    double v = 1.0;
    for (int tau = 0; tau < t; ++tau) v = fmin(v, lb_s[t * (t - 1) / 2 + tau]);
    mp.out_prob_lower[static_cast<int64_t>(cell) * T + t] = v;
  }
}

// Same, reading the reference trajectory and risk constants from global memory.
__device__ void minkowski_cell(const double *C, const double *mu, int T, int cell,
                               const MinkParams &mp, double *lb_s, int tid, int nthreads) {
  const int rsel = mp.cell_ref ? mp.cell_ref[cell] : 0;
  const double *ref = mp.ref_traj + static_cast<int64_t>(rsel) * (2 * T);
  minkowski_cell(C, mu, T, cell, ref, mp.cell_risk[3 * cell + 0], mp.cell_risk[3 * cell + 1],
                 mp.cell_risk[3 * cell + 2], mp, lb_s, tid, nthreads);
}

// The unfused half-space launch (constraints.hip): one wave per (cell, t), lanes = the row's pairs.
void launch_minkowski_rows(const double *mean, const double *cov, int T, int n_cells,
                           const MinkParams &mp, hipStream_t s);

}  // namespace ccmpc
