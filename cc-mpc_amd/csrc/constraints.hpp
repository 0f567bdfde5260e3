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

// Inverse by LU with partial pivoting, as LAPACK getrf/getri does it for 2x2.
__device__ __forceinline__ bool inv2(const M2 &m, M2 &out) {
  if (fabs(m.c) > fabs(m.a)) {
    // pivot rows: P m = [[c, d], [a, b]]
    const double l = m.a / m.c;
    const double u22 = m.b - l * m.d;
    if (m.c == 0.0 || u22 == 0.0) return false;
    // inverse of P m, then columns swapped back
    const double i11 = 1.0 / m.c, i22 = 1.0 / u22;
    const double i12 = -m.d * i11 * i22;
    // inv(U) = [[i11, i12], [0, i22]]; inv(L) = [[1, 0], [-l, 1]]; inv(Pm) = inv(U) inv(L)
    const double x11 = i11 - i12 * l, x12 = i12, x21 = -i22 * l, x22 = i22;
    out = {x12, x11, x22, x21};  // inv(m) = inv(Pm) P
    return true;
  }
  if (m.a == 0.0) return false;
  const double l = m.c / m.a;
  const double u22 = m.d - l * m.b;
  if (u22 == 0.0) return false;
  const double i11 = 1.0 / m.a, i22 = 1.0 / u22;
  const double i12 = -m.b * i11 * i22;
  out = {i11 - i12 * l, i12, -i22 * l, i22};
  return true;
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
  double l1, l2;
  if (disc >= 0.0) {
    const double s = sqrt(disc);
    l1 = half_tr + s;
    l2 = half_tr - s;
  } else {  // complex pair: .real keeps the real part of both
    l1 = half_tr;
    l2 = half_tr;
  }
  // beta' = sqrt(sum 1/w / sum l/w), w = 1 + beta l  ==  sqrt((w1 + w2) / (l1 w2 + l2 w1)):
  // the same fixed point with one division per iteration instead of five (the iteration is a
  // serial chain per record, so the division latency is the tail's critical path).  Rounding
  // differs from the reference's order by ~1 ulp per step; the contraction damps it.
  double b = 1.0;
  for (int it = 0; it < maxiter; ++it) {
    const double w1 = 1.0 + b * l1, w2 = 1.0 + b * l2;
    const double bn = sqrt((w1 + w2) / (l1 * w2 + l2 * w1));
    const bool done = fabs(bn - b) < tol;
    b = bn;
    if (done) break;
  }
  beta = b;
  Q = add(scale(S1, 1.0 + 1.0 / b), scale(S2, 1.0 + b));
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
  int tt = static_cast<int>((1.0 + sqrt(1.0 + 8.0 * p)) * 0.5);
  while (tt * (tt - 1) / 2 > p) --tt;
  while ((tt + 1) * tt / 2 <= p) ++tt;
  t = tt;
  tau = p - tt * (tt - 1) / 2;
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

// One (cell, t, tau) record from the cell's 2T x 2T covariance C (row stride `rows`) and mean mu
// (v8ideal/__init__.py:893-943).  Returns the lower bound (for the per-t minimum).
__device__ double minkowski_pair(const double *C, const double *mu, const double *ref, int rows,
                                 int t, int tau, double chi_r, double chi_p, double gamma,
                                 double R, double tol, int maxiter, ccmpc_halfspace &h) {
  h.status = 0;
  h.t_tau = (t << 16) | tau;
  // predict_moments (makeconstraint.py:41-70): blocks of the 2T x 2T covariance
  const M2 c_t = block(C, rows, t, t);
  const M2 c_x = block(C, rows, t, tau);
  const M2 c_xT = block(C, rows, tau, t);
  const M2 c_tau = block(C, rows, tau, tau);
  M2 inv_tau;
  bool ok = inv2(c_tau, inv_tau);
  const M2 cov_mu = mul(mul(c_x, inv_tau), c_xT);
  const M2 cov_infer = sub(c_t, cov_mu);
  // compute_lower_bound (makeconstraint.py:282-303): independent of the MVOE chain, so it is
  // issued first and its sqrt/div latency overlaps the setup of the first MVOE
  const double root_t = sqrt(fro(c_t));
  const double al = sqrt(fro(cov_infer)) / root_t;
  const double be = sqrt(fro(cov_mu)) / root_t;
  const double x = gamma * (1.0 - al) / be;
  const double lb = -expm1(-0.5 * (x * x));
  // two MVOE calls (:915, :917-918)
  double b1 = NAN, b2 = NAN;
  M2 Q = {NAN, NAN, NAN, NAN}, QR = {NAN, NAN, NAN, NAN};
  ok = ok && compute_mvoe(scale(cov_infer, chi_r), scale(cov_mu, chi_p), tol, maxiter, b1, Q);
  ok = ok && compute_mvoe(Q, M2{R * R, 0.0, 0.0, R * R}, tol, maxiter, b2, QR);
  if (!ok) h.status = CCMPC_REC_SINGULAR;
  // slope-m tangent of the QR ellipse closest to the reference point (:920-924)
  const double m0 = mu[2 * t], m1 = mu[2 * t + 1];
  const double a0 = ref[2 * t], a1 = ref[2 * t + 1];
  const double m = -(a0 - m0) / (a1 - m1);
  const double n0 = -m, n1 = 1.0;
  const double sn0 = QR.a * n0 + QR.b * n1, sn1 = QR.c * n0 + QR.d * n1;
  const double q = n0 * sn0 + n1 * sn1;
  double d = NAN;
  int which = 0, side = 0;
  if (!isfinite(m)) {
    if (h.status == 0) h.status = CCMPC_REC_NONFINITE;
  } else if (!(q > 0.0)) {
    if (h.status == 0) h.status = CCMPC_REC_NO_TANGENT;
  } else {
    const double proj = n0 * m0 + n1 * m1;
    const double delta = 1.0 * sqrt(q);
    const double d1 = proj + delta, d2 = proj - delta;
    const double nrm = sqrt(n0 * n0 + n1 * n1);
    const double na = n0 * a0 + n1 * a1;
    const double dist0 = fabs(na - d1) / nrm, dist1 = fabs(na - d2) / nrm;
    which = (dist1 < dist0) ? 1 : 0;
    d = which ? d2 : d1;
    side = (n0 * m0 + n1 * m1 <= d) ? 1 : -1;  // (:926) n.mean <= d  ->  n.x >= d
  }
  if (h.status == 0 && !(isfinite(d) && isfinite(Q.a) && isfinite(QR.a) && isfinite(m0)))
    h.status = CCMPC_REC_NONFINITE;
  h.n0 = n0;
  h.n1 = n1;
  h.d = d;
  h.q00 = Q.a;
  h.q01 = Q.b;
  h.q11 = Q.d;
  h.r00 = QR.a;
  h.r01 = QR.b;
  h.r11 = QR.d;
  h.beta1 = b1;
  h.beta2 = b2;
  h.lower_bound = lb;
  h.mean0 = m0;
  h.mean1 = m1;
  h.which = which;
  h.side = side;
  return lb;
}

// All pairs of one cell by the threads [0, nthreads) of the calling group, with the cell's
// reference trajectory `ref` ([T][2]) and risk constants already at hand; lb_s has room for
// T(T-1)/2 doubles.  Includes the barrier needed before the per-t minimum.
__device__ void minkowski_cell(const double *C, const double *mu, int T, int cell,
                               const double *ref, double chi_r, double chi_p, double gamma,
                               const MinkParams &mp, double *lb_s, int tid, int nthreads) {
  const int rows = 2 * T;
  const int P = T * (T - 1) / 2;
  for (int p = tid; p < P; p += nthreads) {
    int t, tau;
    pair_of(p, t, tau);
    ccmpc_halfspace h;
    lb_s[p] = minkowski_pair(C, mu, ref, rows, t, tau, chi_r, chi_p, gamma, mp.R, mp.tol,
                             mp.maxiter, h);
    mp.out_rec[static_cast<int64_t>(cell) * P + p] = h;
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

}  // namespace ccmpc
