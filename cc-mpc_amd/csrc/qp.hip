// The planning step's quadratic program, batched over scenes: the caller side of the path
// (SURVEY.md 8f row 3).  Replaces do_highlevel_control's cvxpy + CPLEX problem
// (v8ideal/__init__.py:2850-2930, objective :2478-2507, speed limits :610-626) with the
// road-boundary MILP off (the reference default, :217), which leaves a convex QP in the 2T
// controls u.  The LTV model it needs comes from ccmpc_mpc_ltv (dynamics/bicycle_v2.py
// :240-308, linearised about u_init = 0 as make_local_params does, v8ideal :537-557).
//
// Design (gfx950): one workgroup of 4 waves per scene runs a primal-dual interior point method
// (Mehrotra predictor-corrector) entirely in LDS.  Every constraint acts on a handful of
// "output" rows of the state -- x_t, y_t (obstacle half-spaces, 2 nonzeros in output space)
// and v_t (speed limits) -- or on u itself (control bounds), so the normal matrix is
//   M = H_ctrl + diag(w_box) + Gs^T B Gs,
// Gs = the 3T selected rows of Gamma_f (x, y, v of each step), B = per-step 3x3 blocks holding
// the objective's position weights plus sum_r w_r a_r a_r^T of that step's half-spaces.  The
// records are read in place (the generators' [cell][pair] layout puts step t's half-spaces of
// a cell in one contiguous run), so an iteration costs O(records) + O(T n^2), not O(m n^2),
// and needs no sort.  Per-step sums are wave reductions in a fixed order: the solve is
// bitwise reproducible.  Cholesky and both triangular solves run on wave 0 (lane = row),
// wave-synchronous, with no workgroup barrier per column.
#include "ccmpc_common.hpp"
#include <cstdlib>
#include <cstring>

namespace ccmpc {

#ifdef CCMPC_QP_TRACE
#define QP_MARK(i) (tmark[i] = wall_clock64())
#define PQ_MARK(i) (pmark[i] = pmark[i] ? pmark[i] : wall_clock64())
#else
#define QP_MARK(i) ((void)0)
#define PQ_MARK(i) ((void)0)
#endif

constexpr int kQpThreads = 256;
constexpr int kQpWaves = kQpThreads / 64;
constexpr int kQpMaxT = 40;
constexpr size_t kQpLdsBytes = 160 * 1024;
constexpr int kQpRowDoubles = 10;  // doubles per constraint row in the row store (Rows)
// the IPM tries its one early polish once mu <= kEarlyPolish * max(mu0, 1) (the regular stop is
// at mu <= 1e-3 tol, ~1e-12).  Measured (profiles/r04/qp_early_polish_ab.log): 1e-3 is too
// early (the active set not settled: a failed attempt, 11 iterations, 232 us for the single
// T = 8 solve), 1e-4 133 us (5 iterations), 1e-5 / 1e-6 152 us (7); a C1 episode's 12 QPs
// 2.10 ms at 1e-4 against 2.21 at 1e-5
// (the env var CCMPC_QP_EARLY_POLISH overrides it per call: 0 = no early attempt; a negative
// value -x attempts at x but discards even a verified answer, the test hook that checks a failed
// attempt leaves the IPM bit-identical to a solve without one)
constexpr double kEarlyPolish = 1e-4;
// the default method: the active-set solve where it applies (one wave, n <= 16): a T = 8
// frame's QP 133.8 -> 47.8 us, the 64-scene batch 359 -> 281 us, the same minimiser and
// verdict on every tested scene (profiles/r05/ab_qp_method.log, tests/test_gpu_qp_gi.py)
constexpr int kQpDefaultMethod = CCMPC_QP_METHOD_GI;
// internal status bit: the active-set-only instance handed this scene to the IPM pass
constexpr int kQpNeedIpm = 1 << 20;
// the records' first loads: 1 = with the setup's first reads (before the model), 0 = in the rows
// phase, after the model's barrier (which otherwise waits for them: they sit behind the
// scene-cell load, two dependent round trips)
#ifndef CCMPC_QP_REC_PREFETCH
#define CCMPC_QP_REC_PREFETCH 1
#endif

// ---- the LTV model ---------------------------------------------------------------------------
// About u = 0 the bicycle model's nominal trajectory is straight at constant speed
// (bicycle_kinematics: psi' = v/L cos(beta) tan(u_2) = 0, v' = u_1 = 0, beta from the 'delta'
// parameter, 0), so X_bar[i] = x0 + i Ts v (cos psi, sin psi), and every step shares
// A = d f / d x with A^2 = 0.  Zero-order hold of [[A, B], [0, 0]] is then exact in closed form:
// Ad = I + Ts A, Bd = Ts B + Ts^2/2 A B (cont2discrete 'zoh' = expm of that block matrix).
// Gamma = A_bar^{-1} B_bar (:296-306) is block lower triangular with block (t, k) =
// Ad^{t-k} Bd = (I + (t-k) Ts A) Bd.
// The model of one scene, evaluated entry by entry: mpc_ltv_kernel writes every entry, and the
// QP with a fused LTV rebuild (ccmpc_mpc_qp_ltv) evaluates the ones it reads from the same
// functions (defined here, outside the QP kernel's fp-contract scope, so both round alike).
struct LtvModel {
  double x0, y0, psi, v, cp, sp, Ts;
  double a02, a03, a12, a13;
  double Bd[4][2];
  __device__ LtvModel(const double *x_init, double Ts_, double l_r, double L) {
    x0 = x_init[0];
    y0 = x_init[1];
    psi = x_init[2];
    v = x_init[3];
    Ts = Ts_;
    cp = cos(psi);
    sp = sin(psi);
    // get_dbeta_ddelta at delta = 0 (:19-24): 1 when l_r == L, else 1 / (L / l_r)
    const double dbeta = (l_r == L) ? 1.0 : 1.0 / (L / l_r);
    // A (get_state_matrix :103-115 at delta = 0): nonzeros A[0][2], A[0][3], A[1][2], A[1][3]
    a02 = -v * sp;
    a03 = cp;
    a12 = v * cp;
    a13 = sp;
    // B (get_input_matrix :117-130 at delta = 0)
    const double b01 = -v * sp * dbeta, b11 = v * cp * dbeta, b21 = (v / L) * 1.0, b30 = 1.0;
    // Bd = Ts B + Ts^2/2 A B;  (A B)[r][c] = sum_k A[r][k] B[k][c]
    const double h = 0.5 * Ts * Ts;
    Bd[0][0] = h * (a03 * b30);
    Bd[0][1] = Ts * b01 + h * (a02 * b21);
    Bd[1][0] = h * (a13 * b30);
    Bd[1][1] = Ts * b11 + h * (a12 * b21);
    Bd[2][0] = 0.0;
    Bd[2][1] = Ts * b21;
    Bd[3][0] = Ts * b30;
    Bd[3][1] = 0.0;
  }
  // Gamma[r][c] (r = 4 t + i, c = 2 k + j): (I + (t - k) Ts A) Bd for k <= t, else 0
  __device__ double gamma(int r, int c) const {
    const int t = r >> 2, i = r & 3, k = c >> 1, j = c & 1;
    double g = 0.0;
    if (k <= t) {
      const double mt = static_cast<double>(t - k) * Ts;
      g = Bd[i][j];
      if (i == 0) g += mt * (a02 * Bd[2][j] + a03 * Bd[3][j]);
      if (i == 1) g += mt * (a12 * Bd[2][j] + a13 * Bd[3][j]);
    }
    return g;
  }
  // X_bar[1:][r]
  __device__ double xbar(int r) const {
    const int t = (r >> 2) + 1, i = r & 3;
    const double tt = static_cast<double>(t) * Ts;
    return i == 0 ? x0 + v * cp * tt : i == 1 ? y0 + v * sp * tt : i == 2 ? psi : v;
  }
};

__global__ void mpc_ltv_kernel(const double *__restrict__ x_init, int64_t S, int T, double Ts,
                               double l_r, double L, double *__restrict__ out_xbar,
                               double *__restrict__ out_gamma) {
  const int64_t s = blockIdx.x;
  if (s >= S) return;
  const LtvModel lm(x_init + 4 * s, Ts, l_r, L);
  const int rows = 4 * T, cols = 2 * T;
  for (int e = threadIdx.x; e < rows * cols; e += blockDim.x)
    out_gamma[s * rows * cols + e] = lm.gamma(e / cols, e % cols);
  for (int r = threadIdx.x; r < rows; r += blockDim.x) out_xbar[s * rows + r] = lm.xbar(r);
}

// ---- the QP ---------------------------------------------------------------------------------
struct QpArgs {
  int64_t S;
  int T, Tf, n_ref, u_order, rec_kind, max_iter, rows_in_lds, polish;
  int rec_compact;    // records are ccmpc_gather_rec (32 bytes), rec_kind their source kind
  int early_discard;  // test hook: attempt the early polish, never keep its answer
  int method;         // CCMPC_QP_METHOD_IPM, or _GI (one wave, n <= 32; else the IPM)
  int gi_max_steps;   // the active-set step budget (< 0: 8 (n + 16)); a test hook forces the
                      // hand-over to the IPM with 0
  int fallback_only;  // the IPM pass after an active-set-only launch (kQpNeedIpm scenes only)
  int gi_nostep;      // GI's "no step exists" verdict: 0 kept, 1 always confirmed by the IPM,
                      // 2 kept when it is certain (the default; see gi_solve)
  int64_t max_cells;
  double tol, early;  // early: the early polish threshold on mu / max(mu0, 1) (0 = none)
  const double *gamma, *xbar, *ubar, *u_prev, *goal, *ref;
  // fused LTV rebuild (ccmpc_mpc_qp_ltv): x_init[S][4] != NULL -> the model is computed here,
  // written to ltv_xbar / ltv_gamma (= xbar / gamma) and read from registers, not memory
  const double *ltv_x0;
  double ltv_Ts, ltv_lr, ltv_L;
  double *ltv_xbar, *ltv_gamma;
  const unsigned char *rec;
  const int64_t *scene_cell;
  ccmpc_mpc_params p;
  double *ws;  // per-scene row store when it does not fit LDS
  double *out_u, *out_x, *out_cost;
  int32_t *out_status, *out_iter;
};

// Sizes (doubles) of the LDS image; shared by host (launch sizing) and device (carving).
struct QpLayout {
  int n, T3, ldm;
  int gs, m, hc, c3, y, yd, qf, q, bw, f, z, dz, rd, rh, e2, lb, ub, dinv, red;
  int pw, ps, pact, pdinv;  // the polish step's W = L^{-1} G_A^T, S = W^T W, active rows
  int rows, total;
  __host__ __device__ QpLayout(int T, int64_t R, bool rows_lds, bool polish) {
    n = 2 * T;
    T3 = 3 * T;
    ldm = n + 1;  // odd row stride: column reads of the Cholesky spread over the banks
    int o = 0;
    gs = o; o += T3 * n;
    m = o; o += n * ldm;
    hc = o;  // H_ctrl (constant over the iterations): only the one-wave path (n <= 16)
    if (n <= 16) o += n * n;  // reads the table; the four-wave paths evaluate hctrl()
    c3 = o; o += T3;
    y = o; o += T3;
    z = o; o += n;   // right behind y: the rows index [y | z] as one vector
    yd = o; o += T3;
    dz = o; o += n;  // likewise behind yd
    qf = o; o += T3;
    q = o; o += T3;
    bw = o; o += 4 * T;
    f = o; o += n;
    rd = o; o += n;
    rh = o; o += n;
    e2 = o; o += n;
    lb = o; o += n;
    ub = o; o += n;
    dinv = o; o += n;
    red = o; o += 8 * kQpWaves;
    pw = ps = pact = pdinv = o;
    if (polish) {
      pw = o; o += n * n;
      ps = o; o += n * ldm;
      pact = o; o += n;
      pdinv = o; o += n;
    }
    rows = o;
    const int64_t mrows = 2 * n + 2 * T + R;
    if (rows_lds) o += static_cast<int>(kQpRowDoubles * mrows);
    total = o;
  }
};

__host__ __device__ inline int64_t qp_rows_per_cell(int T, int kind) {
  return kind == CCMPC_REC_KIND_HALFSPACE ? int64_t(T) * (T - 1) / 2 : T;
}

// row store over all m rows (box 2n, speed 2T, obstacle R): s, l, ds, dl, then every row in
// one form, g_r(v) = c0 v[i0] + c1 v[i1] + cst over v = [y (T3) | z (n)] (the layout keeps z
// right behind y, and dz behind yd), so evaluating a row is two loads and two FMAs with no
// branch on the row's kind.  Box row 2j (+1): c0 = +1 (-1) on z_j, cst = -ub_j (lb_j); speed
// row 2t (+1): +1 (-1) on v_t, cst = c_v - max_v (-c_v); obstacle row: c = a, i = (3t, 3t+1),
// cst = -b' (b' = b - a . c_xy, the constant part of the state moved to the right).
struct Rows {
  double *s, *l, *ds, *dl, *c0, *c1, *cst;
  int32_t *ix;      // (i0, i1) per row
  double *rp, *is;  // this iteration's primal residual g + s and 1 / s (set in I1)
};

// Lane moves inside a row of 16 (DPP; f64 as two 32-bit halves).  `old` is what a lane keeps
// if its source is out of range -- never the case for the controls used here, with the whole
// wave active (every caller reduces in wave-uniform control flow).
template <int CTRL>
__device__ __forceinline__ double qp_dpp(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo =
      __builtin_amdgcn_update_dpp(0u, static_cast<uint32_t>(u), CTRL, 0xf, 0xf, false);
  const uint32_t hi =
      __builtin_amdgcn_update_dpp(0u, static_cast<uint32_t>(u >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, (static_cast<uint64_t>(hi) << 32) | lo);
}
constexpr int kDppQuad1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppQuad2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141;  // lane i of 8 <- lane 7-i: the other quad
constexpr int kDppMirror = 0x140;      // lane i of 16 <- lane 15-i: the other half-row

__device__ __forceinline__ double lane_bcast(double v, int src) {  // src wave-uniform
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(u), src);
  const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(u >> 32), src);
  return __builtin_bit_cast(double, (static_cast<uint64_t>(hi) << 32) | lo);
}

// Sum over each group of 4 / 8 consecutive lanes (every lane of the group gets it)
__device__ __forceinline__ double sum4(double v) {
  v += qp_dpp<kDppQuad1>(v);
  return v + qp_dpp<kDppQuad2>(v);
}
__device__ __forceinline__ double sum8(double v) {
  v = sum4(v);
  return v + qp_dpp<kDppHalfMirror>(v);
}

// Whole-wave reductions: four DPP steps reduce each row of 16, then the four row results are
// combined in a fixed order from lanes 0, 16, 32, 48 (uniform result, no LDS round trips)
__device__ __forceinline__ double wave_sum(double v) {
  v = sum8(v);
  v += qp_dpp<kDppMirror>(v);
  return (lane_bcast(v, 0) + lane_bcast(v, 16)) + (lane_bcast(v, 32) + lane_bcast(v, 48));
}
__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, qp_dpp<kDppQuad1>(v));
  v = fmax(v, qp_dpp<kDppQuad2>(v));
  v = fmax(v, qp_dpp<kDppHalfMirror>(v));
  v = fmax(v, qp_dpp<kDppMirror>(v));
  return fmax(fmax(lane_bcast(v, 0), lane_bcast(v, 16)), fmax(lane_bcast(v, 32), lane_bcast(v, 48)));
}
__device__ __forceinline__ double wave_min(double v) {
  v = fmin(v, qp_dpp<kDppQuad1>(v));
  v = fmin(v, qp_dpp<kDppQuad2>(v));
  v = fmin(v, qp_dpp<kDppHalfMirror>(v));
  v = fmin(v, qp_dpp<kDppMirror>(v));
  return fmin(fmin(lane_bcast(v, 0), lane_bcast(v, 16)), fmin(lane_bcast(v, 32), lane_bcast(v, 48)));
}

// Block reductions of up to 2 values (every thread gets the result); two barriers.  NW = 1
// (one wave per scene): the wave reduction alone, no LDS and no barrier.
template <int NW>
__device__ __forceinline__ void block_max2(double &a, double &b, double *red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  a = wave_max(a);
  b = wave_max(b);
  if (NW == 1) return;
  if (lane == 0) {
    red[2 * w] = a;
    red[2 * w + 1] = b;
  }
  __syncthreads();
  a = red[0];
  b = red[1];
  for (int k = 1; k < NW; ++k) {
    a = fmax(a, red[2 * k]);
    b = fmax(b, red[2 * k + 1]);
  }
  __syncthreads();
}
template <int NW>
__device__ __forceinline__ double block_sum(double a, double *red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  a = wave_sum(a);
  if (NW == 1) return a;
  if (lane == 0) red[w] = a;
  __syncthreads();
  a = red[0];
  for (int k = 1; k < NW; ++k) a += red[k];
  __syncthreads();
  return a;
}
template <int NW>
__device__ __forceinline__ double block_min(double a, double *red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  a = wave_min(a);
  if (NW == 1) return a;
  if (lane == 0) red[w] = a;
  __syncthreads();
  a = red[0];
  for (int k = 1; k < NW; ++k) a = fmin(a, red[k]);
  __syncthreads();
  return a;
}

// Block argmax (largest value, smallest index on ties); every thread gets the result.
template <int NW>
__device__ __forceinline__ void block_argmax(double &v, double &idx, double *red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(v, o, 64), oi = __shfl_xor(idx, o, 64);
    if (ov > v || (ov == v && oi < idx)) {
      v = ov;
      idx = oi;
    }
  }
  if (NW == 1) return;
  if (lane == 0) {
    red[2 * w] = v;
    red[2 * w + 1] = idx;
  }
  __syncthreads();
  v = red[0];
  idx = red[1];
  for (int k = 1; k < NW; ++k) {
    if (red[2 * k] > v || (red[2 * k] == v && red[2 * k + 1] < idx)) {
      v = red[2 * k];
      idx = red[2 * k + 1];
    }
  }
  __syncthreads();
}


// wave-level ordering of LDS traffic between the lanes of wave 0 (one wave executes its LDS
// instructions in order; this keeps the compiler from moving them across the step)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The workgroup's barrier; with one wave per scene, the wave-level ordering above (a wave runs
// its LDS instructions in order, so every lane then sees every other lane's writes)
template <int NW>
__device__ __forceinline__ void qp_sync() {
  if (NW == 1)
    wave_sync();
  else
    __syncthreads();
}

// Wave-level dense Cholesky and triangular solves (called by one whole wave; lane = row, two
// rows per lane, so N <= 128).  A holds the lower triangle, row stride ld; it is overwritten by
// L, and dinv[j] = 1 / L[j][j].  With pivot_skip a pivot that cancellation drove to <= 0 is
// replaced by a huge one (see the IPM below); otherwise it fails.  Returns true on failure.
__device__ bool wave_cholesky(double *A, int N, int ld, double *dinv, bool pivot_skip) {
  const int lane = threadIdx.x & 63;
  bool fail = false;
  for (int j = 0; j < N; ++j) {
    double sv[2];
    const double ajj = A[j * ld + j];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = j + lane + 64 * h;
      double v = 0.0;
      if (i < N) {
        v = A[i * ld + j];
        for (int k = 0; k < j; ++k) v -= A[i * ld + k] * A[j * ld + k];
      }
      sv[h] = v;
    }
    double dj = lane_bcast(sv[0], 0);
    fail = fail || !isfinite(dj) || !isfinite(ajj);
    if (!(dj > 1e-30 * ajj)) {
      fail = fail || !pivot_skip;
      dj = 1e128;
    }
    const double ljj = sqrt(dj), inv = 1.0 / ljj;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = j + lane + 64 * h;
      if (i < N) A[i * ld + j] = (i == j) ? ljj : sv[h] * inv;
    }
    if (lane == 0) dinv[j] = inv;
    wave_sync();
  }
  return fail;
}

// b <- L^{-1} b (b[h] is row lane + 64 h)
__device__ __forceinline__ void wave_forward(const double *L, int N, int ld, const double *dinv,
                                             double b[2]) {
  const int lane = threadIdx.x & 63;
  for (int j = 0; j < N; ++j) {
    const double yj = lane_bcast((j >> 6) ? b[1] : b[0], j & 63) * dinv[j];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = lane + 64 * h;
      if (i == j) b[h] = yj;
      else if (i > j && i < N) b[h] -= L[i * ld + j] * yj;
    }
  }
}

// b <- L^{-T} b
__device__ __forceinline__ void wave_backward(const double *L, int N, int ld, const double *dinv,
                                              double b[2]) {
  const int lane = threadIdx.x & 63;
  for (int j = N - 1; j >= 0; --j) {
    const double xj = lane_bcast((j >> 6) ? b[1] : b[0], j & 63) * dinv[j];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = lane + 64 * h;
      if (i == j) b[h] = xj;
      else if (i < j) b[h] -= L[j * ld + i] * xj;
    }
  }
}

__device__ __forceinline__ void wave_load2(const double *x, int N, double b[2]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int h = 0; h < 2; ++h) b[h] = (lane + 64 * h < N) ? x[lane + 64 * h] : 0.0;
}
__device__ __forceinline__ void wave_store2(double *x, int N, const double b[2]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int h = 0; h < 2; ++h)
    if (lane + 64 * h < N) x[lane + 64 * h] = b[h];
}

// Register-resident variants for n <= NM (one row per lane of the calling wave): the
// IPM factors and solves twice per iteration, and with L in registers a column step is a
// readlane and an FMA instead of a dependent LDS round trip.  a[k] = L[lane][k] (row form),
// dl = 1 / L[lane][lane]; the L^T solve reads L's rows from LDS (independent of the chain, so
// the unrolled loads issue ahead of it).  The matrix is padded to NM x NM with the identity
// (rows and columns >= n; the right-hand side 0 there), so every step runs unconditionally:
// straight-line code, no per-column branch on a runtime n.
template <int NM, bool SKIP = true>
__device__ __forceinline__ bool reg_cholesky(double (&a)[NM], double &dl) {
  const int lane = threadIdx.x & 63;
  bool fail = false;
  double diag0 = 0.0;  // the lane's original diagonal (for the pivot-skip threshold)
#pragma unroll
  for (int k = 0; k < NM; ++k)
    if (k == lane) diag0 = a[k];
  fail = __ballot(lane < NM && !isfinite(diag0)) != 0;
#pragma unroll
  for (int j = 0; j < NM; ++j) {
    {
      double d = lane_bcast(a[j], j);
      // lane j's pivot against its own original diagonal, as a ballot bit (no broadcast)
      const bool tiny = (__ballot(!(a[j] > 1e-30 * diag0)) >> j) & 1;
      fail = fail || !isfinite(d);
      if (tiny) {  // pivot skip (the IPM), or a failure (SKIP = false)
        fail = fail || !SKIP;
        d = 1e128;
      }
      // sqrt and 1/sqrt from the hardware rsqrt + one Goldschmidt step (~1 ulp; the IPM's
      // factor needs no IEEE rounding, the polish recomputes the answer from H exactly)
      const double y = __builtin_amdgcn_rsq(d);
      double g = d * y, h = 0.5 * y;
      const double rr = fma(-g, h, 0.5);
      g = fma(g, rr, g);
      h = fma(h, rr, h);
      const double ljj = g, inv = 2.0 * h;
      const double lij = lane > j ? a[j] * inv : (lane == j ? ljj : 0.0);
      a[j] = lij;
      if (lane == j) dl = inv;
      // trailing update without an exec-mask branch: rows above k pick up values in their
      // (never read) upper triangle; lij = 0 for rows < j keeps their finished rows intact
#pragma unroll
      for (int k = j + 1; k < NM; ++k) a[k] = fma(-lij, lane_bcast(lij, k), a[k]);
    }
  }
  return fail;
}

// lt[j] = L[j][lane], the L^T solve's column (from L's lower triangle in LDS, row stride ld)
template <int NM>
__device__ __forceinline__ void reg_load_lt(const double *L, int ld, int n, double (&lt)[NM]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < NM; ++j) {  // every lane loads (in-bounds index), then selects
    const double v = L[(j < n ? j : 0) * ld + (lane < j ? lane : 0)];
    lt[j] = (lane < j && j < n) ? v : 0.0;
  }
}
template <int NM>  // b <- L^{-1} b (b on lane = row)
__device__ __forceinline__ double reg_forward(const double (&a)[NM], double dl, double b) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < NM; ++j) {
    const double yj = lane_bcast(b * dl, j);  // lane j's b is final: one broadcast
    const double upd = fma(-a[j], yj, b);
    b = lane == j ? yj : (lane > j ? upd : b);
  }
  return b;
}
template <int NM>  // b <- L^{-T} b
__device__ __forceinline__ double reg_backward(const double (&lt)[NM], double dl, double b) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = NM - 1; j >= 0; --j) {
    const double xj = lane_bcast(b * dl, j);
    const double upd = fma(-lt[j], xj, b);
    b = lane == j ? xj : (lane < j ? upd : b);
  }
  return b;
}
template <int NM>
__device__ __forceinline__ double reg_solve(const double (&a)[NM], const double *L, int ld,
                                            double dl, int n, double b) {
  double lt[NM];  // read ahead of the chain
  reg_load_lt(L, ld, n, lt);
  return reg_backward(lt, dl, reg_forward(a, dl, b));
}

// control index of U_t component c: cp.reshape(u, (T, 2)) is column-major by default
__device__ __forceinline__ int u_index(int t, int c, int T, int order) {
  return order == CCMPC_U_ORDER_C ? 2 * t + c : t + c * T;
}
__device__ __forceinline__ void u_decode(int i, int T, int order, int &t, int &c) {
  if (order == CCMPC_U_ORDER_C) {
    t = i >> 1;
    c = i & 1;
  } else {
    c = i >= T;
    t = i - c * T;
  }
}

// H_ctrl[i][j] = 2 (R1 + [t >= 1] R2 + [t <= T-2] R2)[a][b] on the diagonal step block,
// -2 R2[a][b] on the two neighbouring step blocks (:2504-2506), 0 elsewhere
__device__ __forceinline__ double hctrl(int i, int j, int T, int order, const ccmpc_mpc_params &p) {
  int ti, ci, tj, cj;
  u_decode(i, T, order, ti, ci);
  u_decode(j, T, order, tj, cj);
  const double r1 = ci == cj ? (ci == 0 ? p.w_accel : p.w_turning) : p.w_joint;
  const double r2 = ci == cj ? (ci == 0 ? p.w_ch_accel : p.w_ch_turning) : p.w_ch_joint;
  if (ti == tj) {
    double k = r1;
    if (ti >= 1) k += r2;
    if (ti <= T - 2) k += r2;
    return 2.0 * k;
  }
  if (ti - tj == 1 || tj - ti == 1) return -2.0 * r2;
  return 0.0;
}

__device__ __forceinline__ double hctrl_mul(const double *z, int i, int T, int order,
                                            const ccmpc_mpc_params &p) {
  int ti, ci;
  u_decode(i, T, order, ti, ci);
  double acc = 0.0;
  for (int tj = ti - 1; tj <= ti + 1; ++tj) {
    if (tj < 0 || tj >= T) continue;
    for (int cj = 0; cj < 2; ++cj) {
      const int j = u_index(tj, cj, T, order);
      acc += hctrl(i, j, T, order, p) * z[j];
    }
  }
  return acc;
}

// NW waves per scene: 4 (the general form), or 1 for n = 2T <= 16 (the reference's ph = 8):
// every barrier is then a wave-level ordering and every reduction a wave butterfly, which
// takes the ~30 workgroup barriers per IPM iteration off the chain.
template <bool ROWS_LDS, int NM, int NW, bool GI = false, bool GIONLY = false>
__global__ __launch_bounds__(64 * NW) void mpc_qp_kernel(QpArgs A) {
  // multiply-adds fused in the solver (the library builds with -ffp-contract=off for the
  // moments' reference arithmetic; the IPM's iterates carry no such contract, and its answer
  // is the verified polish / KKT point, tested against the oracle QP to a tolerance)
#pragma clang fp contract(fast)
  constexpr int NTH = 64 * NW;
  extern __shared__ double lds[];
  const int64_t sc = blockIdx.x;
  if (sc >= A.S) return;
  // the IPM pass after a GIONLY launch solves only the scenes the active-set pass handed over
  if (A.fallback_only && !(A.out_status[sc] & kQpNeedIpm)) return;
#ifdef CCMPC_QP_TRACE
  const uint64_t tk0 = wall_clock64();
  uint64_t smark[4] = {};
#define QS_MARK(i) (smark[i] = wall_clock64())
#else
#define QS_MARK(i) ((void)0)
#endif
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int T = A.T, Tf = A.Tf, Tp = Tf - T;
  const int64_t c0 = A.scene_cell[sc], ncell = A.scene_cell[sc + 1] - c0;
  const int P = static_cast<int>(qp_rows_per_cell(T, A.rec_kind));
  const int64_t R = ncell * P;
  const QpLayout lay(T, ROWS_LDS ? R : 0, ROWS_LDS, A.polish != 0);
  const int n = lay.n, T3 = lay.T3, ldm = lay.ldm;
  const int nbox = 2 * n, nv = 2 * T;
  const int64_t mrows = nbox + nv + R;
  double *Gs = lds + lay.gs, *M = lds + lay.m, *Hc = lds + lay.hc, *c3 = lds + lay.c3,
         *y = lds + lay.y,
         *yd = lds + lay.yd, *qf = lds + lay.qf, *q = lds + lay.q, *bw = lds + lay.bw,
         *z = lds + lay.z, *dz = lds + lay.dz, *rd = lds + lay.rd, *rh = lds + lay.rh,
         *e2 = lds + lay.e2, *lb = lds + lay.lb,
         *ub = lds + lay.ub, *dinv = lds + lay.dinv, *red = lds + lay.red;
  double *rbase;
  if (ROWS_LDS) {
    rbase = lds + lay.rows;
  } else {
    const int64_t mcap = 2 * n + 2 * T + A.max_cells * P;
    rbase = A.ws + sc * kQpRowDoubles * mcap;
  }
  const Rows rw{rbase,
                rbase + mrows,
                rbase + 2 * mrows,
                rbase + 3 * mrows,
                rbase + 4 * mrows,
                rbase + 5 * mrows,
                rbase + 6 * mrows,
                reinterpret_cast<int32_t *>(rbase + 7 * mrows),
                rbase + 8 * mrows,
                rbase + 9 * mrows};
  // the obstacle rows' a0, a1 (indexed by obstacle row o = r - nbox - nv)
  const double *oa0 = rw.c0 + nbox + nv, *oa1 = rw.c1 + nbox + nv;
  // step t of obstacle row o (records of a cell in (t, tau) order, or one per t for affine)
  auto obst_step = [&](int64_t o) -> int {
    const int64_t cell = o / P;
    const int pp = static_cast<int>(o - cell * P);
    if (A.rec_kind != CCMPC_REC_KIND_HALFSPACE) return pp;
    int t = static_cast<int>((1.0f + sqrtf(1.0f + 8.0f * static_cast<float>(pp))) * 0.5f);
    while (t * (t - 1) / 2 > pp) --t;
    while ((t + 1) * t / 2 <= pp) ++t;
    return t;
  };
  const ccmpc_mpc_params &p = A.p;
  const int order = A.u_order;
  const int ncol = 2 * Tf;
  const double *Gam = A.gamma + sc * (4 * Tf) * ncol;
  const double *xb = A.xbar + sc * 4 * Tf;
  const double *ubar = A.ubar ? A.ubar + sc * ncol : nullptr;
  const double *uprev = (A.u_prev && Tp > 0) ? A.u_prev + sc * 2 * Tp : nullptr;
  const double g0 = A.goal[2 * sc], g1 = A.goal[2 * sc + 1];
  const double *ref = A.ref + sc * 2 * A.n_ref;
  // output row k = 3t + a of the selected state rows: x, y, v of step t (state index 0, 1, 3)
  auto grow = [&](int k) { return 4 * (Tp + k / 3) + (k % 3 == 2 ? 3 : k % 3); };

  // ---- setup -------------------------------------------------------------------------------
  // The records (fresh from the cycle kernel, so cold) and the reference points are loaded
  // first, with the model's own reads below, so the setup waits for one round trip of global
  // loads instead of one per phase: the first kRecPre records of every thread in registers
  // (n0 n1 as one 16-byte load, then d and side / status / t_tau)
  constexpr int kRecPre = 4;
  struct RecIn {
    double2 nn;
    int4 a, b;  // full records: d at a.xy (offset 16 or 32), b = bytes 112..127; compact: a
  };
  auto load_rec = [&](int64_t r) -> RecIn {
    const unsigned char *rec = A.rec + (c0 * P + r) * (A.rec_compact ? 32 : 128);
    RecIn v;
    v.nn = *reinterpret_cast<const double2 *>(rec);
    if (A.rec_compact) {
      v.a = *reinterpret_cast<const int4 *>(rec + 16);
      v.b = v.a;
    } else {
      v.a = *reinterpret_cast<const int4 *>(
          rec + (A.rec_kind == CCMPC_REC_KIND_HALFSPACE ? 16 : 32));
      v.b = *reinterpret_cast<const int4 *>(rec + 112);
    }
    return v;
  };
  RecIn rpre[kRecPre];
#if CCMPC_QP_REC_PREFETCH
#pragma unroll
  for (int j = 0; j < kRecPre; ++j) {
    const int64_t r = tid + static_cast<int64_t>(j) * NTH;
    if (r < R) rpre[j] = load_rec(r);
  }
#endif
  double ref_k = 0.0;  // the reference point entry of qf's first row k = tid
  if (tid < T3 && tid % 3 < 2) {
    const int t = tid / 3, tr = t < A.n_ref ? t : A.n_ref - 1;
    ref_k = ref[2 * tr + tid % 3];
  }
  // Gamma's rows in batches of kGsPre loads per thread, every load of a batch issued before
  // its LDS stores (a store between two loads made each load a round trip of its own: ~6 us
  // of the one-wave setup at T = 8, where one batch covers all 384 entries)
  constexpr int kGsPre = 6;
  if (A.ltv_x0) {
    // the fused LTV rebuild: this scene's model into the caller's buffers (later frames read
    // them), Gs and the constant part straight from the model
    const LtvModel lm(A.ltv_x0 + 4 * sc, A.ltv_Ts, A.ltv_lr, A.ltv_L);
    const int gr4 = 4 * Tf;
    double *og = A.ltv_gamma + sc * gr4 * ncol, *ox = A.ltv_xbar + sc * gr4;
    for (int e = tid; e < gr4 * ncol; e += NTH) og[e] = lm.gamma(e / ncol, e % ncol);
    for (int r = tid; r < gr4; r += NTH) ox[r] = lm.xbar(r);
    for (int e = tid; e < T3 * n; e += NTH) Gs[e] = lm.gamma(grow(e / n), 2 * Tp + e % n);
    for (int k = tid; k < T3; k += NTH) {
      const int r = grow(k);
      double c = lm.xbar(r);
      if (uprev)
        for (int j = 0; j < 2 * Tp; ++j) c += lm.gamma(r, j) * uprev[j];
      if (ubar)
        for (int j = 0; j < n; ++j) c -= lm.gamma(r, 2 * Tp + j) * ubar[2 * Tp + j];
      c3[k] = c;
      y[k] = 0.0;
    }
  } else {
  for (int e0 = tid; e0 < T3 * n; e0 += kGsPre * NTH) {
    double gv[kGsPre];
#pragma unroll
    for (int q = 0; q < kGsPre; ++q) {
      const int e = e0 + q * NTH, ee = e < T3 * n ? e : 0;
      gv[q] = Gam[static_cast<int64_t>(grow(ee / n)) * ncol + 2 * Tp + ee % n];
    }
#pragma unroll
    for (int q = 0; q < kGsPre; ++q)
      if (e0 + q * NTH < T3 * n) Gs[e0 + q * NTH] = gv[q];
  }
  for (int k = tid; k < T3; k += NTH) {
    // constant part of the state: x_bar + Gamma_p u_prev - Gamma_f u_bar (:2877-2891)
    const int r = grow(k);
    const double *gr = Gam + static_cast<int64_t>(r) * ncol;
    double c = xb[r];
    if (uprev) {
#pragma unroll 8
      for (int j = 0; j < 2 * Tp; ++j) c += gr[j] * uprev[j];
    }
    if (ubar) {
#pragma unroll 8
      for (int j = 0; j < n; ++j) c -= gr[2 * Tp + j] * ubar[2 * Tp + j];
    }
    c3[k] = c;
    y[k] = 0.0;
  }
  }
  for (int j = tid; j < n; j += NTH) {
    // min_u / max_u = vstack((full(T, a), full(T, delta))).T.ravel() (:2874-2875): the bounds
    // interleave (accel, steer) per step like Gamma's columns, whatever U's reshape order
    const int c = j & 1;
    ub[j] = c == 0 ? p.max_a : p.max_delta;
    lb[j] = c == 0 ? p.min_a : -p.max_delta;
    z[j] = 0.0;
  }
  if constexpr (NW == 1 && NM == 16)  // n <= 16, where the layout reserves the table
    for (int e = tid; e < n * n; e += NTH) Hc[e] = hctrl(e / n, e % n, T, order, p);
  qp_sync<NW>();
  QS_MARK(0);
  for (int k = tid; k < T3; k += NTH) {
    // objective's linear term in output space: 2 (w_ref (c - ref_t) + [t = T-1] w_final (c - g))
    const int t = k / 3, a = k % 3;
    double v = 0.0;
    if (a < 2) {
      const int tr = t < A.n_ref ? t : A.n_ref - 1;
      v = 2.0 * p.w_ref * (c3[k] - (k == tid ? ref_k : ref[2 * tr + a]));
      if (t == T - 1) v += 2.0 * p.w_final * (c3[k] - (a == 0 ? g0 : g1));
    }
    qf[k] = v;
  }
  // obstacle rows: a . (y_xy + c_xy) <= b  ->  a . y_xy <= b' = b - a . c_xy
  int skipped = 0;
  double hmax = 0.0;
  auto obstacle_row = [&](int64_t r, const RecIn &ri) {
    const double n0 = ri.nn.x, n1 = ri.nn.y;
    const double d = __builtin_bit_cast(
        double, (static_cast<uint64_t>(static_cast<uint32_t>(ri.a.y)) << 32) |
                    static_cast<uint32_t>(ri.a.x));
    int side, status, tt;
    if (A.rec_compact) {  // ccmpc_gather_rec: the same fields, packed (int16 side, status)
      side = static_cast<int16_t>(ri.a.z & 0xFFFF);
      status = static_cast<int16_t>(static_cast<uint32_t>(ri.a.z) >> 16);
      tt = ri.a.w;
    } else {
      side = ri.b.y;
      status = ri.b.z;
      tt = ri.b.w;
    }
    const int t = A.rec_kind == CCMPC_REC_KIND_HALFSPACE ? tt >> 16 : tt;
    const bool ok = status == 0 && isfinite(n0) && isfinite(n1) && isfinite(d) && t >= 0 &&
                    t < T && (side == 1 || side == -1);
    double a0 = 0.0, a1 = 0.0, b = 1.0;
    if (ok) {
      // side +1: n . x >= d  ->  -n . x <= -d ;  side -1: n . x <= d  (:926-939, :1503-1515)
      a0 = side == 1 ? -n0 : n0;
      a1 = side == 1 ? -n1 : n1;
      b = (side == 1 ? -d : d) - (a0 * c3[3 * t] + a1 * c3[3 * t + 1]);
    } else {
      skipped = 1;
    }
    const int64_t ro = nbox + nv + r;
    const int ts = obst_step(r);
    rw.c0[ro] = a0;
    rw.c1[ro] = a1;
    rw.cst[ro] = -b;
    rw.ix[2 * ro] = 3 * ts;
    rw.ix[2 * ro + 1] = 3 * ts + 1;
    hmax = fmax(hmax, fabs(b));
  };
#if !CCMPC_QP_REC_PREFETCH
#pragma unroll
  for (int j = 0; j < kRecPre; ++j) {
    const int64_t r = tid + static_cast<int64_t>(j) * NTH;
    if (r < R) rpre[j] = load_rec(r);
  }
#endif
#pragma unroll
  for (int j = 0; j < kRecPre; ++j) {
    const int64_t r = tid + static_cast<int64_t>(j) * NTH;
    if (r < R) obstacle_row(r, rpre[j]);
  }
  for (int64_t r = tid + static_cast<int64_t>(kRecPre) * NTH; r < R; r += NTH)
    obstacle_row(r, load_rec(r));
  for (int r = tid; r < nbox + nv; r += NTH) {  // box and speed rows
    const bool lo = r & 1;
    int i0;
    double cst;
    if (r < nbox) {
      const int j = r >> 1;
      i0 = T3 + j;
      cst = lo ? lb[j] : -ub[j];
    } else {
      const int t = (r - nbox) >> 1;
      i0 = 3 * t + 2;
      cst = lo ? -c3[3 * t + 2] : c3[3 * t + 2] - p.max_v;
    }
    rw.c0[r] = lo ? -1.0 : 1.0;
    rw.c1[r] = 0.0;
    rw.cst[r] = cst;
    rw.ix[2 * r] = i0;
    rw.ix[2 * r + 1] = i0;
  }
  qp_sync<NW>();
  QS_MARK(1);
  // f = Gs^T qf (the scaling of the dual residual; kept in LDS for the polish)
  double fmax_ = 0.0;
  if constexpr (NW == 1 && NM == 16) {  // a quad per control, DPP sum (as the IPM's rd)
    const int j = lane >> 2, kq = lane & 3, jj = j < n ? j : 0;
    double v = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int k = kq + 4 * i, kk = k < T3 ? k : 0;
      const double g = Gs[kk * n + jj], qk = qf[kk];
      v = k < T3 ? fma(g, qk, v) : v;
    }
    v = sum4(v);
    if (kq == 0 && j < n) lds[lay.f + j] = v;
    fmax_ = j < n ? fabs(v) : 0.0;
  } else {
    for (int j = tid; j < n; j += NTH) {
      double v = 0.0;
      for (int k = 0; k < T3; ++k) v += Gs[k * n + j] * qf[k];
      lds[lay.f + j] = v;
      fmax_ = fmax(fmax_, fabs(v));
    }
  }
  QS_MARK(2);
  // initial point: z = 0 (inside the control box), s = max(-g(0), 1), lambda = 1
  // g(z) = row_lin(r, Gs z, z) + row_const(r): the linear part in the state's output rows
  // yy = Gs z (or in z itself for the control bounds), constants folded into b' and the bounds
  // (zz is yy + T3 in every caller: the pairs (y, z), (yd, dz) sit back to back)
  auto row_lin = [&](int64_t r, const double *yy, const double *zz) -> double {
    (void)zz;
    const int2 ix = reinterpret_cast<const int2 *>(rw.ix)[r];
    return rw.c0[r] * yy[ix.x] + rw.c1[r] * yy[ix.y];
  };
  auto row_const = [&](int64_t r) -> double { return rw.cst[r]; };
  auto row_g = [&](int64_t r, const double *yy, const double *zz) -> double {
    return row_lin(r, yy, zz) + row_const(r);
  };
  // Directional derivative of g along dz, given yd = Gs dz.  It must be the linear part
  // itself, never g(dz) - const: near the solution lambda ds / s amplifies any rounding in ds
  // by lambda / s, and an error here that the normal equations did not see leaves a dual
  // residual the iteration can no longer remove.
  auto row_gd = [&](int64_t r, const double *ydd, const double *dzz) -> double {
    return row_lin(r, ydd, dzz);
  };
  for (int64_t r = tid; r < mrows; r += NTH) {
    const double g = row_g(r, y, z);
    rw.s[r] = fmax(-g, 1.0);
    rw.l[r] = 1.0;
    if (r < nbox + nv) hmax = fmax(hmax, fabs(g));  // bounds' right-hand sides (z = y = 0)
  }
  block_max2<NW>(hmax, fmax_, red);
  QS_MARK(3);
  const double tol_p = A.tol * (1.0 + hmax), tol_d = A.tol * (1.0 + fmax_);

  // Per-step sums over a step's obstacle rows, in a fixed order (wave per step, lane-strided,
  // butterfly reduction).  Step t's rows of cell c are the run [start_t, start_t + cnt_t) of
  // the cell's records.  `val(r, t)` returns 2 (or 3) contributions of row r.
  // visit step t's obstacle rows idx = first, first + S, ... (< ncell t, or ncell) in that order,
  // fn(o) with o = cell P + t (t - 1) / 2 + j for idx = cell t + j (half-spaces; o = idx P + t
  // for affine records): (cell, j) advances by (S / t, S % t) per visit, no division per row
  struct StepIt {
    int cell0, j0, qS, rS;  // first / t, first % t, S / t, S % t
  };
  auto step_it = [&](int t, int first, int S) -> StepIt {
    if (A.rec_kind != CCMPC_REC_KIND_HALFSPACE || t < 1) return {0, 0, 0, 0};
    return {first / t, first % t, S / t, S % t};
  };
  auto for_step_it = [&](int t, int first, int S, const StepIt &si, auto &&fn) {
    if (A.rec_kind == CCMPC_REC_KIND_HALFSPACE) {
      if (t < 1) return;
      const int64_t cnt = ncell * t, base_t = t * (t - 1) / 2;
      int64_t cell = si.cell0;
      int j = si.j0;
      const int qS = si.qS, rS = si.rS;
      for (int64_t i = first; i < cnt; i += S) {
        fn(cell * P + base_t + j);
        cell += qS;
        j += rS;
        if (j >= t) {
          j -= t;
          ++cell;
        }
      }
    } else {
      for (int64_t i = first; i < ncell; i += S) fn(i * P + t);
    }
  };
  auto for_step = [&](int t, int first, int S, auto &&fn) {
    for_step_it(t, first, S, step_it(t, first, S), fn);
  };
  // one wave: lane (t, sub) = (lane >> 3, lane & 7) visits step t's rows sub, sub + 8, ...
  // (the same every iteration: the integer divisions happen once)
  const StepIt lane_it = NW == 1 ? step_it(lane >> 3, lane & 7, 8) : StepIt{0, 0, 0, 0};

  int status = 0, it = 0;
  double mu = 0.0, mu0 = 0.0;
  bool infeasible = false;
  bool polished = false, early_tried = false;
#ifdef CCMPC_QP_TRACE
  uint64_t tmark[8] = {};
  uint64_t pmark[8] = {};  // polish: first pass through each point
  const uint64_t tk1 = wall_clock64();
#endif
  constexpr int NR = NM > 0 ? NM : 1;
  double La[NR], Ldl = 0.0;  // wave 0: L of the current M (register path, NM > 0)
  // ---- polish: the equality-constrained QP on the IPM's active set ---------------------------
  // (as OSQP polishes an ADMM iterate).  Rows with s < lambda are taken as active; the KKT
  // system of  min 1/2 z^T H z + f^T z  s.t.  G_A z = h_A  is solved through H = L L^T and
  // S = W^T W, W = L^{-1} G_A^T:  lambda = S^{-1}(W^T y0 - h_A), y0 = -L^{-1} f,
  // z = L^{-T}(y0 - W lambda).  H carries no barrier weights, so this is as accurate as the
  // problem itself.  The result is kept only if it is a verified KKT point: every row within
  // tol_p and lambda >= -tol_d (stationarity holds by construction), which also makes a
  // stalled IPM's answer exact and leaves infeasible problems reported as such.  It depends on
  // the iterate only through the active set; it overwrites M (H and its factor), which the
  // early call site rebuilds on failure, and writes z only on success, so the IPM can try it
  // early: once mu is small the active set is usually settled, and a verified answer ends the
  // solve several iterations before the interior point would.  Returns true on a verified answer (z, status = 0).
  auto polish = [&](bool commit) -> bool {
    bool ok = false;
    double *Wm = lds + lay.pw, *Sm = lds + lay.ps, *act = lds + lay.pact,
           *sdinv = lds + lay.pdinv;
    double *fu = lds + lay.f, *y0 = rh, *rs = e2, *lam = q, *zp = dz, *yp = yd;
    PQ_MARK(0);
    // H (no barrier terms) into M; f in control space (fu) is the setup's
    if constexpr (NW == 1 && NM == 16) {  // as the IPM's M: lane column jm, rows (lane >> 4) + 4 m
      const int jm = lane & 15, jc = jm < n ? jm : 0;
      double hx[8], hy[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int tt = t < T ? t : 0;
        const double wp = 2.0 * (p.w_ref + (t == T - 1 ? p.w_final : 0.0));
        hx[t] = t < T ? wp * Gs[(3 * tt) * n + jc] : 0.0;
        hy[t] = t < T ? wp * Gs[(3 * tt + 1) * n + jc] : 0.0;
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int im = (lane >> 4) + 4 * m;
        const bool on = im < n && jm <= im;
        const int ic = on ? im : 0;
        double v = Hc[ic * n + jc];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int tt = t < T ? t : 0;
          v = fma(Gs[(3 * tt) * n + ic], hx[t], fma(Gs[(3 * tt + 1) * n + ic], hy[t], v));
        }
        if (on) M[im * ldm + jm] = v;
      }
    } else {
      for (int e = tid; e < n * n; e += NTH) {
        const int i = e / n, j = e % n;
        if (j > i) continue;
        double v = hctrl(i, j, T, order, p);
        for (int t = 0; t < T; ++t) {
          const double wp = 2.0 * (p.w_ref + (t == T - 1 ? p.w_final : 0.0));
          v += wp * (Gs[(3 * t) * n + i] * Gs[(3 * t) * n + j] +
                     Gs[(3 * t + 1) * n + i] * Gs[(3 * t + 1) * n + j]);
        }
        M[i * ldm + j] = v;
      }
    }
    PQ_MARK(1);
    // active rows, compacted in row order (ballot + prefix: deterministic)
    int na = 0;
    for (int64_t base = 0; base < mrows; base += NTH) {
      const int64_t r = base + tid;
      const bool on = r < mrows && rw.s[r] < rw.l[r];
      const uint64_t mask = __ballot(on);
      if (lane == 0) red[w] = static_cast<double>(__popcll(mask));
      qp_sync<NW>();
      int off = na;
      for (int k = 0; k < w; ++k) off += static_cast<int>(red[k]);
      int tot = na;
      for (int k = 0; k < NW; ++k) tot += static_cast<int>(red[k]);
      const int pos = off + __popcll(mask & ((uint64_t(1) << lane) - 1));
      if (on && pos < n) act[pos] = static_cast<double>(r);
      na = tot;
      qp_sync<NW>();
    }
    if constexpr (NM > 0 && NW == 1) {
      PQ_MARK(2);
      // One wave, n <= 16: the same polish with every factor in registers (identity-padded
      // to 16 x 16, straight-line; reg_cholesky without the pivot skip), the L^T columns read
      // ahead of each backward chain, the vectors moved between lanes by readlane.
      wave_sync();
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        const double v = M[(lane < n ? lane : 0) * ldm + (k < n ? k : 0)];
        La[k] = (lane < n && k <= lane) ? v : (k == lane ? 1.0 : 0.0);
      }
      const bool hfail = reg_cholesky<NR, false>(La, Ldl);
#pragma unroll
      for (int k = 0; k < NR; ++k)
        if (k < n && lane < n && k <= lane) M[lane * ldm + k] = La[k];
      wave_sync();
      double ltH[NR];
      reg_load_lt(M, ldm, n, ltH);
      const double y0r = reg_forward(La, Ldl, lane < n ? -fu[lane] : 0.0);  // y0 = -L^{-1} f
      if (lane < n) y0[lane] = y0r;
      if (hfail) status = CCMPC_QP_NUMERIC;  // H itself is not positive definite (bad weights)
      for (int round = 0; !hfail && round < 4 && na <= n; ++round) {
        PQ_MARK(3);
        // W rows w_a = L^{-1} g_a, rs_a = w_a . y0 - h_a: one active row per lane (na <= n),
        // each lane's own forward substitution (L's entries are the same address on every
        // lane: broadcast LDS reads), so all rows advance together instead of one triangular
        // solve per row.  The row's gradient from its one-form (c0, c1, i0, i1): d v[i] / d z_j
        // is Gs[i][j] for an output row i < T3, else [i - T3 == j].
        {
          const int a = lane < na ? lane : 0;
          const int64_t r = static_cast<int64_t>(act[a]);
          const int2 ix = reinterpret_cast<const int2 *>(rw.ix)[r];
          const double c0 = rw.c0[r], c1 = rw.c1[r];
          const int x0c = ix.x < T3 ? ix.x : 0, x1c = ix.y < T3 ? ix.y : 0;
          double wv[NR];
          double d = 0.0;
#pragma unroll
          for (int j = 0; j < NR; ++j) {
            const int jc = j < n ? j : 0;
            const double ga = Gs[x0c * n + jc], gb = Gs[x1c * n + jc];
            const double g0 = ix.x < T3 ? ga : (ix.x - T3 == j ? 1.0 : 0.0);
            const double g1 = ix.y < T3 ? gb : (ix.y - T3 == j ? 1.0 : 0.0);
            double v = c0 * g0 + c1 * g1;
#pragma unroll
            for (int k = 0; k < j; ++k) v = fma(-M[jc * ldm + k], wv[k], v);
            wv[j] = j < n ? v * lane_bcast(Ldl, j) : 0.0;
            d = fma(wv[j], lane_bcast(y0r, j), d);
          }
          if (lane < na) {
#pragma unroll
            for (int j = 0; j < NR; ++j)
              if (j < n) Wm[lane * n + j] = wv[j];
            rs[lane] = d + row_const(r);
          }
        }
        wave_sync();
        PQ_MARK(4);
        // S = W W^T: lane (i, kq) = (lane & 15, lane >> 4) forms S[i][kq + 4 m]
        {
          const int i = lane & 15, kq = lane >> 4, ic = i < na ? i : 0;
          double wi[NR];
#pragma unroll
          for (int k = 0; k < NR; ++k) wi[k] = Wm[ic * n + (k < n ? k : 0)];
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const int jr = kq + 4 * m, jc = jr < na ? jr : 0;
            double v = 0.0;
#pragma unroll
            for (int k = 0; k < NR; ++k)
              v = k < n ? fma(wi[k], Wm[jc * n + (k < n ? k : 0)], v) : v;
            if (i < na && jr <= i) Sm[i * ldm + jr] = v;
          }
        }
        wave_sync();
        double Ls[NR], Sdl = 0.0;
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          const double v = Sm[(lane < na ? lane : 0) * ldm + (k < na ? k : 0)];
          Ls[k] = (lane < na && k <= lane) ? v : (k == lane ? 1.0 : 0.0);
        }
        const bool sfail = reg_cholesky<NR, false>(Ls, Sdl);
        if (sfail) break;  // dependent active rows
#pragma unroll
        for (int k = 0; k < NR; ++k)
          if (k < na && lane < na && k <= lane) Sm[lane * ldm + k] = Ls[k];
        wave_sync();
        const double lamr = reg_solve(Ls, Sm, ldm, Sdl, na, lane < na ? rs[lane] : 0.0);
        if (lane < na) lam[lane] = lamr;
        PQ_MARK(5);
        // z = L^{-T}(y0 - W^T lambda)
        double v = y0r;
        {
          const int j = lane < n ? lane : 0;
#pragma unroll
          for (int a = 0; a < NR; ++a) {  // rows past na are never written (with na = 0 not
            // even row 0): select, never multiply, what may be stale LDS
            const double wa = Wm[(a < na ? a : 0) * n + j];
            v = a < na ? fma(-wa, lane_bcast(lamr, a), v) : v;
          }
        }
        const double zpr = reg_backward(ltH, Ldl, lane < n ? v : 0.0);
        if (lane < n) zp[lane] = zpr;
        {
          const int kk = lane < T3 ? lane : 0;
          double yv = 0.0;
#pragma unroll
          for (int j = 0; j < NR; ++j)
            yv = fma(Gs[kk * n + (j < n ? j : 0)], lane_bcast(zpr, j), yv);
          if (lane < T3) yp[lane] = yv;
        }
        wave_sync();
        PQ_MARK(6);
        double viol = -1e300, vrow = 0.0, lneg = 0.0, bad = 0.0;
        for (int64_t r = tid; r < mrows; r += NTH) {
          const double g = row_g(r, yp, zp);
          if (!isfinite(g)) bad = 1.0;
          if (g > viol) {
            viol = g;
            vrow = static_cast<double>(r);
          }
        }
        if (lane < na) {
          if (!isfinite(lamr)) bad = 1.0;
          lneg = -lamr;
        }
        block_argmax<NW>(viol, vrow, red);
        block_max2<NW>(lneg, bad, red);
        if (bad != 0.0) break;
        if (viol <= tol_p && lneg <= tol_d) {
          if (commit && lane < n) z[lane] = zpr;
          status = 0;
          ok = true;
          wave_sync();
          break;
        }
        // next active set (lane 0; na <= n entries)
        if (lane == 0) {
          int m2 = 0;
          if (lneg > tol_d) {
            for (int a = 0; a < na; ++a)
              if (lam[a] >= -tol_d) act[m2++] = act[a];
          } else {
            m2 = na;
            if (na < n) act[m2++] = vrow;
            else m2 = n + 1;  // nowhere to add: give up
          }
          red[8 * kQpWaves - 2] = static_cast<double>(m2);
        }
        wave_sync();
        na = static_cast<int>(red[8 * kQpWaves - 2]);
        wave_sync();
      }
    } else {
      // factor H once; y0 = -L^{-1} f
      if (w == 0) {
        const bool fail = wave_cholesky(M, n, ldm, dinv, false);
        double b[2];
        wave_load2(fu, n, b);
        b[0] = -b[0];
        b[1] = -b[1];
        wave_forward(M, n, ldm, dinv, b);
        wave_store2(y0, n, b);
        if (lane == 0) red[8 * kQpWaves - 1] = fail ? 1.0 : 0.0;
      }
      qp_sync<NW>();
      const bool h_ok = red[8 * kQpWaves - 1] == 0.0;
      if (!h_ok) status = CCMPC_QP_NUMERIC;  // H itself is not positive definite (bad weights)
      // up to 4 rounds of active-set correction, as the oracle's polish does: drop rows whose
      // multiplier comes out negative, else add the most violated row
      for (int round = 0; h_ok && round < 4 && na <= n; ++round) {
        // W rows (one per active row a, wave per row): w_a = L^{-1} g_a;  rs_a = w_a . y0 - h_a
        for (int a = w; a < na; a += NW) {
          const int64_t r = static_cast<int64_t>(act[a]);
          double b[2];
  #pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int j = lane + 64 * h;
            double g = 0.0;
            if (j < n) {
              if (r < nbox) {
                g = (j == static_cast<int>(r >> 1)) ? ((r & 1) ? -1.0 : 1.0) : 0.0;
              } else if (r < nbox + nv) {
                const int t = static_cast<int>((r - nbox) >> 1);
                g = ((r - nbox) & 1) ? -Gs[(3 * t + 2) * n + j] : Gs[(3 * t + 2) * n + j];
              } else {
                // the row's gradient in control space: a . (Gs_x, Gs_y) of its step
                const int64_t o = r - nbox - nv;
                const int t = rw.ix[2 * (nbox + nv + o)] / 3;
                g = oa0[o] * Gs[(3 * t) * n + j] + oa1[o] * Gs[(3 * t + 1) * n + j];
              }
            }
            b[h] = g;
          }
          wave_forward(M, n, ldm, dinv, b);
          wave_store2(Wm + a * n, n, b);
          double d = 0.0;
  #pragma unroll
          for (int h = 0; h < 2; ++h)
            if (lane + 64 * h < n) d += b[h] * y0[lane + 64 * h];
          d = wave_sum(d);
          if (lane == 0) rs[a] = d + row_const(r);
        }
        qp_sync<NW>();
        for (int e = tid; e < na * na; e += NTH) {
          const int i = e / na, j = e % na;
          if (j > i) continue;
          double v = 0.0;
          for (int k = 0; k < n; ++k) v += Wm[i * n + k] * Wm[j * n + k];
          Sm[i * ldm + j] = v;
        }
        qp_sync<NW>();
        if (w == 0) {
          const bool fail = na > 0 && wave_cholesky(Sm, na, ldm, sdinv, false);
          double b[2];
          if (!fail) {
            wave_load2(rs, na, b);
            wave_forward(Sm, na, ldm, sdinv, b);
            wave_backward(Sm, na, ldm, sdinv, b);
            wave_store2(lam, na, b);
          }
          if (lane == 0) red[8 * kQpWaves - 1] = fail ? 1.0 : 0.0;
        }
        qp_sync<NW>();
        if (red[8 * kQpWaves - 1] != 0.0) break;  // dependent active rows
        // z = L^{-T}(y0 - W^T lambda)
        for (int j = tid; j < n; j += NTH) {
          double v = y0[j];
          for (int a = 0; a < na; ++a) v -= Wm[a * n + j] * lam[a];
          zp[j] = v;
        }
        qp_sync<NW>();
        if (w == 0) {
          double b[2];
          wave_load2(zp, n, b);
          wave_backward(M, n, ldm, dinv, b);
          wave_store2(zp, n, b);
        }
        qp_sync<NW>();
        for (int k = tid; k < T3; k += NTH) {
          double v = 0.0;
          for (int j = 0; j < n; ++j) v += Gs[k * n + j] * zp[j];
          yp[k] = v;
        }
        qp_sync<NW>();
        double viol = -1e300, vrow = 0.0, lneg = 0.0, bad = 0.0;
        for (int64_t r = tid; r < mrows; r += NTH) {
          const double g = row_g(r, yp, zp);
          if (!isfinite(g)) bad = 1.0;
          if (g > viol) {
            viol = g;
            vrow = static_cast<double>(r);
          }
        }
        for (int a = tid; a < na; a += NTH) {
          if (!isfinite(lam[a])) bad = 1.0;
          lneg = fmax(lneg, -lam[a]);
        }
        block_argmax<NW>(viol, vrow, red);
        block_max2<NW>(lneg, bad, red);
        if (bad != 0.0) break;
        if (viol <= tol_p && lneg <= tol_d) {
          if (commit)
            for (int j = tid; j < n; j += NTH) z[j] = zp[j];
          status = 0;
          ok = true;
          qp_sync<NW>();
          break;
        }
        // next active set (thread 0; na <= n entries)
        if (tid == 0) {
          int m2 = 0;
          if (lneg > tol_d) {
            for (int a = 0; a < na; ++a)
              if (lam[a] >= -tol_d) act[m2++] = act[a];
          } else {
            m2 = na;
            if (na < n) act[m2++] = vrow;
            else m2 = n + 1;  // nowhere to add: give up
          }
          red[8 * kQpWaves - 2] = static_cast<double>(m2);
        }
        qp_sync<NW>();
        na = static_cast<int>(red[8 * kQpWaves - 2]);
        qp_sync<NW>();
      }
    }
    return ok;
  };

  // M = H_ctrl + D_box + sum_t Gs_t^T B_t Gs_t (the barrier-weighted normal matrix of I2).
  // A lambda so a failed early polish, which factors H in M's storage, can rebuild it.
  auto normal_matrix = [&]() {
    if constexpr (NW == 1 && NM == 16) {
      // lane column jm = lane & 15 (its weighted Gs columns in registers), rows
      // im = (lane >> 4) + 4 m
      const int jm = lane & 15, jc = jm < n ? jm : 0;
      double wx[8], wy[8], wv[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int tt = t < T ? t : 0;
        const double xj = Gs[(3 * tt) * n + jc], yj = Gs[(3 * tt + 1) * n + jc],
                     vj = Gs[(3 * tt + 2) * n + jc];
        const double b0 = bw[4 * tt], b1 = bw[4 * tt + 1], b2 = bw[4 * tt + 2],
                     b3 = bw[4 * tt + 3];
        wx[t] = t < T ? fma(b0, xj, b1 * yj) : 0.0;
        wy[t] = t < T ? fma(b1, xj, b2 * yj) : 0.0;
        wv[t] = t < T ? b3 * vj : 0.0;
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int im = (lane >> 4) + 4 * m;
        const bool on = im < n && jm <= im;
        const int ic = on ? im : 0;
        double v2 = Hc[ic * n + jc];
        if (ic == jc) v2 += rw.l[2 * ic] * rw.is[2 * ic] + rw.l[2 * ic + 1] * rw.is[2 * ic + 1];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int tt = t < T ? t : 0;
          const double xi = Gs[(3 * tt) * n + ic], yi = Gs[(3 * tt + 1) * n + ic],
                       vi = Gs[(3 * tt + 2) * n + ic];
          v2 = fma(xi, wx[t], fma(yi, wy[t], fma(vi, wv[t], v2)));
        }
        if (on) M[im * ldm + jm] = v2;
      }
    } else {
      for (int e = tid; e < n * n; e += NTH) {
        const int i = e / n, j = e % n;
        if (j > i) continue;
        double v = hctrl(i, j, T, order, p);
        if (i == j) v += rw.l[2 * i] * rw.is[2 * i] + rw.l[2 * i + 1] * rw.is[2 * i + 1];
        for (int t = 0; t < T; ++t) {
          const double xi = Gs[(3 * t) * n + i], yi = Gs[(3 * t + 1) * n + i],
                       vi = Gs[(3 * t + 2) * n + i];
          const double xj = Gs[(3 * t) * n + j], yj = Gs[(3 * t + 1) * n + j],
                       vj = Gs[(3 * t + 2) * n + j];
          v += xi * (bw[4 * t] * xj + bw[4 * t + 1] * yj) + yi * (bw[4 * t + 1] * xj +
               bw[4 * t + 2] * yj) + bw[4 * t + 3] * vi * vj;
        }
        M[i * ldm + j] = v;
      }
    }
  };

  // ---- Goldfarb-Idnani dual active-set solve (one wave, n <= 32; CCMPC_QP_METHOD_GI) --------
  // The strictly convex QP  min 1/2 z^T H z + f^T z  s.t.  g_r(z) <= 0  from its unconstrained
  // minimum: the most violated row (normalised by its gradient's norm) enters the active set,
  // primal steps along J2 d2 and dual steps along R^{-1} d1 keep the active multipliers >= 0
  // (dropping a row whose multiplier reaches 0), until no row is violated beyond tol_p (an
  // exact KKT point: the active rows hold as equalities, every multiplier >= 0) or no step
  // exists (the rows are infeasible: CCMPC_QP_MAXITER, the reference's solve failure).  H =
  // L L^T, J = L^{-T} rotated so that J^T N_A = [R; 0] (Givens rotations as rows enter and
  // leave).  J lives in M's storage (row-major, stride ldm), R in the polish's S (row-major,
  // upper triangle), the active rows and multipliers in the polish's act / dinv slots, the
  // row norms and active flags in the IPM's row arrays is / dl.  A solve that exceeds its step
  // budget or meets a non-finite value hands the problem to the IPM (returns false, z = y = 0).
  // Each active-set change is a handful of wave-wide LDS phases, and a T = 8 frame enters only
  // a few rows, where the IPM spends ~5 iterations and a polish (~130 us).
  bool gi_done = false;
  if constexpr (GI && NW == 1 && (NM == 16 || NM == 32)) {
    auto gi_solve = [&]() -> bool {
#ifdef CCMPC_QP_TRACE
      uint64_t gmark[6] = {}, gacc[6] = {}, gt = 0;
#define GI_MARK(i) (gmark[i] = wall_clock64())
#define GI_T0() (gt = wall_clock64())
#define GI_ACC(k)                         \
  do {                                    \
    const uint64_t gn_ = wall_clock64();  \
    gacc[k] += gn_ - gt;                  \
    gt = gn_;                             \
  } while (0)
#else
#define GI_MARK(i) ((void)0)
#define GI_T0() ((void)0)
#define GI_ACC(k) ((void)0)
#endif
      GI_MARK(0);
      double *Jm = M, *Rm = lds + lay.ps, *actv = lds + lay.pact, *uact = lds + lay.pdinv;
      const double *fu = lds + lay.f;
      double *inorm = rw.is, *aflag = rw.dl;
      const int li = lane < n ? lane : 0;
      auto gcol = [&](int i, int j) -> double {  // d v[i] / d z_j
        return i < T3 ? Gs[i * n + j] : (i - T3 == j ? 1.0 : 0.0);
      };
      auto update_y = [&]() {  // y = Gs z (the output rows' linear part)
        wave_sync();
        if (lane < T3) {
          double v = 0.0;
  #pragma unroll
          for (int j = 0; j < NM; ++j)
            if (j < n) v = fma(Gs[lane * n + j], z[j], v);
          y[lane] = v;
        }
        wave_sync();
      };
      auto give_up = [&]() -> bool {  // back to the IPM's starting point
        wave_sync();
        if (lane < n) z[lane] = 0.0;
        if (lane < T3) y[lane] = 0.0;
        for (int64_t r = lane; r < mrows; r += 64) rw.is[r] = 1.0 / rw.s[r];
        wave_sync();
        return false;
      };
      // H (no barrier terms) into M's lower triangle, as the polish builds it (n <= 32: entry by
      // entry, as the four-wave polish does)
      if constexpr (NM == 32) {
        for (int e = lane; e < n * n; e += 64) {
          const int i = e / n, j = e % n;
          if (j > i) continue;
          double v = hctrl(i, j, T, order, p);
          for (int t = 0; t < T; ++t) {
            const double wp = 2.0 * (p.w_ref + (t == T - 1 ? p.w_final : 0.0));
            v += wp * (Gs[(3 * t) * n + i] * Gs[(3 * t) * n + j] +
                       Gs[(3 * t + 1) * n + i] * Gs[(3 * t + 1) * n + j]);
          }
          M[i * ldm + j] = v;
        }
      } else {
        const int jm = lane & 15, jc = jm < n ? jm : 0;
        double hx[8], hy[8];
  #pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int tt = t < T ? t : 0;
          const double wp = 2.0 * (p.w_ref + (t == T - 1 ? p.w_final : 0.0));
          hx[t] = t < T ? wp * Gs[(3 * tt) * n + jc] : 0.0;
          hy[t] = t < T ? wp * Gs[(3 * tt + 1) * n + jc] : 0.0;
        }
  #pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int im = (lane >> 4) + 4 * m;
          const bool on = im < n && jm <= im;
          const int ic = on ? im : 0;
          double v = Hc[ic * n + jc];
  #pragma unroll
          for (int t = 0; t < 8; ++t) {
            const int tt = t < T ? t : 0;
            v = fma(Gs[(3 * tt) * n + ic], hx[t], fma(Gs[(3 * tt + 1) * n + ic], hy[t], v));
          }
          if (on) M[im * ldm + jm] = v;
        }
      }
      wave_sync();
      double La[NM], Ldl = 0.0;
  #pragma unroll
      for (int k = 0; k < NM; ++k) {
        const double v = M[li * ldm + (k < n ? k : 0)];
        La[k] = (lane < n && k <= lane) ? v : (k == lane ? 1.0 : 0.0);
      }
      if (reg_cholesky<NM, false>(La, Ldl)) return give_up();
      GI_MARK(1);
      // L (rows) and 1 / L_ii into R's storage (free until the first row enters) for the
      // column-parallel inverse below
      double *Ls = Rm, *Ldi = lds + lay.dinv;
      if (lane < n) {
#pragma unroll
        for (int k = 0; k < NM; ++k)
          if (k <= lane && k < n) Ls[lane * ldm + k] = La[k];
        Ldi[lane] = Ldl;
      }
      wave_sync();  // (every read of H is done too: J overwrites it)
      GI_MARK(2);
      // J = L^{-T}: lane c solves L x = e_c (all columns at once, L's entries broadcast from
      // LDS), x_k = L^{-1}[k][c] = J[c][k] -- lane c ends with row c of J
      double Jrow[NM];
#pragma unroll
      for (int k = 0; k < NM; ++k) {
        double acc = (k == lane) ? 1.0 : 0.0;
#pragma unroll
        for (int j = 0; j < k; ++j)
          if (k < n) acc = fma(-Ls[k * ldm + j], Jrow[j], acc);
        Jrow[k] = k < n ? acc * Ldi[k < n ? k : 0] : 0.0;
      }
      if (lane < n) {
#pragma unroll
        for (int k = 0; k < NM; ++k)
          if (k < n) Jm[lane * ldm + k] = Jrow[k];
      }
      // row gradient norms (the violation's scale) from each step's output-row Gram: an
      // obstacle row's gradient is a0 Gs_x(t) + a1 Gs_y(t), a speed row's +-Gs_v(t), a box
      // row's +-e_j
      double *Ngr = bw;  // (the IPM's per-step weights: recomputed in its I1)
      if (lane < T) {
        double xx = 0.0, xy = 0.0, yy = 0.0, vv = 0.0;
#pragma unroll
        for (int j = 0; j < NM; ++j) {
          if (j >= n) continue;
          const double gx = Gs[(3 * lane) * n + j], gy = Gs[(3 * lane + 1) * n + j],
                       gv = Gs[(3 * lane + 2) * n + j];
          xx = fma(gx, gx, xx);
          xy = fma(gx, gy, xy);
          yy = fma(gy, gy, yy);
          vv = fma(gv, gv, vv);
        }
        Ngr[4 * lane] = xx;
        Ngr[4 * lane + 1] = xy;
        Ngr[4 * lane + 2] = yy;
        Ngr[4 * lane + 3] = vv;
      }
      wave_sync();
      for (int64_t r = lane; r < mrows; r += 64) {
        const int2 ix = reinterpret_cast<const int2 *>(rw.ix)[r];
        const double a0 = rw.c0[r], a1 = rw.c1[r];
        double s2;
        if (ix.x >= T3) {
          s2 = a0 * a0 + a1 * a1;                        // a box row (i0 == i1)
        } else {
          const int t = ix.x / 3;
          s2 = (ix.x % 3 == 2) ? (a0 + a1) * (a0 + a1) * Ngr[4 * t + 3]
                               : a0 * a0 * Ngr[4 * t] + 2.0 * a0 * a1 * Ngr[4 * t + 1] +
                                     a1 * a1 * Ngr[4 * t + 2];
        }
        inorm[r] = s2 > 0.0 ? 1.0 / sqrt(s2) : 0.0;
        aflag[r] = 0.0;
      }
      GI_MARK(3);
      // the unconstrained minimum z = -J L^{-1} f (the forward solve on lane = row, then each
      // lane's row of J against it)
      {
        const double y0 = reg_forward<NM>(La, Ldl, lane < n ? fu[lane] : 0.0);
        double zi = 0.0;
#pragma unroll
        for (int k = 0; k < NM; ++k)
          if (k < n) zi = fma(Jrow[k], lane_bcast(y0, k), zi);
        wave_sync();
        if (lane < n) z[lane] = -zi;
      }
      update_y();
      GI_MARK(4);
      int q = 0, steps = 0;
      const int max_steps = A.gi_max_steps >= 0 ? A.gi_max_steps : 8 * (n + 16);
      double *Rdi = lds + lay.dinv;  // 1 / R[k][k] (L's reciprocals are no longer needed)
      // J stays in registers (lane i: row i, every rotation local); its LDS mirror serves the
      // column reads of d = J^T m
      auto store_j = [&]() {
        if (lane < n) {
#pragma unroll
          for (int k = 0; k < NM; ++k)
            if (k < n) Jm[lane * ldm + k] = Jrow[k];
        }
      };
      // a Givens rotation zeroing b against a: c = a / h, s = b / h, h = |(a, b)|, from the
      // hardware rsqrt with one Newton step (the rotation chain is serial; IEEE sqrt and two
      // divisions per rotation were most of an active-set change)
      auto givens = [](double a, double b, double &c, double &s, double &h) {
        const double n2 = fma(a, a, b * b);
        if (!(n2 > 0.0)) {
          c = 1.0;
          s = 0.0;
          h = 0.0;
          return;
        }
        double y = __builtin_amdgcn_rsq(n2);
        y = y * fma(-0.5 * n2 * y, y, 1.5);
        c = a * y;
        s = b * y;
        h = n2 * y;
      };
      while (true) {
        GI_T0();
        // the most violated row (normalised by its gradient), inactive rows only
        double best = 0.0, bidx = -1.0, cviol = 0.0;
#pragma unroll 2
        for (int64_t r = lane; r < mrows; r += 64) {
          const int2 ix = reinterpret_cast<const int2 *>(rw.ix)[r];
          const double g = row_g(r, y, z);
          const double inr = inorm[r];
          const bool on = aflag[r] == 0.0 && g > tol_p;
          if (!isfinite(g)) cviol = 2.0;
          if (on && inr == 0.0) cviol = fmax(cviol, 1.0);  // a violated constant row
          const double v = g * inr;
          if (on && v > best) {
            best = v;
            bidx = static_cast<double>(r);
          }
          (void)ix;
        }
        block_argmax<1>(best, bidx, red);
        const double cv = wave_max(cviol);
        GI_ACC(0);
        if (cv >= 2.0) return give_up();
        if (cv > 0.0) {  // no point satisfies it: infeasible
          status = CCMPC_QP_MAXITER;
          infeasible = true;
          it = steps;
          return true;
        }
        if (bidx < 0.0) break;  // every row holds: optimal
        const int64_t pr = static_cast<int64_t>(bidx);
        const int2 pix = reinterpret_cast<const int2 *>(rw.ix)[pr];
        const double pc0 = rw.c0[pr], pc1 = rw.c1[pr];
        // the entering row as m . z >= beta (m = -grad g): m_j on lane j
        const double mj = lane < n ? -(pc0 * gcol(pix.x, li) + pc1 * gcol(pix.y, li)) : 0.0;
        double sp = -row_g(pr, y, z);  // its slack (< 0)
        double uplus = 0.0;
        // m, fixed while this row enters: broadcast through LDS (the IPM's rh slots, free
        // here), read as VGPR operands -- sixteen readlane results held in SGPRs were part of
        // the kernel's SGPR spilling
        double *mvec = lds + lay.rh, *dvec = lds + lay.e2;
        wave_sync();
        if (lane < n) mvec[lane] = mj;
        wave_sync();
        while (true) {
          if (++steps > max_steps) return give_up();
          // d = J^T m (lane j), r = R^{-1} d[:q] (lane k < q)
          double dj = 0.0;
#pragma unroll
          for (int i = 0; i < NM; ++i)
            if (i < n) dj = fma(Jm[i * ldm + li], mvec[i], dj);
          // back substitution with this lane's row of R and 1 / R_jj read from LDS up front
          // (independent loads), the chain unrolled over j: a broadcast and an FMA per column
          // instead of a dependent LDS round trip (the same operations, the same bits)
          double rhs = dj, rk = 0.0;
          double Rrow[NM];
#pragma unroll
          for (int k = 0; k < NM; ++k) Rrow[k] = Rm[li * ldm + k];
          const double rdl = Rdi[li];
#pragma unroll
          for (int j = NM - 1; j >= 0; --j) {
            if (j >= q) continue;  // uniform
            const double xj = lane_bcast(rhs, j) * lane_bcast(rdl, j);
            if (lane == j) rk = xj;
            if (lane < j) rhs = fma(-Rrow[j], xj, rhs);
          }
          GI_ACC(1);
          double dd[NM];
          wave_sync();
          if (lane < n) dvec[lane] = dj;
          wave_sync();
#pragma unroll
          for (int k = 0; k < NM; ++k) dd[k] = dvec[k < n ? k : 0];
          double d2 = 0.0, dn2 = 0.0, zi = 0.0;
#pragma unroll
          for (int k = 0; k < NM; ++k) {
            if (k >= n) continue;
            dn2 = fma(dd[k], dd[k], dn2);
            if (k >= q) {
              d2 = fma(dd[k], dd[k], d2);
              zi = fma(Jrow[k], dd[k], zi);  // J2 d2: the primal direction
            }
          }
          if (!isfinite(dn2)) return give_up();
          const bool zero_step = !(d2 > 1e-24 * dn2);
          // partial step: the first active multiplier to reach 0 (smallest lane on ties)
          const double ratio =
              (lane < q && rk > 0.0) ? uact[lane < q ? lane : 0] / rk : INFINITY;
          const double t1 = wave_min(ratio);
          const int l =
              t1 < INFINITY
                  ? __ffsll(static_cast<long long>(__ballot(lane < q && ratio == t1))) - 1
                  : -1;
          const double t2 = zero_step ? INFINITY : -sp / d2;
          // no step exists: the entering row's normal lies in the span of the active normals
          // (d2 ~ 0) with coefficients r <= 0, and the row is violated at a point where every
          // active row holds -- a Farkas certificate that the rows are infeasible (the
          // reference's solve failure): any z meeting the active rows has m.z <= sum_j r_j
          // beta_j = beta + sp < beta.  Its tests compare against round-off scales (zero_step,
          // rk > 0), which near-parallel rows of several cells at one t can tip;
          // an entry r_j ~ 0 of the wrong sign moves m.z by |r_j| |n_j . z| only, so the
          // verdict is kept when the entering row's violation is far above that scale (1e-6 of
          // its gradient's norm), and a marginal one is handed to the IPM, which confirms it
          // or finds the point
          if (!(t1 < INFINITY) && !(t2 < INFINITY)) {
            const double viol = -sp * inorm[pr];
            const bool certain = viol > 1e-6;
            if (A.gi_nostep == 1 || (A.gi_nostep == 2 && !certain)) return give_up();
            status = CCMPC_QP_MAXITER;
            infeasible = true;
            it = steps;
            return true;
          }
          GI_ACC(2);
          const double t = fmin(t1, t2);
          wave_sync();
          if (lane < q) uact[lane] -= t * rk;
          if (!zero_step && lane < n) z[lane] += t * zi;
          uplus += t;
          if (!zero_step) sp = fma(t, d2, sp);
          const bool full = !zero_step && t2 <= t1;
          if (full) {
            // add the row: rotate d[q:] onto d[q] (J's columns q .. n-1), R's new column
            double (&dv)[NM] = dd;  // rotated in place (dd is not read again)
#pragma unroll
            for (int j = NM - 1; j >= 1; --j) {
              if (j >= n || j <= q) continue;
              double c, s, h;
              givens(dv[j - 1], dv[j], c, s, h);
              dv[j - 1] = h;
              dv[j] = 0.0;
              const double x0 = Jrow[j - 1], x1 = Jrow[j];
              Jrow[j - 1] = fma(c, x0, s * x1);
              Jrow[j] = fma(-s, x0, c * x1);
            }
            double rqq = 0.0;
#pragma unroll
            for (int k = 0; k < NM; ++k)
              if (k == q) rqq = dv[k];
            if (rqq < 0.0) {
              rqq = -rqq;
#pragma unroll
              for (int k = 0; k < NM; ++k)
                if (k == q) Jrow[k] = -Jrow[k];
            }
            if (!(rqq > 1e-300)) return give_up();  // dependent row with a primal step
            wave_sync();
            store_j();
            if (lane < q) Rm[lane * ldm + q] = dj;
            if (lane == q) {
              Rm[q * ldm + q] = rqq;
              Rdi[q] = 1.0 / rqq;
              actv[q] = static_cast<double>(pr);
              uact[q] = uplus;
            }
            if (lane == 0) aflag[pr] = 1.0;
            ++q;
            GI_ACC(3);
            update_y();
            GI_ACC(5);
            break;
          }
          // drop active row l: R's columns l+1 .. q-1 shift left (lane = column), then
          // rotations on rows (k, k+1), k = l .. q-2, restore the triangle; J's columns
          // (k, k+1) likewise
          double Rc[NM];
          {
            const int col = (lane >= l && lane < q - 1) ? lane + 1 : (lane < q ? lane : 0);
#pragma unroll
            for (int i = 0; i < NM; ++i) Rc[i] = (i < q) ? Rm[i * ldm + col] : 0.0;
          }
          // (k unrolled: registers indexed directly, no select over the whole row per rotation)
#pragma unroll
          for (int k = 0; k < NM - 1; ++k) {
            if (k < l || k >= q - 1) continue;  // uniform
            double c, s, h;
            givens(lane_bcast(Rc[k], k), lane_bcast(Rc[k + 1], k), c, s, h);
            const double r0 = Rc[k], r1 = Rc[k + 1];
            Rc[k] = fma(c, r0, s * r1);
            Rc[k + 1] = fma(-s, r0, c * r1);
            const double x0 = Jrow[k], x1 = Jrow[k + 1];
            Jrow[k] = fma(c, x0, s * x1);
            Jrow[k + 1] = fma(-s, x0, c * x1);
          }
          double rdg = 1.0;
#pragma unroll
          for (int i = 0; i < NM; ++i)
            if (i == lane) rdg = Rc[i];
          const double act_next = actv[(lane + 1 < q ? lane + 1 : 0)];
          const double u_next = uact[(lane + 1 < q ? lane + 1 : 0)];
          const double dropped = actv[l];
          wave_sync();
          if (lane < q - 1) {
#pragma unroll
            for (int i = 0; i < NM; ++i)
              if (i <= lane) Rm[i * ldm + lane] = Rc[i];
            Rdi[lane] = 1.0 / rdg;
            if (lane >= l) {
              actv[lane] = act_next;
              uact[lane] = u_next;
            }
          }
          store_j();
          if (lane == 0) aflag[static_cast<int64_t>(dropped)] = 0.0;
          --q;
          GI_ACC(4);
          update_y();
          GI_ACC(5);
          if (!zero_step) sp = -row_g(pr, y, z);  // the entering row's slack at the new point
        }
      }
      status = 0;
      it = steps;
#ifdef CCMPC_QP_TRACE
      GI_MARK(5);
      if (tid == 0 && sc == 0)
        printf("gi phases (10ns): H+chol %d L %d J+norms %d z0 %d loop %d (steps %d, q %d)\n"
               "   loop: scan %d d+r %d dir+ratios %d add %d drop %d update_y %d\n",
               int(gmark[1] - gmark[0]), int(gmark[2] - gmark[1]), int(gmark[3] - gmark[2]),
               int(gmark[4] - gmark[3]), int(gmark[5] - gmark[4]), steps, q, int(gacc[0]),
               int(gacc[1]), int(gacc[2]), int(gacc[3]), int(gacc[4]), int(gacc[5]));
#endif
#undef GI_MARK
#undef GI_T0
#undef GI_ACC
      return true;
    };
    if (A.polish) gi_done = gi_solve();
    if constexpr (GIONLY) {
      if (!gi_done) status = kQpNeedIpm;  // the IPM pass launched next takes this scene
    }
  }

#ifdef CCMPC_QP_TRACE
  uint64_t tk2 = 0;
#endif
  // the IPM and the polish: compiled out of the active-set-only instance (its registers)
  if constexpr (!GIONLY) {
  for (; !gi_done && it <= A.max_iter; ++it) {
    QP_MARK(0);
    // ---- I1: residual norms, mu, per-step sums for r_d and M -------------------------------
    double rpmax = 0.0, sl = 0.0;
    for (int64_t r = tid; r < mrows; r += NTH) {
      const double s = rw.s[r];
      const double rp = row_g(r, y, z) + s;
      rw.rp[r] = rp;
      rw.is[r] = 1.0 / s;
      rpmax = fmax(rpmax, fabs(rp));
      sl += s * rw.l[r];
    }
    qp_sync<NW>();
    // step sums of one row: lambda a and the weights' (lambda / s) a a^T
    double la0, la1, w00, w01, w11;
    auto step_acc = [&](int64_t o) {
      const int64_t r = nbox + nv + o;
      const double a0 = oa0[o], a1 = oa1[o], lam = rw.l[r], wr = lam * rw.is[r];
      la0 = fma(lam, a0, la0);
      la1 = fma(lam, a1, la1);
      const double wa0 = wr * a0;
      w00 = fma(wa0, a0, w00);
      w01 = fma(wa0, a1, w01);
      w11 = fma(wr * a1, a1, w11);
    };
    if constexpr (NW == 1) {
      // one wave, T <= 8: lanes (t, sub) = (lane >> 3, lane & 7), every step's sums at once
      const int t = lane >> 3, sub = lane & 7;
      la0 = la1 = w00 = w01 = w11 = 0.0;
      if (t < T) for_step_it(t, sub, 8, lane_it, step_acc);
      la0 = sum8(la0);
      la1 = sum8(la1);
      w00 = sum8(w00);
      w01 = sum8(w01);
      w11 = sum8(w11);
      if (sub == 0 && t < T) {
        const double wp = 2.0 * (p.w_ref + (t == T - 1 ? p.w_final : 0.0));
        const int64_t rv = nbox + 2 * t;
        q[3 * t] = wp * y[3 * t] + qf[3 * t] + la0;
        q[3 * t + 1] = wp * y[3 * t + 1] + qf[3 * t + 1] + la1;
        q[3 * t + 2] = rw.l[rv] - rw.l[rv + 1];
        bw[4 * t] = wp + w00;
        bw[4 * t + 1] = w01;
        bw[4 * t + 2] = wp + w11;
        bw[4 * t + 3] = rw.l[rv] * rw.is[rv] + rw.l[rv + 1] * rw.is[rv + 1];
      }
    } else for (int t = w; t < T; t += NW) {
      la0 = la1 = w00 = w01 = w11 = 0.0;
      for_step(t, lane, 64, step_acc);
      la0 = wave_sum(la0);
      la1 = wave_sum(la1);
      w00 = wave_sum(w00);
      w01 = wave_sum(w01);
      w11 = wave_sum(w11);
      if (lane == 0) {
        const double wp = 2.0 * (p.w_ref + (t == T - 1 ? p.w_final : 0.0));
        const int64_t rv = nbox + 2 * t;
        q[3 * t] = wp * y[3 * t] + qf[3 * t] + la0;  // H_pos z + f + G^T lambda, output space
        q[3 * t + 1] = wp * y[3 * t + 1] + qf[3 * t + 1] + la1;
        q[3 * t + 2] = rw.l[rv] - rw.l[rv + 1];
        bw[4 * t] = wp + w00;
        bw[4 * t + 1] = w01;
        bw[4 * t + 2] = wp + w11;
        bw[4 * t + 3] = rw.l[rv] * rw.is[rv] + rw.l[rv + 1] * rw.is[rv + 1];
      }
    }
    qp_sync<NW>();
    QP_MARK(1);
    // ---- I2: dual residual, normal matrix ---------------------------------------------------
    double rdmax = 0.0;
    if constexpr (NW == 1) {
      // lanes (j, kq) = (lane >> 2, lane & 3): a quad per control, each lane a quarter of the
      // T3 <= 24 output rows, summed by DPP; every load in-bounds, out-of-range terms selected
      // away, so the unrolled loads all issue ahead of the FMA chain
      const int j = lane >> 2, kq = lane & 3, jj = j < n ? j : 0;
      double v = 0.0;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int k = kq + 4 * i, kk = k < T3 ? k : 0;
        const double g = Gs[kk * n + jj], qk = q[kk];
        v = k < T3 ? fma(g, qk, v) : v;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // + H_ctrl z
        const int k = kq + 4 * i, kk = k < n ? k : 0;
        const double h = Hc[jj * n + kk], zk = z[kk];
        v = k < n ? fma(h, zk, v) : v;
      }
      v = sum4(v) + (rw.l[2 * jj] - rw.l[2 * jj + 1]);
      if (kq == 0 && j < n) rd[j] = v;
      rdmax = j < n ? fabs(v) : 0.0;
    } else {
    for (int j = tid; j < n; j += NTH) {
      double v = hctrl_mul(z, j, T, order, p) + rw.l[2 * j] - rw.l[2 * j + 1];
      for (int k = 0; k < T3; ++k) v += Gs[k * n + j] * q[k];
      rd[j] = v;
      rdmax = fmax(rdmax, fabs(v));
    }
    }
    normal_matrix();
    block_max2<NW>(rpmax, rdmax, red);
    mu = block_sum<NW>(sl, red) / static_cast<double>(mrows);
#ifdef CCMPC_QP_TRACE
    const double tr_rp = rpmax, tr_rd = rdmax;
    if (it == 0 && tid == 0 && sc == 0)
      printf("qp it %d rp %.3e/%.3e rd %.3e/%.3e mu %.3e\n", it, tr_rp, tol_p, tr_rd, tol_d, mu);
#endif
    if (it == 0) mu0 = mu;
    if (rpmax <= tol_p && rdmax <= tol_d && mu <= A.tol) break;
    // mu far below the tolerance: the active set is settled, and from here the normal
    // equations lose accuracy (weights ~ 1/mu), so stop and leave the last digits to the polish
    // step; the iterate counts as solved if it is primal feasible with a near-zero dual
    // residual, else only a verified polish can answer
    if (mu <= 1e-3 * A.tol) {
      status = (rpmax <= tol_p && rdmax <= 1e3 * tol_d) ? 0 : CCMPC_QP_MAXITER;
      break;
    }
    // complementarity growing without bound: no interior solution (infeasible), no polish
    if (mu > 1e6 * fmax(mu0, 1.0)) {
      status = CCMPC_QP_MAXITER;
      infeasible = true;
      break;
    }
    if (it == A.max_iter || !isfinite(mu) || !isfinite(rpmax) || !isfinite(rdmax)) {
      status = CCMPC_QP_MAXITER;
      break;
    }
    // one early polish attempt once mu has fallen by A.early (kEarlyPolish)
    if (A.polish && A.early > 0.0 && !early_tried && it >= 2 && mu <= A.early * fmax(mu0, 1.0)) {
      early_tried = true;
      if (polish(!A.early_discard) && !A.early_discard) {
        polished = true;
        break;
      }
      // the polish factored H in M's storage (and may have set a status): restore the
      // barrier-weighted normal matrix this iteration's factor needs, so a failed attempt
      // leaves the IPM exactly where it was
      status = 0;
      qp_sync<NW>();
      normal_matrix();
      qp_sync<NW>();
    }
    QP_MARK(2);
    // ---- I3: Cholesky on wave 0 (left-looking, lane = row) ---------------------------------
    // Near the solution the active rows' weights lambda/s grow without bound, and a pivot of
    // the (mathematically positive definite) M can come out <= 0 after cancellation against
    // them.  Such a pivot is replaced by a huge one (the pivot-skip modified Cholesky of
    // interior point codes): that direction's component of dz becomes 0, which is what the
    // huge weight enforces anyway.
    bool chol_fail = false;  // wave-uniform (NW == 1: the only wave)
    if (w == 0) {
      bool fail;
      if constexpr (NM > 0) {
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          const double v = M[(lane < n ? lane : 0) * ldm + (k < n ? k : 0)];
          La[k] = (lane < n && k <= lane) ? v : (k == lane ? 1.0 : 0.0);
        }
        fail = reg_cholesky(La, Ldl);
        // L overwrites M's lower triangle (read by the L^T solves)
#pragma unroll
        for (int k = 0; k < NR; ++k)
          if (k < n && lane < n && k <= lane) M[lane * ldm + k] = La[k];
        wave_sync();
      } else {
        fail = wave_cholesky(M, n, ldm, dinv, true);
      }
      if (NW == 1)
        chol_fail = fail;
      else if (lane == 0)
        red[8 * kQpWaves - 1] = fail ? 1.0 : 0.0;
    }
    if constexpr (NW > 1) {
      qp_sync<NW>();
      chol_fail = red[8 * kQpWaves - 1] != 0.0;
    }
    if (chol_fail) {  // weights overflowed: the iteration broke down;
      status = CCMPC_QP_MAXITER;           // only a verified polish can still answer
      break;
    }
    // triangular solves on wave 0: L L^T x = rhs (rhs in registers, lane = row)
    auto chol_solve = [&](double *x) {
      if (w != 0) return;
      if constexpr (NM > 0) {
        const double b = reg_solve(La, M, ldm, Ldl, n, lane < n ? x[lane] : 0.0);
        if (lane < n) x[lane] = b;
        if constexpr (NW == 1) {  // yd = Gs dz, dz read back by readlane (0 beyond n)
          const int kk = lane < T3 ? lane : 0;
          double v = 0.0;
#pragma unroll
          for (int j = 0; j < NM; ++j) v = fma(Gs[kk * n + (j < n ? j : 0)], lane_bcast(b, j), v);
          if (lane < T3) yd[lane] = v;
          wave_sync();
        }
      } else {
        double b[2];
        wave_load2(x, n, b);
        wave_forward(M, n, ldm, dinv, b);
        wave_backward(M, n, ldm, dinv, b);
        wave_store2(x, n, b);
      }
    };
    auto gs_times_dz = [&]() {
      if constexpr (NW == 1) return;  // done inside chol_solve from the registers
      for (int k = tid; k < T3; k += NTH) {
        double v = 0.0;
        for (int j = 0; j < n; ++j) v += Gs[k * n + j] * dz[j];
        yd[k] = v;
      }
      qp_sync<NW>();
    };
    // rhs = -r_d - G^T u with u_r given per row; q (output space) and dz (rhs) staged in LDS
    auto build_rhs = [&](auto urow) {
      double u0, u1;
      auto acc = [&](int64_t o) {
        const double u = urow(nbox + nv + o);
        u0 = fma(u, oa0[o], u0);
        u1 = fma(u, oa1[o], u1);
      };
      if constexpr (NW == 1) {   // as I1: lanes (t, sub), every step at once
        const int t = lane >> 3, sub = lane & 7;
        u0 = u1 = 0.0;
        if (t < T) for_step_it(t, sub, 8, lane_it, acc);
        u0 = sum8(u0);
        u1 = sum8(u1);
        if (sub == 0 && t < T) {
          const int64_t rv = nbox + 2 * t;
          q[3 * t] = u0;
          q[3 * t + 1] = u1;
          q[3 * t + 2] = urow(rv) - urow(rv + 1);
        }
      } else for (int t = w; t < T; t += NW) {
        u0 = u1 = 0.0;
        for_step(t, lane, 64, acc);
        u0 = wave_sum(u0);
        u1 = wave_sum(u1);
        if (lane == 0) {
          const int64_t rv = nbox + 2 * t;
          q[3 * t] = u0;
          q[3 * t + 1] = u1;
          q[3 * t + 2] = urow(rv) - urow(rv + 1);
        }
      }
      qp_sync<NW>();
      if constexpr (NW == 1) {  // quad per control, as rd
        const int j = lane >> 2, kq = lane & 3, jj = j < n ? j : 0;
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const int k = kq + 4 * i, kk = k < T3 ? k : 0;
          const double g = Gs[kk * n + jj], qk = q[kk];
          v = k < T3 ? fma(g, qk, v) : v;
        }
        v = (-rd[jj] - (urow(2 * jj) - urow(2 * jj + 1))) - sum4(v);
        if (kq == 0 && j < n) dz[j] = v;
      } else {
        for (int j = tid; j < n; j += NTH) {
          double v = -rd[j] - (urow(2 * j) - urow(2 * j + 1));
          for (int k = 0; k < T3; ++k) v -= Gs[k * n + j] * q[k];
          dz[j] = v;
        }
      }
      qp_sync<NW>();
      chol_solve(dz);
      qp_sync<NW>();
      gs_times_dz();
    };
    QP_MARK(3);
    // ---- predictor (affine scaling): r_c = s l  ->  u = w r_p - l ---------------------------
    build_rhs([&](int64_t r) {
      const double l = rw.l[r];
      return l * rw.is[r] * rw.rp[r] - l;
    });
    QP_MARK(4);
    // the largest step keeping s, lambda >= 0: min over rows of -s / ds (ds < 0) and -l / dl
    // (dl < 0), kept as a fraction num / den (both > 0; compared by cross-multiplication) so
    // each lane divides once
    double anum = 1.0, aden = 1.0;
    auto ratio_min = [&](double num, double den) {  // candidate num / den, den > 0
      if (num * aden < anum * den) {
        anum = num;
        aden = den;
      }
    };
    for (int64_t r = tid; r < mrows; r += NTH) {
      const double s = rw.s[r], l = rw.l[r], rp = rw.rp[r];
      const double gd = row_gd(r, yd, dz);
      const double ds = -rp - gd, dl = l * rw.is[r] * (gd + rp) - l;
      rw.ds[r] = ds;
      rw.dl[r] = dl;
      if (ds < 0.0) ratio_min(s, -ds);
      if (dl < 0.0) ratio_min(l, -dl);
    }
    const double aaff = block_min<NW>(anum / aden, red);
    double slaff = 0.0;
    for (int64_t r = tid; r < mrows; r += NTH)
      slaff += (rw.s[r] + aaff * rw.ds[r]) * (rw.l[r] + aaff * rw.dl[r]);
    const double muaff = block_sum<NW>(slaff, red) / static_cast<double>(mrows);
    const double sr = muaff / mu, sigma = sr * sr * sr;
    QP_MARK(5);
    // ---- corrector: r_c = s l + ds_aff dl_aff - sigma mu;  u = w r_p - r_c / s ----------
    auto rc_of = [&](int64_t r) {
      return rw.s[r] * rw.l[r] + rw.ds[r] * rw.dl[r] - sigma * mu;
    };
    build_rhs([&](int64_t r) {
      return (rw.l[r] * rw.rp[r] - rc_of(r)) * rw.is[r];
    });
    QP_MARK(6);
    anum = 1e300;
    aden = 1.0;
    for (int64_t r = tid; r < mrows; r += NTH) {
      const double s = rw.s[r], l = rw.l[r], rp = rw.rp[r];
      const double gd = row_gd(r, yd, dz);
      const double rc = rc_of(r);
      const double ds = -rp - gd, dl = (-rc - l * ds) * rw.is[r];
      rw.ds[r] = ds;  // every read of this row's ds_aff / dl_aff happened above in this thread
      rw.dl[r] = dl;
      if (ds < 0.0) ratio_min(s, -ds);
      if (dl < 0.0) ratio_min(l, -dl);
    }
    const double alpha = fmin(1.0, 0.995 * block_min<NW>(anum / aden, red));

    for (int j = tid; j < n; j += NTH) z[j] += alpha * dz[j];
    for (int k = tid; k < T3; k += NTH) y[k] += alpha * yd[k];
    for (int64_t r = tid; r < mrows; r += NTH) {
      rw.s[r] += alpha * rw.ds[r];
      rw.l[r] += alpha * rw.dl[r];
    }
    qp_sync<NW>();
#ifdef CCMPC_QP_TRACE
    QP_MARK(7);
    if (tid == 0 && sc == 0)
      printf("qp it %d rp %.3e rd %.3e mu %.3e alpha %.3e\n   t(10ns) I1 %d I2 %d chol %d "
             "pred_rhs %d pred_step %d corr_rhs %d corr_step %d\n", it, tr_rp, tr_rd, mu, alpha,
             int(tmark[1] - tmark[0]), int(tmark[2] - tmark[1]), int(tmark[3] - tmark[2]),
             int(tmark[4] - tmark[3]), int(tmark[5] - tmark[4]), int(tmark[6] - tmark[5]),
             int(tmark[7] - tmark[6]));
#endif
  }

#ifdef CCMPC_QP_TRACE
  tk2 = wall_clock64();
#endif
  if (A.polish && !infeasible && !polished && !gi_done) polished = polish(true);
  }
#ifdef CCMPC_QP_TRACE
  const uint64_t tk3 = wall_clock64();
#endif
  // ---- outputs: u, X = Gamma_f u + const (all four state rows), the objective value ----------
  for (int j = tid; j < n; j += NTH) A.out_u[sc * n + j] = z[j];
  double part = 0.0;
  for (int r = tid; r < 4 * T; r += NTH) {
    const int gr = 4 * Tp + r;
    const double *g = Gam + static_cast<int64_t>(gr) * ncol;
    double x = xb[gr];
    if (uprev)
      for (int j = 0; j < 2 * Tp; ++j) x += g[j] * uprev[j];
    for (int j = 0; j < n; ++j) x += g[2 * Tp + j] * (z[j] - (ubar ? ubar[2 * Tp + j] : 0.0));
    A.out_x[sc * 4 * T + r] = x;
    const int t = r / 4, a = r % 4;
    if (a < 2) {  // compute_objective_referenceTraj (:2478-2507) at the solution
      const int tr = t < A.n_ref ? t : A.n_ref - 1;
      const double e = x - ref[2 * tr + a];
      part += p.w_ref * e * e;
      if (t == T - 1) {
        const double ef = x - (a == 0 ? g0 : g1);
        part += p.w_final * ef * ef;
      }
    }
  }
  for (int t = tid; t < T; t += NTH) {
    const double a0 = z[u_index(t, 0, T, order)], a1 = z[u_index(t, 1, T, order)];
    part += a0 * (p.w_accel * a0 + p.w_joint * a1) + a1 * (p.w_joint * a0 + p.w_turning * a1);
    if (t >= 1) {
      const double d0 = a0 - z[u_index(t - 1, 0, T, order)];
      const double d1 = a1 - z[u_index(t - 1, 1, T, order)];
      part += d0 * (p.w_ch_accel * d0 + p.w_ch_joint * d1) +
              d1 * (p.w_ch_joint * d0 + p.w_ch_turning * d1);
    }
  }
  const double cost = block_sum<NW>(part, red);
  double sk = skipped;
  double dummy = 0.0;
  block_max2<NW>(sk, dummy, red);
  if (tid == 0) {
    A.out_cost[sc] = cost;
    A.out_status[sc] = status | (sk > 0.0 ? CCMPC_QP_SKIPPED_ROWS : 0);
    A.out_iter[sc] = it;
  }
#ifdef CCMPC_QP_TRACE
  const uint64_t tk4 = wall_clock64();
  if (tid == 0 && sc == 0)
    printf("qp setup (10ns): model %d rows %d f %d init %d\n"
           "qp phases (10ns): setup %d iterations %d polish %d outputs %d\n"
           "   polish (first round): H %d act %d factor %d W %d S %d z %d\n",
           int(smark[0] - tk0), int(smark[1] - smark[0]), int(smark[2] - smark[1]),
           int(smark[3] - smark[2]), int(tk1 - tk0),
           int(tk2 - tk1), int(tk3 - tk2), int(tk4 - tk3), int(pmark[1] - pmark[0]),
           int(pmark[2] - pmark[1]), int(pmark[3] - pmark[2]), int(pmark[4] - pmark[3]),
           int(pmark[5] - pmark[4]), int(pmark[6] - pmark[5]));
#endif
}

// Where the per-scene state lives: the polish step's matrices come first (they make the
// answer exact), then the row store if it still fits; otherwise the rows go to the workspace.
struct QpPlan {
  bool rows_lds, polish;
};
inline bool qp_fits(int T, int64_t R, bool rows_lds, bool polish) {
  return static_cast<size_t>(QpLayout(T, rows_lds ? R : 0, rows_lds, polish).total) *
             sizeof(double) <= kQpLdsBytes;
}
inline QpPlan qp_plan(int T, int64_t R) {
  if (qp_fits(T, R, true, true)) return {true, true};
  if (qp_fits(T, R, false, true)) return {false, true};
  if (qp_fits(T, R, true, false)) return {true, false};
  return {false, false};
}

template <bool ROWS_LDS, int NM, int NW, bool GI = false, bool GIONLY = false>
hipError_t launch_qp(dim3 grid, size_t lds, hipStream_t s, const QpArgs &a) {
  const dim3 block(64 * NW);
  // the dynamic-LDS limit is a per-device attribute: set it on every launch (cheap), so a
  // process that drives several devices raises it on each, and report a failure as such
  if (lds > 48 * 1024) {
    const hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void *>(mpc_qp_kernel<ROWS_LDS, NM, NW, GI, GIONLY>),
        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kQpLdsBytes));
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((mpc_qp_kernel<ROWS_LDS, NM, NW, GI, GIONLY>), grid, block, lds, s, a);
  return hipSuccess;
}

}  // namespace ccmpc

using namespace ccmpc;

extern "C" int ccmpc_mpc_ltv(const double *x_init, int64_t n_scenes, int64_t T, double Ts,
                             double l_r, double L, double *out_xbar, double *out_gamma,
                             ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T >= 1 && T <= kQpMaxT, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_scenes >= 0, "bad n_scenes");
  if (n_scenes == 0) return CCMPC_OK;
  CCMPC_REQUIRE(x_init && out_xbar && out_gamma, "null pointer");
  CCMPC_REQUIRE(Ts > 0.0 && L > 0.0 && l_r > 0.0, "Ts, L, l_r must be positive");
  hipLaunchKernelGGL(mpc_ltv_kernel, dim3(static_cast<unsigned>(n_scenes)), dim3(256), 0,
                     as_stream(stream), x_init, n_scenes, static_cast<int>(T), Ts, l_r, L,
                     out_xbar, out_gamma);
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}

extern "C" size_t ccmpc_mpc_qp_workspace_bytes(int64_t n_scenes, int64_t T,
                                               int64_t max_cells_per_scene, int rec_kind) {
  if (T < 1 || T > kQpMaxT || n_scenes < 0 || max_cells_per_scene < 0) return 0;
  const int64_t R = max_cells_per_scene * qp_rows_per_cell(static_cast<int>(T), rec_kind & 1);
  if (qp_plan(static_cast<int>(T), R).rows_lds) return 16;  // rows live in LDS
  const int64_t m = 4 * T + 2 * T + R;
  return static_cast<size_t>(n_scenes * kQpRowDoubles * m) * sizeof(double) + 16;
}

static int mpc_qp_impl(const ccmpc_qp_ltv *ltv, int64_t n_scenes, int64_t T, int64_t T_full,
                       const double *gamma, const double *xbar, const double *ubar,
                       const double *u_prev, const double *goal, const double *ref,
                       int64_t n_ref, const void *rec, int rec_kind, const int64_t *scene_cell,
                       int64_t max_cells_per_scene, const ccmpc_mpc_params *params, int u_order,
                       int32_t max_iter, double tol, void *workspace, size_t workspace_bytes,
                       double *out_u, double *out_x, double *out_cost, int32_t *out_status,
                       int32_t *out_iter, ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T >= 1 && T <= kQpMaxT, "T must be in [1, 40]");
  CCMPC_REQUIRE(T_full >= T && T_full <= kQpMaxT, "T_full must be in [T, 40]");
  CCMPC_REQUIRE(n_scenes >= 0 && n_scenes < (int64_t(1) << 31), "bad n_scenes");
  if (n_scenes == 0) return CCMPC_OK;
  CCMPC_REQUIRE(gamma && xbar && goal && ref && scene_cell && params, "null pointer");
  CCMPC_REQUIRE(out_u && out_x && out_cost && out_status && out_iter, "null pointer");
  CCMPC_REQUIRE(T_full == T || u_prev, "u_prev is required when T < T_full");
  CCMPC_REQUIRE(n_ref >= 1, "n_ref must be >= 1");
  CCMPC_REQUIRE(rec_kind >= CCMPC_REC_KIND_HALFSPACE && rec_kind <= CCMPC_REC_KIND_AFFINE_COMPACT,
                "bad rec_kind");
  CCMPC_REQUIRE(u_order == CCMPC_U_ORDER_F || u_order == CCMPC_U_ORDER_C, "bad u_order");
  CCMPC_REQUIRE(max_cells_per_scene >= 0, "bad max_cells_per_scene");
  CCMPC_REQUIRE(max_cells_per_scene == 0 || rec, "null records");
  CCMPC_REQUIRE(max_iter >= 1 && tol > 0.0, "max_iter >= 1 and tol > 0 required");
  if (workspace_bytes < ccmpc_mpc_qp_workspace_bytes(n_scenes, T, max_cells_per_scene,
                                                     rec_kind)) {
    set_error("ccmpc_mpc_qp: workspace too small");
    return CCMPC_ERR_WORKSPACE;
  }
  const int Ti = static_cast<int>(T);
  const int64_t R = max_cells_per_scene * qp_rows_per_cell(Ti, rec_kind & 1);
  const QpPlan plan = qp_plan(Ti, R);
  const bool in_lds = plan.rows_lds;
  CCMPC_REQUIRE(in_lds || workspace, "null workspace");
  QpArgs a{};
  a.S = n_scenes;
  a.T = Ti;
  a.Tf = static_cast<int>(T_full);
  a.n_ref = static_cast<int>(n_ref);
  a.u_order = u_order;
  a.rec_kind = rec_kind & 1;  // the source kind: halfspace (0 / 2) or affine (1 / 3)
  a.rec_compact = rec_kind >= CCMPC_REC_KIND_HALFSPACE_COMPACT;
  a.max_iter = max_iter;
  a.rows_in_lds = in_lds;
  a.polish = plan.polish;
  {
    const char *e = getenv("CCMPC_QP_METHOD");  // per call (tests switch it)
    a.method = (e && strcmp(e, "ipm") == 0) ? CCMPC_QP_METHOD_IPM
               : (e && strcmp(e, "gi") == 0) ? CCMPC_QP_METHOD_GI : kQpDefaultMethod;
  }
  {
    const char *e = getenv("CCMPC_QP_GI_MAX_STEPS");  // per call (test hook)
    a.gi_max_steps = e ? atoi(e) : -1;
    const char *ns = getenv("CCMPC_QP_GI_NOSTEP");    // per call (A/B and tests)
    a.gi_nostep = ns ? atoi(ns) : 2;
  }
  {
    const char *e = getenv("CCMPC_QP_EARLY_POLISH");  // per call (a test switches it)
    const double v = e ? atof(e) : kEarlyPolish;
    a.early = fabs(v);
    a.early_discard = v < 0.0;
  }
  a.max_cells = max_cells_per_scene;
  a.tol = tol;
  a.gamma = gamma;
  a.xbar = xbar;
  a.ubar = ubar;
  a.u_prev = u_prev;
  a.goal = goal;
  a.ref = ref;
  a.rec = static_cast<const unsigned char *>(rec);
  a.scene_cell = scene_cell;
  a.p = *params;
  a.ws = static_cast<double *>(workspace);
  a.out_u = out_u;
  a.out_x = out_x;
  a.out_cost = out_cost;
  a.out_status = out_status;
  a.out_iter = out_iter;
  if (ltv) {
    CCMPC_REQUIRE(ltv->x_init, "null x_init");
    CCMPC_REQUIRE(ltv->Ts > 0.0 && ltv->L > 0.0 && ltv->l_r > 0.0,
                  "Ts, L, l_r must be positive");
    CCMPC_REQUIRE(!ubar, "the fused LTV rebuild is the model about u = 0 (ubar must be NULL)");
    a.ltv_x0 = ltv->x_init;
    a.ltv_Ts = ltv->Ts;
    a.ltv_lr = ltv->l_r;
    a.ltv_L = ltv->L;
    a.ltv_xbar = const_cast<double *>(xbar);
    a.ltv_gamma = const_cast<double *>(gamma);
  }
  const size_t lds = static_cast<size_t>(QpLayout(Ti, in_lds ? R : 0, in_lds, plan.polish).total) *
                     sizeof(double);
  CCMPC_REQUIRE(lds <= kQpLdsBytes, "T too large for the LDS image");
  const int n = 2 * Ti;
  // register-resident factor up to n = 16 (T <= 8, the reference's ph); larger n spills
  const int nm = n <= 16 ? 16 : 0;
  // one wave per scene with the register factor (n <= 16), unless CCMPC_QP_WAVES=4 asks for the
  // four-wave form (A/B)
  static const int waves_env = [] {
    const char *e = getenv("CCMPC_QP_WAVES");
    return e ? atoi(e) : 1;
  }();
  const bool one_wave = nm == 16 && waves_env == 1;
  const dim3 grid(static_cast<unsigned>(n_scenes));
  hipStream_t s = as_stream(stream);
  hipError_t attr;
  const bool gi = one_wave && a.method == CCMPC_QP_METHOD_GI && plan.polish;
  // a batch runs the active-set pass without the IPM's code in its instance (189 instead of
  // 488 VGPRs, far fewer SGPR spills), then an IPM pass that solves only the scenes it handed
  // over -- the IPM's own answer, byte for byte, as the combined instance's hand-over gives;
  // a single scene keeps the combined instance (the second launch would cost it more)
  // (CCMPC_QP_GI_SPLIT: 0 never, 1 batches -- the default --, 2 a single scene too)
  const char *se = getenv("CCMPC_QP_GI_SPLIT");
  const int split_env = se ? atoi(se) : 1;
  // n = 17 .. 32 (T = 9 .. 16): the active-set pass on one wave (factor and J in registers,
  // 32 per lane), then the four-wave IPM pass for the scenes it handed over
  const bool gi32 = n > 16 && n <= 32 && a.method == CCMPC_QP_METHOD_GI && plan.polish;
  if (gi32) {
    attr = in_lds ? launch_qp<true, 32, 1, true, true>(grid, lds, s, a)
                  : launch_qp<false, 32, 1, true, true>(grid, lds, s, a);
    if (attr == hipSuccess) {
      QpArgs f = a;
      f.fallback_only = 1;
      attr = in_lds ? launch_qp<true, 0, 4>(grid, lds, s, f)
                    : launch_qp<false, 0, 4>(grid, lds, s, f);
    }
  } else if (gi && split_env > 0 && (n_scenes > 1 || split_env > 1)) {
    attr = in_lds ? launch_qp<true, 16, 1, true, true>(grid, lds, s, a)
                  : launch_qp<false, 16, 1, true, true>(grid, lds, s, a);
    if (attr == hipSuccess) {
      QpArgs f = a;
      f.fallback_only = 1;
      attr = in_lds ? launch_qp<true, 16, 1>(grid, lds, s, f)
                    : launch_qp<false, 16, 1>(grid, lds, s, f);
    }
  } else if (gi) {
    attr = in_lds ? launch_qp<true, 16, 1, true>(grid, lds, s, a)
                  : launch_qp<false, 16, 1, true>(grid, lds, s, a);
  } else if (in_lds) {
    attr = one_wave ? launch_qp<true, 16, 1>(grid, lds, s, a)
                    : (nm == 16 ? launch_qp<true, 16, 4>(grid, lds, s, a)
                                : launch_qp<true, 0, 4>(grid, lds, s, a));
  } else {
    attr = one_wave ? launch_qp<false, 16, 1>(grid, lds, s, a)
                    : (nm == 16 ? launch_qp<false, 16, 4>(grid, lds, s, a)
                                : launch_qp<false, 0, 4>(grid, lds, s, a));
  }
  if (attr != hipSuccess) {
    set_error(std::string(__func__) + ": hipFuncSetAttribute(MaxDynamicSharedMemorySize) "
              "failed: " + hipGetErrorString(attr));
    return CCMPC_ERR_LAUNCH;
  }
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}

extern "C" int ccmpc_mpc_qp(int64_t n_scenes, int64_t T, int64_t T_full, const double *gamma,
                            const double *xbar, const double *ubar, const double *u_prev,
                            const double *goal, const double *ref, int64_t n_ref,
                            const void *rec, int rec_kind, const int64_t *scene_cell,
                            int64_t max_cells_per_scene, const ccmpc_mpc_params *params,
                            int u_order, int32_t max_iter, double tol, void *workspace,
                            size_t workspace_bytes, double *out_u, double *out_x,
                            double *out_cost, int32_t *out_status, int32_t *out_iter,
                            ccmpc_stream_t stream) {
  return mpc_qp_impl(nullptr, n_scenes, T, T_full, gamma, xbar, ubar, u_prev, goal, ref, n_ref,
                     rec, rec_kind, scene_cell, max_cells_per_scene, params, u_order, max_iter,
                     tol, workspace, workspace_bytes, out_u, out_x, out_cost, out_status,
                     out_iter, stream);
}

extern "C" int ccmpc_mpc_qp_ltv(const ccmpc_qp_ltv *ltv, int64_t n_scenes, int64_t T,
                                int64_t T_full, double *gamma, double *xbar,
                                const double *u_prev, const double *goal, const double *ref,
                                int64_t n_ref, const void *rec, int rec_kind,
                                const int64_t *scene_cell, int64_t max_cells_per_scene,
                                const ccmpc_mpc_params *params, int u_order, int32_t max_iter,
                                double tol, void *workspace, size_t workspace_bytes,
                                double *out_u, double *out_x, double *out_cost,
                                int32_t *out_status, int32_t *out_iter, ccmpc_stream_t stream) {
  CCMPC_REQUIRE(ltv, "null ltv");
  return mpc_qp_impl(ltv, n_scenes, T, T_full, gamma, xbar, nullptr, u_prev, goal, ref, n_ref,
                     rec, rec_kind, scene_cell, max_cells_per_scene, params, u_order, max_iter,
                     tol, workspace, workspace_bytes, out_u, out_x, out_cost, out_status,
                     out_iter, stream);
}
