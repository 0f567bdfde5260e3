// predict_ideal: affine conditional-Gaussian forward rollout (v8ideal/__init__.py:2620-2711).
//
// For each cell, step t maps the previous planning step's moments to
//   A_t = C(t+1, t) inv(Sigma_t),  L_t = chol(Sigma_{t+1} - A_t C(t+1, t)^T)
//   x_{t+1} = mu_{t+1} + A_t (x_t - mu_t) + L_t z,     z ~ N(0, I)
// with ONE shared x0 for all rows (:2664-2665).  The per-step (A_t, L_t) are 2x2 and computed
// on the device from the moments the previous step left in HBM -- the reference's pickle round
// trip (:2612-2635) becomes a pointer.
//
// Two forms:
//  * ideal_rollout_kernel writes the trajectories (plane-major f64), one sample per lane.
//  * ideal_gram_kernel never stores them: each wave rolls 64 samples, stages them through LDS
//    as [row][sample] (row stride 66 doubles -> conflict-free ds_write_b64 and ds_read_b64 in
//    the MFMA layout) and feeds the same f64 MFMA Gram reduction as ccmpc_moments.  The
//    reference's only consumer of the 1e6-row ideal trajectories is np.cov (:886-907,
//    :2586-2606), so this removes 32 * n * T bytes of HBM traffic per cell.
#include "gram.hpp"

namespace ccmpc {

struct StepPlan {
  double a00, a01, a10, a11;  // A_t
  double l00, l10, l11;       // L_t (lower)
  double mu0, mu1;            // mu_t
  double nu0, nu1;            // mu_{t+1}
};

// Builds plan[t] for t < T (called by lanes t < T).  Returns a CCMPC_REC_* code or 0.
__device__ int build_step(const double *__restrict__ mean, const double *__restrict__ cov,
                          int rows_src, int t, StepPlan &sp) {
  auto blk = [&](int i, int j, double &a, double &b, double &c, double &d) {
    const double *p = cov + (2 * i) * rows_src + 2 * j;
    a = p[0];
    b = p[1];
    c = p[rows_src];
    d = p[rows_src + 1];
  };
  double s0, s1, s2, s3, n0, n1, n2, n3, c0, c1, c2, c3;
  blk(t, t, s0, s1, s2, s3);          // cov_tau
  blk(t + 1, t + 1, n0, n1, n2, n3);  // cov_next
  blk(t + 1, t, c0, c1, c2, c3);      // C_t_tp1 = cross_cov[t+1][t]
  const double det = s0 * s3 - s1 * s2;
  if (det == 0.0 || !isfinite(det)) return CCMPC_REC_SINGULAR;
  const double inv_det = 1.0 / det;
  const double i0 = s3 * inv_det, i1 = -s1 * inv_det, i2 = -s2 * inv_det, i3 = s0 * inv_det;
  sp.a00 = c0 * i0 + c1 * i2;
  sp.a01 = c0 * i1 + c1 * i3;
  sp.a10 = c2 * i0 + c3 * i2;
  sp.a11 = c2 * i1 + c3 * i3;
  // cond_cov = cov_next - A C^T ; Cholesky reads the lower triangle (potrf 'L')
  const double k00 = n0 - (sp.a00 * c0 + sp.a01 * c1);
  const double k10 = n2 - (sp.a10 * c0 + sp.a11 * c1);
  const double k11 = n3 - (sp.a10 * c2 + sp.a11 * c3);
  if (!(k00 > 0.0)) return CCMPC_REC_NOT_PD;
  sp.l00 = sqrt(k00);
  sp.l10 = k10 / sp.l00;
  const double r = k11 - sp.l10 * sp.l10;
  if (!(r > 0.0)) return CCMPC_REC_NOT_PD;
  sp.l11 = sqrt(r);
  sp.mu0 = mean[2 * t];
  sp.mu1 = mean[2 * t + 1];
  sp.nu0 = mean[2 * t + 2];
  sp.nu1 = mean[2 * t + 3];
  return 0;
}

// x0 = given, or mean_0 + chol(cov_0) z with z = Philox pair (0, 0, rng, X0 stream)
__device__ void initial_draw(const double *__restrict__ mean, const double *__restrict__ cov,
                             int rows_src, const double *__restrict__ x0, int cell, uint32_t rng,
                             uint64_t seed, double &x, double &y, int &status) {
  if (x0) {
    x = x0[2 * cell];
    y = x0[2 * cell + 1];
    return;
  }
  const double a = cov[0], b = cov[rows_src], d = cov[rows_src + 1];
  double z0, z1;
  normal_pair(0u, 0u, rng, STREAM_IDEAL_X0, seed, z0, z1);
  if (!(a > 0.0) || !(d - (b / sqrt(a)) * (b / sqrt(a)) > 0.0)) {
    status = CCMPC_REC_NOT_PD;
    x = y = NAN;
    return;
  }
  const double l00 = sqrt(a), l10 = b / l00, l11 = sqrt(d - l10 * l10);
  x = mean[0] + l00 * z0;
  y = mean[1] + (l10 * z0 + l11 * z1);
}

__device__ __forceinline__ void advance(const StepPlan &sp, double z0, double z1, double &x,
                                        double &y) {
  const double d0 = x - sp.mu0, d1 = y - sp.mu1;
  const double c0 = sp.nu0 + (d0 * sp.a00 + d1 * sp.a01);
  const double c1 = sp.nu1 + (d0 * sp.a10 + d1 * sp.a11);
  x = c0 + (z0 * sp.l00);
  y = c1 + (z0 * sp.l10 + z1 * sp.l11);
}

__global__ __launch_bounds__(256) void ideal_rollout_kernel(
    const double *__restrict__ prev_mean, const double *__restrict__ prev_cov, int T_src,
    const int32_t *__restrict__ src_cell, int T, int64_t n, const double *__restrict__ x0,
    const double *__restrict__ Z, uint64_t seed, const int32_t *__restrict__ rng_cell,
    double *__restrict__ out, int64_t ld, int32_t *__restrict__ out_status) {
  __shared__ StepPlan plan[40];
  __shared__ int status_s;
  __shared__ double x0_s[2];
  const int cell = blockIdx.y;
  const int rows_src = 2 * T_src;
  const int src = src_cell ? src_cell[cell] : cell;
  const double *mu = prev_mean + static_cast<int64_t>(src) * rows_src;
  const double *cv = prev_cov + static_cast<int64_t>(src) * rows_src * rows_src;
  const uint32_t rng = rng_cell ? static_cast<uint32_t>(rng_cell[cell]) : static_cast<uint32_t>(cell);
  if (threadIdx.x == 0) status_s = 0;
  __syncthreads();
  if (threadIdx.x < T) {
    const int st = build_step(mu, cv, rows_src, threadIdx.x, plan[threadIdx.x]);
    if (st) atomicMin(&status_s, st);
  }
  if (threadIdx.x == 64) {
    int st = 0;
    initial_draw(mu, cv, rows_src, x0, cell, rng, seed, x0_s[0], x0_s[1], st);
    if (st) atomicMin(&status_s, st);
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0 && out_status) out_status[cell] = status_s;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x = x0_s[0], y = x0_s[1];
  double *o = out + static_cast<int64_t>(cell) * ((n + 3) & ~int64_t(3)) + i;
  for (int t = 0; t < T; ++t) {
    double z0, z1;
    if (Z) {
      const double *zp = Z + ((static_cast<int64_t>(cell) * T + t) * 2) * n + i;
      z0 = zp[0];
      z1 = zp[n];
    } else {
      normal_pair(static_cast<uint32_t>(i), static_cast<uint32_t>(t), rng, STREAM_IDEAL_Z, seed, z0,
                  z1);
    }
    advance(plan[t], z0, z1, x, y);
    o[(2 * t) * ld] = x;
    o[(2 * t + 1) * ld] = y;
  }
}

constexpr int kStageStride = 66;  // doubles per LDS row: bank-conflict-free both ways

template <int RB>
__global__ __launch_bounds__(64) void ideal_gram_kernel(
    const double *__restrict__ prev_mean, const double *__restrict__ prev_cov, int T_src,
    const int32_t *__restrict__ src_cell, int T, int64_t n, int64_t chunk, int64_t items_per_cell,
    const double *__restrict__ x0, uint64_t seed, const int32_t *__restrict__ rng_cell,
    double *__restrict__ partial, double *__restrict__ shift_buf,
    int32_t *__restrict__ out_status) {
  constexpr int NT = n_tiles(RB);
  constexpr int D = 16 * RB;
  __shared__ StepPlan plan[40];
  __shared__ double stage[D * kStageStride];
  __shared__ double shift_s[D];
  __shared__ int status_s;
  const int lane = threadIdx.x;
  const int64_t item = blockIdx.x;
  const int cell = static_cast<int>(item / items_per_cell);
  const int64_t cidx = item % items_per_cell;
  const int rows = 2 * T, rows_src = 2 * T_src;
  const int src = src_cell ? src_cell[cell] : cell;
  const double *mu = prev_mean + static_cast<int64_t>(src) * rows_src;
  const double *cv = prev_cov + static_cast<int64_t>(src) * rows_src * rows_src;
  const uint32_t rng = rng_cell ? static_cast<uint32_t>(rng_cell[cell]) : static_cast<uint32_t>(cell);
  if (lane == 0) status_s = 0;
  __syncthreads();
  for (int t = lane; t < T; t += 64) {
    const int st = build_step(mu, cv, rows_src, t, plan[t]);
    if (st) atomicMin(&status_s, st);
  }
  __syncthreads();
  double x0x, x0y;
  {
    int st = 0;
    initial_draw(mu, cv, rows_src, x0, cell, rng, seed, x0x, x0y, st);
    if (st && lane == 0) atomicMin(&status_s, st);
  }
  // shift = the noise-free path (the rollout's exact mean given x0): same for every item
  if (lane == 0) {
    double x = x0x, y = x0y;
    for (int t = 0; t < T; ++t) {
      advance(plan[t], 0.0, 0.0, x, y);
      shift_s[2 * t] = x;
      shift_s[2 * t + 1] = y;
    }
    for (int R = rows; R < D; ++R) shift_s[R] = 0.0;
  }
  __syncthreads();
  if (cidx == 0) {
    for (int R = lane; R < rows; R += 64) shift_buf[static_cast<int64_t>(cell) * rows + R] = shift_s[R];
    if (lane == 0 && out_status) out_status[cell] = status_s;
  }

  typedef double d4v __attribute__((ext_vector_type(4)));
  d4v acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = d4v{0.0, 0.0, 0.0, 0.0};
  double s1[RB];
#pragma unroll
  for (int b = 0; b < RB; ++b) s1[b] = 0.0;
  const int r = lane & 15, g = lane >> 4;
  const int64_t p0 = cidx * chunk;
  const int64_t p1 = (p0 + chunk < n) ? p0 + chunk : n;

  for (int64_t base = p0; base < p1; base += 64) {
    const int64_t i = base + lane;
    const bool valid = i < p1;
    double x = x0x, y = x0y;
    for (int t = 0; t < T; ++t) {
      double z0, z1;
      normal_pair(static_cast<uint32_t>(i), static_cast<uint32_t>(t), rng, STREAM_IDEAL_Z, seed, z0,
                  z1);
      advance(plan[t], z0, z1, x, y);
      stage[(2 * t) * kStageStride + lane] = valid ? x - shift_s[2 * t] : 0.0;
      stage[(2 * t + 1) * kStageStride + lane] = valid ? y - shift_s[2 * t + 1] : 0.0;
    }
    __syncthreads();
#pragma unroll 4
    for (int j = 0; j < 16; ++j) {
      double v[RB];
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        const int R = 16 * b + r;
        v[b] = (R < rows) ? stage[R * kStageStride + 4 * j + g] : 0.0;
        s1[b] += v[b];
      }
      int t = 0;
#pragma unroll
      for (int bi = 0; bi < RB; ++bi)
#pragma unroll
        for (int bj = bi; bj < RB; ++bj) {
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(v[bi], v[bj], acc[t], 0, 0, 0);
          ++t;
        }
    }
    __syncthreads();
  }

  double *slab = partial + item * slab_doubles(RB);
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int k = 0; k < 4; ++k) slab[t * 256 + k * 64 + lane] = acc[t][k];
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    double x = s1[b];
    x += __shfl_xor(x, 16, 64);
    x += __shfl_xor(x, 32, 64);
    if (lane < 16) slab[NT * 256 + b * 16 + lane] = x;
  }
}

inline int64_t ideal_chunk(int64_t n_cells, int64_t n) {
  int64_t c = (n_cells * n + 2047) / 2048;
  c = ((c + 63) / 64) * 64;
  if (c < 256) c = 256;
  if (c > 16384) c = 16384;
  return c;
}

template <int RB>
static void launch_ideal_gram(const double *pm, const double *pc, int T_src, const int32_t *src,
                              int n_cells, int T, int64_t n, const double *x0, uint64_t seed,
                              const int32_t *rng, double *partial, double *shift,
                              double *out_mean, double *out_cov, int32_t *status, hipStream_t s) {
  const int64_t chunk = ideal_chunk(n_cells, n);
  const int64_t ipc = (n + chunk - 1) / chunk;
  hipLaunchKernelGGL((ideal_gram_kernel<RB>), dim3(static_cast<unsigned>(ipc * n_cells)), dim3(64),
                     0, s, pm, pc, T_src, src, T, n, chunk, ipc, x0, seed, rng, partial, shift,
                     status);
  hipLaunchKernelGGL((gram_finalize_kernel<double, RB>), dim3(n_cells), dim3(256), 0, s,
                     static_cast<const double *>(nullptr), int64_t(0), T,
                     static_cast<const double *>(shift), static_cast<const double *>(nullptr),
                     static_cast<const int64_t *>(nullptr), static_cast<const int64_t *>(nullptr),
                     n, chunk, static_cast<const double *>(partial), out_mean, out_cov);
}

}  // namespace ccmpc

using namespace ccmpc;

extern "C" int ccmpc_ideal_rollout(const double *prev_mean, const double *prev_cov,
                                   int64_t T_src, const int32_t *src_cell, int64_t n_cells,
                                   int64_t T, int64_t n_samples, const double *x0,
                                   const double *Z, uint64_t seed, const int32_t *rng_cell,
                                   double *out_positions, int64_t ld, int32_t *out_status,
                                   ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T_src >= 2 && T_src <= kMaxT, "T_src must be in [2, 40]");
  CCMPC_REQUIRE(T >= 1 && T <= T_src - 1, "T must be in [1, T_src - 1]");
  CCMPC_REQUIRE(n_cells >= 0 && n_cells < 65536, "bad n_cells");
  CCMPC_REQUIRE(n_samples >= 1 && n_samples < (int64_t(1) << 32), "bad n_samples");
  if (n_cells == 0) return CCMPC_OK;
  CCMPC_REQUIRE(prev_mean && prev_cov && out_positions, "null pointer");
  CCMPC_REQUIRE(ld >= n_cells * ((n_samples + 3) & ~int64_t(3)),
                "ld must be >= n_cells * round_up(n_samples, 4)");
  const unsigned bx = static_cast<unsigned>((n_samples + 255) / 256);
  hipLaunchKernelGGL(ideal_rollout_kernel, dim3(bx, static_cast<unsigned>(n_cells)), dim3(256), 0,
                     as_stream(stream), prev_mean, prev_cov, static_cast<int>(T_src), src_cell,
                     static_cast<int>(T), n_samples, x0, Z, seed, rng_cell, out_positions, ld,
                     out_status);
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}

extern "C" size_t ccmpc_ideal_moments_workspace_bytes(int64_t T, int64_t n_cells,
                                                      int64_t n_samples) {
  if (T < 1 || T > kMaxT || n_cells < 0 || n_samples < 1) return 0;
  const int64_t chunk = ideal_chunk(n_cells, n_samples);
  const int64_t items = ((n_samples + chunk - 1) / chunk) * n_cells;
  const int rb = row_blocks(T);
  return static_cast<size_t>(items * slab_doubles(rb) + n_cells * 2 * T) * sizeof(double);
}

extern "C" int ccmpc_ideal_moments(const double *prev_mean, const double *prev_cov,
                                   int64_t T_src, const int32_t *src_cell, int64_t n_cells,
                                   int64_t T, int64_t n_samples, const double *x0, uint64_t seed,
                                   const int32_t *rng_cell, void *workspace,
                                   size_t workspace_bytes, double *out_mean, double *out_cov,
                                   int32_t *out_status, ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T_src >= 2 && T_src <= kMaxT, "T_src must be in [2, 40]");
  CCMPC_REQUIRE(T >= 1 && T <= T_src - 1, "T must be in [1, T_src - 1]");
  CCMPC_REQUIRE(n_cells >= 0 && n_cells < 65536, "bad n_cells");
  CCMPC_REQUIRE(n_samples >= 2 && n_samples < (int64_t(1) << 32), "bad n_samples");
  if (n_cells == 0) return CCMPC_OK;
  CCMPC_REQUIRE(prev_mean && prev_cov && out_mean && out_cov, "null pointer");
  const size_t need = ccmpc_ideal_moments_workspace_bytes(T, n_cells, n_samples);
  if (workspace_bytes < need || !workspace) {
    set_error("ccmpc_ideal_moments: workspace too small");
    return CCMPC_ERR_WORKSPACE;
  }
  const int64_t chunk = ideal_chunk(n_cells, n_samples);
  const int64_t items = ((n_samples + chunk - 1) / chunk) * n_cells;
  const int rb = row_blocks(T);
  double *partial = static_cast<double *>(workspace);
  double *shift = partial + items * slab_doubles(rb);
  hipStream_t s = as_stream(stream);
  const int nc = static_cast<int>(n_cells), Ti = static_cast<int>(T), Ts = static_cast<int>(T_src);
  switch (rb) {
    case 1: launch_ideal_gram<1>(prev_mean, prev_cov, Ts, src_cell, nc, Ti, n_samples, x0, seed, rng_cell, partial, shift, out_mean, out_cov, out_status, s); break;
    case 2: launch_ideal_gram<2>(prev_mean, prev_cov, Ts, src_cell, nc, Ti, n_samples, x0, seed, rng_cell, partial, shift, out_mean, out_cov, out_status, s); break;
    case 3: launch_ideal_gram<3>(prev_mean, prev_cov, Ts, src_cell, nc, Ti, n_samples, x0, seed, rng_cell, partial, shift, out_mean, out_cov, out_status, s); break;
    case 4: launch_ideal_gram<4>(prev_mean, prev_cov, Ts, src_cell, nc, Ti, n_samples, x0, seed, rng_cell, partial, shift, out_mean, out_cov, out_status, s); break;
    case 5: launch_ideal_gram<5>(prev_mean, prev_cov, Ts, src_cell, nc, Ti, n_samples, x0, seed, rng_cell, partial, shift, out_mean, out_cov, out_status, s); break;
    default: set_error("ccmpc_ideal_moments: unsupported T"); return CCMPC_ERR_UNSUPPORTED;
  }
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}
