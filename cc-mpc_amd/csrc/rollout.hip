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
#include "constraints.hpp"
#include "gram.hpp"

// ideal_gram_kernel's work items per launch (all cells): 512 keeps a 1- or 2-cell launch to one
// round of workgroups (tools/time_ideal.py: T = 1 41 -> 33 us, T = 4 68 -> 62 us against 1024)
#ifndef CCMPC_IDEAL_ITEMS
#define CCMPC_IDEAL_ITEMS 512
#endif
// size the plan / lower-bound tables for the instance's horizon (T <= 8 RB) instead of kMaxT:
// at RB = 1 the kernel's LDS drops from 54 to 47 KB, three workgroups per CU instead of two
#ifndef CCMPC_IDEAL_LDS_SHRINK
#define CCMPC_IDEAL_LDS_SHRINK 1
#endif

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

#ifndef CCMPC_IDEAL_WAVES1
#define CCMPC_IDEAL_WAVES1 4
#endif
__host__ __device__ constexpr int ideal_waves(int rb) {
  return rb == 1 ? CCMPC_IDEAL_WAVES1 : rb <= 2 ? 4 : 2;
}

template <int RB, bool MINK>
__global__ __launch_bounds__(64 * ideal_waves(RB)) void ideal_gram_kernel(
    const double *__restrict__ prev_mean, const double *__restrict__ prev_cov, int T_src,
    const int32_t *__restrict__ src_cell, int T, int64_t n, int64_t chunk, int64_t items_per_cell,
    const double *__restrict__ x0, uint64_t seed_arg, const uint64_t *__restrict__ seed_dev,
    const int32_t *__restrict__ rng_cell, TreeLayout tree, double *__restrict__ out_mean,
    double *__restrict__ out_cov, int32_t *__restrict__ out_status, MinkParams mp) {
  // seed_dev: the Philox seed from device memory (a graph replays with a fresh seed per frame)
  const uint64_t seed = seed_dev ? *seed_dev : seed_arg;
  constexpr int NT = n_tiles(RB);
  constexpr int D = 16 * RB;
  constexpr int E = slab_doubles(RB);
  constexpr int NW = ideal_waves(RB);
#if CCMPC_IDEAL_LDS_SHRINK
  __shared__ StepPlan plan[8 * RB];
#else
  __shared__ StepPlan plan[40];
#endif
  __shared__ double stage_all[NW * D * kStageStride];
  __shared__ double xch[combine_xch_doubles(RB, NW)];
  __shared__ double shift_s[D];
  __shared__ double S_lds[D];
  __shared__ double mean_lds[D];
#if CCMPC_IDEAL_LDS_SHRINK
  __shared__ double lb_s[MINK ? (8 * RB) * (8 * RB - 1) / 2 : 1];
#else
  __shared__ double lb_s[MINK ? 40 * 39 / 2 : 1];
#endif
  __shared__ int status_s;
  __shared__ int flag;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  double *stage = stage_all + w * D * kStageStride;
  const int64_t item = blockIdx.x;
  const int cell = static_cast<int>(item / items_per_cell);
  const int64_t cidx = item % items_per_cell;
  const int rows = 2 * T, rows_src = 2 * T_src;
  const int src = src_cell ? src_cell[cell] : cell;
  const double *mu = prev_mean + static_cast<int64_t>(src) * rows_src;
  const double *cv = prev_cov + static_cast<int64_t>(src) * rows_src * rows_src;
  const uint32_t rng = rng_cell ? static_cast<uint32_t>(rng_cell[cell]) : static_cast<uint32_t>(cell);
  if (threadIdx.x == 0) status_s = 0;
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += blockDim.x) {
    const int st = build_step(mu, cv, rows_src, t, plan[t]);
    if (st) atomicMin(&status_s, st);
  }
  __syncthreads();
  double x0x, x0y;
  {
    int st = 0;
    initial_draw(mu, cv, rows_src, x0, cell, rng, seed, x0x, x0y, st);
    if (st && threadIdx.x == 0) atomicMin(&status_s, st);
  }
  // shift = the noise-free path (the rollout's exact mean given x0): same for every item
  if (threadIdx.x == 0) {
    double x = x0x, y = x0y;
    for (int t = 0; t < T; ++t) {
      advance(plan[t], 0.0, 0.0, x, y);
      shift_s[2 * t] = x;
      shift_s[2 * t + 1] = y;
    }
    for (int R = rows; R < D; ++R) shift_s[R] = 0.0;
  }
  __syncthreads();
  if (cidx == 0 && threadIdx.x == 0 && out_status) out_status[cell] = status_s;

  d4 acc[1][NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[0][t] = d4{0.0, 0.0, 0.0, 0.0};
  double s1[RB];
#pragma unroll
  for (int b = 0; b < RB; ++b) s1[b] = 0.0;
  const int r = lane & 15, g = lane >> 4;
  const int64_t wq = chunk / NW;  // samples per wave (multiple of 64)
  const int64_t i0 = cidx * chunk;
  const int64_t i1 = (i0 + chunk < n) ? i0 + chunk : n;
  const int64_t p0 = i0 + w * wq;
  const int64_t p1 = (p0 + wq < i1) ? p0 + wq : i1;

  // the trip count differs between waves only at the tail: keep barriers wave-local
  for (int64_t base = p0; base < p1; base += 64) {
    const int64_t i = base + lane;
    const bool valid = i < p1;
    double x = x0x, y = x0y;
    auto put = [&](int t) {
      stage[(2 * t) * kStageStride + lane] = valid ? x - shift_s[2 * t] : 0.0;
      stage[(2 * t + 1) * kStageStride + lane] = valid ? y - shift_s[2 * t + 1] : 0.0;
    };
    for (int t = 0; t < T; ++t) {
      double z0, z1;
      normal_pair(static_cast<uint32_t>(i), static_cast<uint32_t>(t), rng, STREAM_IDEAL_Z, seed, z0,
                  z1);
      advance(plan[t], z0, z1, x, y);
      put(t);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
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
          acc[0][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(v[bi], v[bj], acc[0][t], 0, 0, 0);
          ++t;
        }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // reads done before the next batch overwrites
    __builtin_amdgcn_wave_barrier();
  }

  combine_waves<RB, 1, NW>(acc, s1, xch, tree.slabs[0] + item * E, false);
  const double *root;
  int32_t root_n;
  if (!tree_climb<E>(tree, static_cast<int32_t>(cidx), static_cast<int32_t>(items_per_cell),
                     static_cast<int32_t>(cell * items_per_cell), cell, &flag, &root, &root_n))
    return;
  double *mean = out_mean + static_cast<int64_t>(cell) * rows;
  double *cov = out_cov + static_cast<int64_t>(cell) * rows * rows;
  static_assert(NW * D * kStageStride >= E, "root staging reuses the sample stage");
  gather_root<E>(root, root_n, stage_all);  // the sample stage is free after combine_waves
  finalize_cell<Scheme16<RB>>([&](int e) { return double2{stage_all[e], stage_all[e + 1]}; }, n, T,
                    shift_s, S_lds, 0.0, 0.0, mean, cov, mean_lds, nullptr);
  if (MINK) minkowski_cell(cov, mean_lds, T, cell, mp, lb_s, threadIdx.x, blockDim.x);
}

// samples per work item (multiple of 256 = 4 waves x 64): ~CCMPC_IDEAL_ITEMS items per launch
inline int64_t ideal_chunk(int64_t n_cells, int64_t n) {
  int64_t c = (n_cells * n + CCMPC_IDEAL_ITEMS - 1) / CCMPC_IDEAL_ITEMS;
  constexpr int64_t q = 64 * (CCMPC_IDEAL_WAVES1 > 4 ? CCMPC_IDEAL_WAVES1 : 4);
  c = ((c + q - 1) / q) * q;
  if (c < q) c = q;
  if (c > 16384) c = 16384;
  return c;
}

template <int RB, bool MINK>
static int launch_ideal_gram(const double *pm, const double *pc, int T_src, const int32_t *src,
                             int n_cells, int T, int64_t n, const double *x0, uint64_t seed,
                             const uint64_t *seed_dev, const int32_t *rng, void *ws,
                             size_t ws_bytes, double *out_mean,
                             double *out_cov, int32_t *status, const MinkParams &mp,
                             hipStream_t s) {
  const int64_t chunk = ideal_chunk(n_cells, n);
  const int64_t ipc = (n + chunk - 1) / chunk;
  TreeLayout tree;
  if (!tree_layout(ws, ws_bytes, ipc * n_cells, n_cells, slab_doubles(RB), tree))
    return CCMPC_ERR_WORKSPACE;
  hipLaunchKernelGGL((ideal_gram_kernel<RB, MINK>), dim3(static_cast<unsigned>(ipc * n_cells)),
                     dim3(64 * ideal_waves(RB)), 0, s, pm, pc, T_src, src, T, n, chunk, ipc, x0,
                     seed, seed_dev, rng, tree, out_mean, out_cov, status, mp);
  return CCMPC_OK;
}

template <bool MINK>
static int run_ideal(const double *prev_mean, const double *prev_cov, int64_t T_src,
                     const int32_t *src_cell, int64_t n_cells, int64_t T, int64_t n_samples,
                     const double *x0, uint64_t seed, const uint64_t *seed_dev,
                     const int32_t *rng_cell, void *workspace, size_t ws_bytes,
                     double *out_mean, double *out_cov, int32_t *out_status,
                     const MinkParams &mp, ccmpc_stream_t stream) {
  hipStream_t s = as_stream(stream);
  const int nc = static_cast<int>(n_cells), Ti = static_cast<int>(T), Ts = static_cast<int>(T_src);
#define IDEAL_ARGS                                                                            \
  prev_mean, prev_cov, Ts, src_cell, nc, Ti, n_samples, x0, seed, seed_dev, rng_cell, workspace, \
      ws_bytes, out_mean, out_cov, out_status, mp, s
  int rc;
  switch (row_blocks(T)) {
    case 1: rc = launch_ideal_gram<1, MINK>(IDEAL_ARGS); break;
    case 2: rc = launch_ideal_gram<2, MINK>(IDEAL_ARGS); break;
    case 3: rc = launch_ideal_gram<3, MINK>(IDEAL_ARGS); break;
    case 4: rc = launch_ideal_gram<4, MINK>(IDEAL_ARGS); break;
    case 5: rc = launch_ideal_gram<5, MINK>(IDEAL_ARGS); break;
    default: set_error("ideal moments: unsupported T"); return CCMPC_ERR_UNSUPPORTED;
  }
#undef IDEAL_ARGS
  if (rc != CCMPC_OK) {
    set_error("ideal moments: workspace too small");
    return rc;
  }
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
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
  return tree_bytes(items, n_cells, slab_doubles(row_blocks(T)));
}

#define CHECK_IDEAL_ARGS()                                                                     \
  CCMPC_REQUIRE(T_src >= 2 && T_src <= kMaxT, "T_src must be in [2, 40]");                     \
  CCMPC_REQUIRE(T >= 1 && T <= T_src - 1, "T must be in [1, T_src - 1]");                      \
  CCMPC_REQUIRE(n_cells >= 0 && n_cells < 65536, "bad n_cells");                               \
  CCMPC_REQUIRE(n_samples >= 2 && n_samples < (int64_t(1) << 32), "bad n_samples");            \
  if (n_cells == 0) return CCMPC_OK;                                                           \
  CCMPC_REQUIRE(prev_mean && prev_cov && out_mean && out_cov, "null pointer");                 \
  CCMPC_REQUIRE(workspace && aligned(workspace, 16), "workspace must be 16-byte aligned");     \
  if (workspace_bytes < ccmpc_ideal_moments_workspace_bytes(T, n_cells, n_samples)) {          \
    set_error(std::string(__func__) + ": workspace too small");                                \
    return CCMPC_ERR_WORKSPACE;                                                                \
  }

extern "C" int ccmpc_ideal_moments(const double *prev_mean, const double *prev_cov,
                                   int64_t T_src, const int32_t *src_cell, int64_t n_cells,
                                   int64_t T, int64_t n_samples, const double *x0, uint64_t seed,
                                   const int32_t *rng_cell, void *workspace,
                                   size_t workspace_bytes, double *out_mean, double *out_cov,
                                   int32_t *out_status, ccmpc_stream_t stream) {
  CHECK_IDEAL_ARGS();
  const MinkParams none{};
  return run_ideal<false>(prev_mean, prev_cov, T_src, src_cell, n_cells, T, n_samples, x0, seed,
                          nullptr, rng_cell, workspace, workspace_bytes, out_mean, out_cov,
                          out_status, none, stream);
}

extern "C" int ccmpc_ideal_minkowski_cycle_ex(
    const double *prev_mean, const double *prev_cov, int64_t T_src, const int32_t *src_cell,
    int64_t n_cells, int64_t T, int64_t n_samples, const double *x0, uint64_t seed,
    const uint64_t *seed_dev, const int32_t *rng_cell, void *workspace, size_t workspace_bytes,
    const double *ref_traj, const int32_t *cell_ref, const double *cell_risk, double R,
    double tol, int32_t maxiter, double *out_mean, double *out_cov, int32_t *out_status,
    ccmpc_halfspace *out_rec, double *out_prob_lower, ccmpc_stream_t stream) {
  CHECK_IDEAL_ARGS();
  CCMPC_REQUIRE(ref_traj && cell_risk && out_rec && out_prob_lower, "null pointer");
  CCMPC_REQUIRE(maxiter >= 1, "maxiter must be >= 1");
  const MinkParams mp{ref_traj, cell_ref, cell_risk, R, tol, maxiter, out_rec, out_prob_lower};
  return run_ideal<true>(prev_mean, prev_cov, T_src, src_cell, n_cells, T, n_samples, x0, seed,
                         seed_dev, rng_cell, workspace, workspace_bytes, out_mean, out_cov,
                         out_status, mp, stream);
}

extern "C" int ccmpc_ideal_minkowski_cycle(
    const double *prev_mean, const double *prev_cov, int64_t T_src, const int32_t *src_cell,
    int64_t n_cells, int64_t T, int64_t n_samples, const double *x0, uint64_t seed,
    const int32_t *rng_cell, void *workspace, size_t workspace_bytes, const double *ref_traj,
    const int32_t *cell_ref, const double *cell_risk, double R, double tol, int32_t maxiter,
    double *out_mean, double *out_cov, int32_t *out_status, ccmpc_halfspace *out_rec,
    double *out_prob_lower, ccmpc_stream_t stream) {
  return ccmpc_ideal_minkowski_cycle_ex(prev_mean, prev_cov, T_src, src_cell, n_cells, T,
                                        n_samples, x0, seed, nullptr, rng_cell, workspace,
                                        workspace_bytes, ref_traj, cell_ref, cell_risk, R, tol,
                                        maxiter, out_mean, out_cov, out_status, out_rec,
                                        out_prob_lower, stream);
}
