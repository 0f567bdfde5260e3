// Segmented moment (Gram) reduction of particle clouds -- the dominant kernel of the path.
//
// Replaces every np.mean / np.cov the reference runs over particle clouds
// (v8ideal/__init__.py:864-875, :896, :907 -> makeconstraint.py:41-70, :1485-1493,
// :2584-2606).  The reference calls np.cov once per (t, tau) pair on a strided 4xN gather;
// every one of those 4x4 matrices is a block of ONE 2T x 2T covariance per cell, so the
// particle cloud is read exactly once.
//
// Design (gfx950):
//  * Work item = (cell, chunk of `chunk` particles), one wavefront per workgroup.
//  * The Gram matrix G = X X^T of the shifted data X[r][p] = pos[r][p] - pos[r][first]
//    (r = 2t + xy) runs on the f64 matrix core: v_mfma_f64_16x16x4_f64 takes A[i][k] from lane
//    (i + 16k) and B[k][j] from lane (j + 16k), so a lane holding X[16b + (lane&15)][p_k]
//    feeds BOTH operands; tile (bi, bj) of G accumulates with no data movement.  The 2T(2T+1)/2
//    fp64 accumulators live spread over 64 lanes (4 doubles per lane per 16x16 tile), instead of
//    in every lane's registers as a VALU version would need.
//  * Each lane loads 4 consecutive particles of its row (two 16-byte loads), so a row of a
//    16-particle step is one 128-byte line.  Sub-step j feeds particle p = base + 4k + j to
//    group k -- summation order is irrelevant for a Gram sum.
//  * Shift by the cell's first particle (shifted one-pass formula): positions sit around
//    x ~ 200 m with sub-metre spread, and the un-shifted one-pass form loses every digit.
//  * Partial slabs per item are summed in a fixed order by the finalize kernel (bitwise
//    reproducible; no float atomics).
#include "gram.hpp"

namespace ccmpc {

template <typename P, int RB>
__global__ __launch_bounds__(64) void gram_partial_kernel(
    const P *__restrict__ pos, int64_t ld, int T, const int64_t *__restrict__ cell_off,
    const int64_t *__restrict__ cell_cnt, int n_cells, int64_t chunk,
    double *__restrict__ partial) {
  constexpr int NT = n_tiles(RB);
  constexpr int NACC = (NT == 1) ? 2 : 1;  // two chains hide MFMA latency when there is one tile
  int cell;
  int64_t cidx;
  const int64_t item = blockIdx.x;
  if (!locate_item(item, cell_cnt, n_cells, chunk, cell, cidx)) return;

  const int lane = threadIdx.x;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int rows = 2 * T;
  const int64_t off = cell_off[cell];
  const int64_t cnt = cell_cnt[cell];
  const int64_t p0 = cidx * chunk;
  const int64_t p1 = (p0 + chunk < cnt) ? p0 + chunk : cnt;

  double sh[RB];
  const P *rowp[RB];
  bool live[RB];
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    const int R = 16 * b + r;
    live[b] = R < rows;
    rowp[b] = pos + static_cast<int64_t>(live[b] ? R : 0) * ld + off;
    sh[b] = live[b] ? static_cast<double>(rowp[b][0]) : 0.0;
  }

  d4 acc[NACC][NT];
#pragma unroll
  for (int a = 0; a < NACC; ++a)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[a][t] = d4{0.0, 0.0, 0.0, 0.0};
  double s1[RB];
#pragma unroll
  for (int b = 0; b < RB; ++b) s1[b] = 0.0;

  for (int64_t base = p0; base < p1; base += 16) {
    const int64_t q = base + 4 * g;
    double v[RB][4];
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      if (live[b] && q + 3 < p1) {
        load4<P>(rowp[b] + q, v[b]);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[b][j] -= sh[b];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[b][j] = (live[b] && q + j < p1) ? static_cast<double>(rowp[b][q + j]) - sh[b] : 0.0;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int a = (NACC == 2) ? (j & 1) : 0;
      int t = 0;
#pragma unroll
      for (int bi = 0; bi < RB; ++bi)
#pragma unroll
        for (int bj = bi; bj < RB; ++bj) {
          acc[a][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(v[bi][j], v[bj][j], acc[a][t], 0, 0, 0);
          ++t;
        }
    }
#pragma unroll
    for (int b = 0; b < RB; ++b) s1[b] += (v[b][0] + v[b][1]) + (v[b][2] + v[b][3]);
  }

  double *slab = partial + item * slab_doubles(RB);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    d4 s = acc[0][t];
    if (NACC == 2) s += acc[NACC - 1][t];
#pragma unroll
    for (int k = 0; k < 4; ++k) slab[t * 256 + k * 64 + lane] = s[k];
  }
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    double x = s1[b];
    x += __shfl_xor(x, 16, 64);
    x += __shfl_xor(x, 32, 64);
    if (lane < 16) slab[NT * 256 + b * 16 + lane] = x;
  }
}

template <typename P, int RB>
static void launch_moments(const P *pos, int64_t ld, int T, const double *origin,
                           const int64_t *off, const int64_t *cnt, int n_cells, int64_t chunk,
                           int64_t items, double *partial, double *mean, double *cov,
                           hipStream_t s) {
  hipLaunchKernelGGL((gram_partial_kernel<P, RB>), dim3(static_cast<unsigned>(items)), dim3(64),
                     0, s, pos, ld, T, off, cnt, n_cells, chunk, partial);
  hipLaunchKernelGGL((gram_finalize_kernel<P, RB>), dim3(n_cells), dim3(256), 0, s, pos, ld, T,
                     static_cast<const double *>(nullptr), origin, off, cnt, int64_t(0), chunk,
                     partial, mean, cov);
}

template <typename P>
static int dispatch_moments(const P *pos, int64_t ld, int T, const double *origin,
                            const int64_t *off, const int64_t *cnt, int n_cells, int64_t chunk,
                            int64_t items, double *partial, double *mean, double *cov,
                            hipStream_t s) {
  switch (row_blocks(T)) {
    case 1: launch_moments<P, 1>(pos, ld, T, origin, off, cnt, n_cells, chunk, items, partial, mean, cov, s); break;
    case 2: launch_moments<P, 2>(pos, ld, T, origin, off, cnt, n_cells, chunk, items, partial, mean, cov, s); break;
    case 3: launch_moments<P, 3>(pos, ld, T, origin, off, cnt, n_cells, chunk, items, partial, mean, cov, s); break;
    case 4: launch_moments<P, 4>(pos, ld, T, origin, off, cnt, n_cells, chunk, items, partial, mean, cov, s); break;
    case 5: launch_moments<P, 5>(pos, ld, T, origin, off, cnt, n_cells, chunk, items, partial, mean, cov, s); break;
    default: return CCMPC_ERR_UNSUPPORTED;
  }
  return CCMPC_OK;
}

}  // namespace ccmpc

using namespace ccmpc;

extern "C" size_t ccmpc_moments_workspace_bytes(int64_t T, int64_t n_cells,
                                                int64_t n_particles_bound) {
  if (T < 1 || T > kMaxT || n_cells < 0 || n_particles_bound < 0) return 0;
  const int64_t chunk = pick_chunk(T, n_particles_bound);
  const int64_t items = max_items(n_cells, n_particles_bound, chunk);
  return static_cast<size_t>(items) * slab_doubles(row_blocks(T)) * sizeof(double);
}

extern "C" int ccmpc_moments(const void *positions, int dtype, int64_t ld, int64_t T,
                             const double *origin, const int64_t *cell_off,
                             const int64_t *cell_cnt, int64_t n_cells,
                             int64_t n_particles_bound, void *workspace, size_t workspace_bytes,
                             double *out_mean, double *out_cov, ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T >= 1 && T <= kMaxT, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_cells >= 0 && n_cells < (1 << 30), "bad n_cells");
  if (n_cells == 0) return CCMPC_OK;
  CCMPC_REQUIRE(positions && cell_off && cell_cnt && out_mean && out_cov, "null pointer");
  CCMPC_REQUIRE(ld % 4 == 0 && ld > 0, "ld must be a positive multiple of 4");
  CCMPC_REQUIRE(dtype == CCMPC_F64 || dtype == CCMPC_F32, "dtype must be CCMPC_F64 or CCMPC_F32");
  CCMPC_REQUIRE(aligned(positions, 16), "positions must be 16-byte aligned");
  const size_t need = ccmpc_moments_workspace_bytes(T, n_cells, n_particles_bound);
  if (workspace_bytes < need || (need && !workspace)) {
    set_error("ccmpc_moments: workspace too small");
    return CCMPC_ERR_WORKSPACE;
  }
  const int64_t chunk = pick_chunk(T, n_particles_bound);
  const int64_t items = max_items(n_cells, n_particles_bound, chunk);
  hipStream_t s = as_stream(stream);
  int rc;
  if (dtype == CCMPC_F64)
    rc = dispatch_moments<double>(static_cast<const double *>(positions), ld, static_cast<int>(T),
                                  origin, cell_off, cell_cnt, static_cast<int>(n_cells), chunk,
                                  items, static_cast<double *>(workspace), out_mean, out_cov, s);
  else
    rc = dispatch_moments<float>(static_cast<const float *>(positions), ld, static_cast<int>(T),
                                 origin, cell_off, cell_cnt, static_cast<int>(n_cells), chunk,
                                 items, static_cast<double *>(workspace), out_mean, out_cov, s);
  if (rc != CCMPC_OK) {
    set_error("ccmpc_moments: unsupported T");
    return rc;
  }
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}
