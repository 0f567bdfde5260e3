// Shared pieces of the segmented Gram reduction (moments.hip, rollout.hip).
// Slab layout per work item: NT = RB(RB+1)/2 tiles of the f64 16x16x4 MFMA C layout
// (entry (tile, reg, lane) <-> row (lane>>4) + 4 reg, col lane&15 of tile (bi, bj)), then
// RB*16 shifted row sums.
#pragma once
#include "ccmpc_common.hpp"

namespace ccmpc {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kMaxT = 40;

__host__ __device__ constexpr int n_tiles(int rb) { return rb * (rb + 1) / 2; }
__host__ __device__ constexpr int slab_doubles(int rb) { return n_tiles(rb) * 256 + rb * 16; }

inline int row_blocks(int64_t T) { return static_cast<int>((2 * T + 15) / 16); }

// particles per work item: enough items to cover the chip, not so small that the partial
// slab (>= 2 KiB) dominates the bytes read
inline int64_t pick_chunk(int64_t T, int64_t n_bound) {
  int64_t target_items = 2048;
  int64_t c = (n_bound + target_items - 1) / target_items;
  c = ((c + 15) / 16) * 16;
  const int64_t min_c = (T > 16) ? 128 : 64;
  if (c < min_c) c = min_c;
  if (c > 8192) c = 8192;
  return c;
}

inline int64_t max_items(int64_t n_cells, int64_t n_bound, int64_t chunk) {
  return (n_bound + chunk - 1) / chunk + n_cells;
}

// Item id -> (cell, chunk index), wave-parallel scan over ceil(cnt/chunk).  Returns false for
// ids past the last item (the grid is sized by an upper bound).
__device__ __forceinline__ bool locate_item(int64_t item, const int64_t *__restrict__ cnt,
                                            int n_cells, int64_t chunk, int &cell,
                                            int64_t &chunk_idx) {
  const int lane = threadIdx.x & 63;
  int64_t before = 0;
  for (int base = 0; base < n_cells; base += 64) {
    const int c = base + lane;
    const int64_t n = (c < n_cells) ? cnt[c] : 0;
    const int64_t my = n > 0 ? (n + chunk - 1) / chunk : 0;
    int64_t incl = my;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    const int64_t total = __shfl(incl, 63, 64);
    if (item < before + total) {
      const unsigned long long m = __ballot(before + incl > item);
      const int l = __ffsll(static_cast<long long>(m)) - 1;
      const int64_t excl = __shfl(incl - my, l, 64);
      cell = base + l;
      chunk_idx = item - before - excl;
      return true;
    }
    before += total;
  }
  return false;
}

// first item of `cell` (same enumeration as locate_item)
__device__ __forceinline__ int64_t first_item(int cell, const int64_t *__restrict__ cnt,
                                              int64_t chunk) {
  int64_t s = 0;
  for (int c = 0; c < cell; ++c) {
    const int64_t n = cnt[c];
    s += n > 0 ? (n + chunk - 1) / chunk : 0;
  }
  return s;
}

template <typename P>
__device__ __forceinline__ void load4(const P *__restrict__ p, double (&v)[4]);

template <>
__device__ __forceinline__ void load4<double>(const double *__restrict__ p, double (&v)[4]) {
  const double2 a = *reinterpret_cast<const double2 *>(p);
  const double2 b = *reinterpret_cast<const double2 *>(p + 2);
  v[0] = a.x;
  v[1] = a.y;
  v[2] = b.x;
  v[3] = b.y;
}

template <>
__device__ __forceinline__ void load4<float>(const float *__restrict__ p, double (&v)[4]) {
  const float4 a = *reinterpret_cast<const float4 *>(p);
  v[0] = a.x;
  v[1] = a.y;
  v[2] = a.z;
  v[3] = a.w;
}

// One workgroup per cell: sum the cell's slabs in item order, then cov = (G - S S^T / n)/(n-1).
template <typename P, int RB>
__global__ __launch_bounds__(256) void gram_finalize_kernel(
    const P *__restrict__ pos, int64_t ld, int T, const double *__restrict__ shift_buf,
    const double *__restrict__ origin,
    const int64_t *__restrict__ cell_off, const int64_t *__restrict__ cell_cnt,
    int64_t uniform_cnt, int64_t chunk, const double *__restrict__ partial,
    double *__restrict__ out_mean, double *__restrict__ out_cov) {
  constexpr int NT = n_tiles(RB);
  constexpr int E = slab_doubles(RB);
  constexpr int D = 16 * RB;
  __shared__ double G[D][D + 1];
  __shared__ double S[D];
  __shared__ double shift[D];
  const int cell = blockIdx.x;
  // cell_cnt == NULL: every cell holds uniform_cnt particles (fused ideal rollout)
  const int64_t cnt = cell_cnt ? cell_cnt[cell] : uniform_cnt;
  const int64_t nit = cnt > 0 ? (cnt + chunk - 1) / chunk : 0;
  const int64_t it0 = cell_cnt ? first_item(cell, cell_cnt, chunk) : cell * nit;
  const int rows = 2 * T;

  for (int e = threadIdx.x; e < E; e += blockDim.x) {
    double s = 0.0;
    for (int64_t i = 0; i < nit; ++i) s += partial[(it0 + i) * E + e];
    if (e < NT * 256) {
      // decode (tile, reg, lane) -> (row, col) of the f64 16x16x4 C layout
      const int tile = e >> 8, k = (e >> 6) & 3, l = e & 63;
      const int row = (l >> 4) + 4 * k, col = l & 15;
      int bi = 0, t = tile;
      while (t >= RB - bi) {
        t -= RB - bi;
        ++bi;
      }
      const int bj = bi + t;
      G[16 * bi + row][16 * bj + col] = s;
      if (bi != bj) G[16 * bj + col][16 * bi + row] = s;
    } else {
      S[e - NT * 256] = s;
    }
  }
  const int64_t off = cell_off ? cell_off[cell] : 0;
  for (int R = threadIdx.x; R < D; R += blockDim.x) {
    double v = 0.0;
    if (R < rows && cnt > 0)
      v = shift_buf ? shift_buf[static_cast<int64_t>(cell) * rows + R]
                    : static_cast<double>(pos[static_cast<int64_t>(R) * ld + off]);
    shift[R] = v;
  }
  __syncthreads();

  const double n = static_cast<double>(cnt);
  double *cov = out_cov + static_cast<int64_t>(cell) * rows * rows;
  for (int e = threadIdx.x; e < rows * rows; e += blockDim.x) {
    const int i = e / rows, j = e % rows;
    const int a = i < j ? i : j, b = i < j ? j : i;  // one value for both triangles
    cov[e] = (G[a][b] - S[a] * S[b] / n) / (n - 1.0);
  }
  double *mean = out_mean + static_cast<int64_t>(cell) * rows;
  for (int R = threadIdx.x; R < rows; R += blockDim.x) {
    const double o = origin ? origin[2 * cell + (R & 1)] : 0.0;
    mean[R] = (shift[R] + S[R] / n) + o;
  }
}

}  // namespace ccmpc
