// Segmented Gram reduction shared by moments.hip (particle stores) and rollout.hip (fused
// ideal rollout): MFMA accumulation, partial-slab publication and the in-launch per-cell
// combine by the last-arriving work item.
//
// Slab layout per work item: NT = RB(RB+1)/2 tiles of the f64 16x16x4 MFMA C layout
// (entry (tile, reg, lane) <-> row (lane>>4) + 4 reg, col lane&15 of tile (bi, bj)), then
// RB*16 shifted row sums.
//
// Cross-workgroup hand-off (MI355X_MICROARCH.md "Valid forms", first table row; guide §6 G16):
// every slab store is an agent-scope write-through (sc1) store, the wave drains with
// s_waitcnt vmcnt(0), then ONE lane adds to the cell's arrival counter (agent scope).  The item
// that draws ticket nit-1 is the reducer: it reads every slab of the cell with sc1 loads (no L1,
// so no acquire fence is needed) in a fixed item order -- bitwise reproducible, no float
// atomics -- and resets the counter to 0 for the next launch.
#pragma once
#include "ccmpc_common.hpp"

namespace ccmpc {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kMaxT = 40;
constexpr int kCounterAlign = 256;  // bytes reserved at the head of every workspace

__host__ __device__ constexpr int n_tiles(int rb) { return rb * (rb + 1) / 2; }
__host__ __device__ constexpr int slab_doubles(int rb) { return n_tiles(rb) * 256 + rb * 16; }

inline int row_blocks(int64_t T) { return static_cast<int>((2 * T + 15) / 16); }

inline size_t counter_bytes(int64_t n_cells) {
  const size_t b = static_cast<size_t>(n_cells) * sizeof(int32_t);
  return (b + kCounterAlign - 1) / kCounterAlign * kCounterAlign;
}

// particles per work item (one wavefront): ~8 items for a 2000-particle cell keeps the combine
// short; large inputs get >= 2048 items to fill 256 CUs
inline int64_t pick_chunk(int64_t n_bound) {
  int64_t c = (n_bound + 2047) / 2048;
  c = ((c + 63) / 64) * 64;
  if (c < 256) c = 256;
  if (c > 8192) c = 8192;
  return c;
}

inline int64_t max_items(int64_t n_cells, int64_t n_bound, int64_t chunk) {
  return (n_bound + chunk - 1) / chunk + n_cells;
}

// items of a cell: at least one, so an empty cell is still finalised (to NaN, as np.cov does)
__device__ __forceinline__ int64_t items_of(int64_t n, int64_t chunk) {
  return n > 0 ? (n + chunk - 1) / chunk : 1;
}

// Item id -> (cell, chunk index, first item of the cell), wave-parallel scan.
// False for ids past the last item (the grid is sized by an upper bound).
__device__ __forceinline__ bool locate_item(int64_t item, const int64_t *__restrict__ cnt,
                                            int n_cells, int64_t chunk, int &cell,
                                            int64_t &chunk_idx, int64_t &first) {
  const int lane = threadIdx.x & 63;
  int64_t before = 0;
  for (int base = 0; base < n_cells; base += 64) {
    const int c = base + lane;
    const int64_t my = (c < n_cells) ? items_of(cnt[c], chunk) : 0;
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
      first = before + excl;
      chunk_idx = item - first;
      return true;
    }
    before += total;
  }
  return false;
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

__device__ __forceinline__ void st_sc1(double *p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p),
                     static_cast<unsigned long long>(__double_as_longlong(v)), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double ld_sc1(const double *p) {
  return __longlong_as_double(static_cast<long long>(__hip_atomic_load(
      reinterpret_cast<const unsigned long long *>(p), __ATOMIC_RELAXED,
      __HIP_MEMORY_SCOPE_AGENT)));
}

// Write one item's accumulators (tiles + row sums) write-through.
template <int RB, int NACC>
__device__ __forceinline__ void publish_slab(double *slab, const d4 (&acc)[NACC][n_tiles(RB)],
                                             const double (&s1)[RB]) {
  constexpr int NT = n_tiles(RB);
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    d4 s = acc[0][t];
    if (NACC == 2) s += acc[NACC - 1][t];
#pragma unroll
    for (int k = 0; k < 4; ++k) st_sc1(slab + t * 256 + k * 64 + lane, s[k]);
  }
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    double x = s1[b];
    x += __shfl_xor(x, 16, 64);
    x += __shfl_xor(x, 32, 64);
    if (lane < 16) st_sc1(slab + NT * 256 + b * 16 + lane, x);
  }
}

// Drain this wave's slab stores, take a ticket; true for the last of `nit` arrivals (which
// also resets the counter for the next launch).  One-wave workgroups only.
__device__ __forceinline__ bool arrive_last(int32_t *counter, int64_t nit) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int ticket = 0;
  if ((threadIdx.x & 63) == 0)
    ticket = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ticket = __shfl(ticket, 0, 64);
  const bool last = static_cast<int64_t>(ticket) == nit - 1;
  if (last && (threadIdx.x & 63) == 0)
    __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep slab loads below the ticket
  return last;
}

// Sum entry e over the cell's nit slabs (sc1 loads, 4 independent chains, fixed order).
__device__ __forceinline__ double sum_items(const double *__restrict__ slab0, int64_t nit, int E,
                                            int e) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int64_t i = 0;
  for (; i + 4 <= nit; i += 4) {
    a0 += ld_sc1(slab0 + (i + 0) * E + e);
    a1 += ld_sc1(slab0 + (i + 1) * E + e);
    a2 += ld_sc1(slab0 + (i + 2) * E + e);
    a3 += ld_sc1(slab0 + (i + 3) * E + e);
  }
  for (; i < nit; ++i) a0 += ld_sc1(slab0 + i * E + e);
  return (a0 + a1) + (a2 + a3);
}

// The reducer: slabs of one cell -> mean[T][2] (+ origin) and cov[2T][2T] (ddof = 1),
// cov = (G - S S^T / n) / (n - 1) on data shifted by shift_lds (LDS, D entries).
// Uses S_lds (LDS, D entries) as scratch.  One wavefront; ends with a barrier so the caller can
// read mean/cov back.
template <int RB>
__device__ void reduce_cell(const double *__restrict__ slab0, int64_t nit, int64_t cnt, int T,
                            const double *shift_lds, double *S_lds, double o0, double o1,
                            double *__restrict__ mean, double *__restrict__ cov) {
  constexpr int NT = n_tiles(RB);
  constexpr int E = slab_doubles(RB);
  constexpr int D = 16 * RB;
  const int lane = threadIdx.x & 63;
  const int rows = 2 * T;
  const double n = static_cast<double>(cnt);
  for (int r = lane; r < D; r += 64)
    S_lds[r] = r < rows ? sum_items(slab0, nit, E, NT * 256 + r) : 0.0;
  __syncthreads();
  for (int r = lane; r < rows; r += 64)
    mean[r] = (shift_lds[r] + S_lds[r] / n) + ((r & 1) ? o1 : o0);
  for (int e = lane; e < NT * 256; e += 64) {
    const int tile = e >> 8, k = (e >> 6) & 3, l = e & 63;
    const int row = (l >> 4) + 4 * k, col = l & 15;
    int bi = 0, t = tile;
    while (t >= RB - bi) {
      t -= RB - bi;
      ++bi;
    }
    const int bj = bi + t;
    const int i = 16 * bi + row, j = 16 * bj + col;
    if (i >= rows || j >= rows || i > j) continue;  // one value per symmetric pair
    const double g = sum_items(slab0, nit, E, e);
    const double c = (g - S_lds[i] * S_lds[j] / n) / (n - 1.0);
    cov[i * rows + j] = c;
    cov[j * rows + i] = c;
  }
  __syncthreads();
}

}  // namespace ccmpc
