// Bucketing pieces shared by the three-kernel bucketing (bucket.hip) and the fused sampler +
// bucketing kernel (sample_bucket.hip), so that both produce bit-identical cells.
#pragma once
#include "gram.hpp"

namespace ccmpc {

constexpr int kMaxBins = 1024;
constexpr int kMaxKept = 16;
constexpr int kCentreGroup = 64;  // particles per centre partial (one wave, sample order)
constexpr int kCentreSuper = 64;  // partials per sequential superblock (a multiple of 16)
static_assert(kCentreSuper % 16 == 0, "superblock_sum / lds_row_sum read rounds of 16");

// Sum of v over the 64 lanes of a wave (xor butterfly 32, 16, ..., 1: every lane ends with the
// same value, since each step adds the same two operands on both partners).
__device__ __forceinline__ double group_sum64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// The canonical centre of kept mode k (v8ideal/__init__.py:477-482 take the mean final position
// of the mode's own particles; this fixes the summation order so that any kernel shape gives the
// same bits):
//   P_g  = group_sum64 over particles 64 g .. 64 g + 63 (lane = particle, non-members add 0.0)
//   S_j  = 0.0 + P_{64 j} + P_{64 j + 1} + ... (left to right over the superblock's partials)
//   sum  = 0.0 + S_0 + S_1 + ...               (left to right)
//   centre = sum / n_k
// superblock_sum(j, G, load) evaluates S_j for partials load(g, true), g < G; load(g, false)
// must return -0.0 (an LDS sentinel slot: the address is selected, not the value), the exact
// identity of IEEE addition (x + -0.0 == x for every x, -0.0 included).  So the chain is one add
// per partial, and all sixteen reads of a round land in registers of their own before the first
// add (a predicated add put four selects on the dependent path, and a select of the loaded value
// let the compiler recycle the landing registers, two reads in flight: ~2.3 us of the rare
// placement at G = 79).
template <typename Load>
__device__ __forceinline__ double2 superblock_sum(int j, int G, Load load) {
  const int g0 = j * kCentreSuper, g1 = min(G, g0 + kCentreSuper);
  double2 acc = {0.0, 0.0};
  for (int g = g0; g < g1; g += 16) {
    double2 v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = load(g + q, g + q < g1);
    __builtin_amdgcn_sched_barrier(0);  // every read issued before the first add waits
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      acc.x += v[q].x;
      acc.y += v[q].y;
    }
  }
  return acc;
}

// acc + row[0] + row[1] + ... + row[n - 1], left to right, as the chain of superblock_sum; the
// row holds kCentreSuper slots, those past n set to -0.0 by the caller.
__device__ __forceinline__ void lds_row_sum(double2 &acc, const double2 *row, int n) {
  for (int q0 = 0; q0 < n; q0 += 16) {
    double2 v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = row[q0 + q];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      acc.x += v[q].x;
      acc.y += v[q].y;
    }
  }
}

// Bucket key of a particle (see bucket.hip): kept mode k's own particle -> k (L + 1); a rare
// latent zv -> owner (L + 1) + 1 + zv, owner = argmin_k ||final - centre_k|| (first minimum,
// scipy.spatial.distance_matrix + np.argmin).  keep_s and the centres are LDS copies.
__device__ __forceinline__ int key_staged(int zv, double x, double y, const int *keep_s,
                                          const double (*cen_s)[2], int K, int L) {
  const int k = keep_s[zv];
  if (k >= 0) return k * (L + 1);
  int best = 0;
  double bd = INFINITY;
  for (int j = 0; j < K; ++j) {
    const double dx = x - cen_s[j][0], dy = y - cen_s[j][1];
    const double d = sqrt(dx * dx + dy * dy);
    if (d < bd) {
      bd = d;
      best = j;
    }
  }
  return best * (L + 1) + 1 + zv;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void *base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st1_sc1(__amdgpu_buffer_rsrc_t r, int byte_off, int32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32(static_cast<uint32_t>(v), r, byte_off, 0, 16);
}
__device__ __forceinline__ int32_t ld1_sc1(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return static_cast<int32_t>(__builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 16));
}
__device__ __forceinline__ void stf_sc1(__amdgpu_buffer_rsrc_t r, int byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, byte_off, 0, 16);
}
__device__ __forceinline__ float ldf_sc1(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 16));
}

}  // namespace ccmpc
