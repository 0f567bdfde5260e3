// Segmented Gram reduction shared by moments.hip (particle stores) and rollout.hip (fused
// ideal rollout): workgroup geometry, MFMA load groups, the cross-wave combine, the in-launch
// combine tree across workgroups, and the per-cell finalisation.
//
// Slab layout (one per work item / tree node): NT = RB(RB+1)/2 tiles of the f64 16x16x4 MFMA
// C layout, lane-major (entry t*256 + 4 lane + reg <-> row (lane>>4) + 4 reg, col lane&15 of
// tile (bi, bj)), then RB*16 shifted row sums; every access is a 16-byte pair.
//
// Cross-workgroup hand-off (MI355X_MICROARCH.md "Valid forms", first table row; guide §6 G16):
// every slab store is an agent-scope write-through (sc1) store, every storing wave drains with
// s_waitcnt vmcnt(0) before the workgroup barrier, then ONE lane adds to the group's arrival
// counter (agent scope).  The last arriver reads the slabs with sc1 loads (no L1 involved, so
// no acquire fence is needed) in a fixed order -- bitwise reproducible, no float atomics -- and
// resets the counter to 0 for the next launch.
#pragma once
#include "ccmpc_common.hpp"

namespace ccmpc {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kMaxT = 40;
constexpr int kCounterAlign = 256;

__host__ __device__ constexpr int n_tiles(int rb) { return rb * (rb + 1) / 2; }
__host__ __device__ constexpr int slab_doubles(int rb) { return n_tiles(rb) * 256 + rb * 16; }

inline int row_blocks(int64_t T) { return static_cast<int>((2 * T + 15) / 16); }

// ---- work-item geometry of the particle-store kernel ----------------------------------------
// One work item = one workgroup of NW waves; each wave owns WQ consecutive particles and loads
// S 16-particle steps per group, double-buffered, so ~2 groups of 16-byte loads are in flight.
// WQ is picked per launch: the f64 MFMA work of a small problem must be spread over many CUs
// (one CU's 4 matrix pipes need ~4 us for a 2000-particle T=8 cell), so latency-bound sizes
// use WQ = 64 (one load group per wave, one tree level); bandwidth-bound sizes use WQ = 256
// (fewer slabs, shallower tree).  A cell that fits one item never leaves its workgroup.
#ifndef CCMPC_LG_NW1  // log2 waves per work item at RB = 1 (T <= 8); build-time knob: 4-wave
#define CCMPC_LG_NW1 2  // items (256 particles) against 8-wave ones: C2 cycle 11.33 -> 10.78 us,
#endif                  // C3 np=1e3 -9.7 -> 9.1, np=2e4 / 1e5 +0.3 / +0.5 us (r06/ab/cycle_item_waves_*)
#ifndef CCMPC_LG_NW_BIG  // log2 waves per work item at RB >= 3 (T > 24); build-time knob
#define CCMPC_LG_NW_BIG 3
#endif
#ifndef CCMPC_MINW_BIG  // waves per SIMD the RB >= 3 register budget must allow; build knob
#define CCMPC_MINW_BIG 2
#endif
template <int RB>
struct Geo {
  static constexpr int NW = RB == 1 ? (1 << CCMPC_LG_NW1) : (RB <= 2 ? 4 : (1 << CCMPC_LG_NW_BIG));
  static constexpr int S = RB == 1 ? 4 : (RB == 2 ? 2 : 1);
  static constexpr int NACC = (n_tiles(RB) == 1) ? 2 : 1;  // 2 chains when there is one tile
  static constexpr int MIN_WAVES_PER_SIMD = RB == 1 ? 4 : (RB <= 2 ? 2 : CCMPC_MINW_BIG);
};

// log2 of the particles per wave.  Small inputs are latency-bound: 64 per wave spreads the
// MFMA work over many CUs.  Large inputs are bandwidth-bound: 256 per wave means fewer slabs
// and a shallower tree.  (64 at RB >= 3 balances the f64 matrix pipes better per wave but
// pays the per-workgroup combine ~3x more often: C5 went from 94 to 134 us.)
#ifndef CCMPC_LGWQ_SMALL  // build-time knobs (tools/build_variant.sh experiments)
#define CCMPC_LGWQ_SMALL 6
#endif
#ifndef CCMPC_LGWQ_MID
#define CCMPC_LGWQ_MID CCMPC_LGWQ_SMALL
#endif
#ifndef CCMPC_LGWQ_LARGE
#define CCMPC_LGWQ_LARGE 9
#endif
#ifndef CCMPC_LG_TINY_INPUT
#define CCMPC_LG_TINY_INPUT 15
#endif
#ifndef CCMPC_LG_SMALL_INPUT
#define CCMPC_LG_SMALL_INPUT 18
#endif
inline int store_lg_wave_quota(int /*rb*/, int64_t n_bound) {
#if CCMPC_PROBE & 8  // diagnostic build only: CCMPC_LG_WQ overrides the large-input quota
  static const int ov = [] { const char *e = getenv("CCMPC_LG_WQ"); return e ? atoi(e) : 0; }();
  if (ov && n_bound > (int64_t(1) << CCMPC_LG_SMALL_INPUT)) return ov;
#endif
  if (n_bound <= (int64_t(1) << CCMPC_LG_TINY_INPUT)) return CCMPC_LGWQ_SMALL;
  return n_bound <= (int64_t(1) << CCMPC_LG_SMALL_INPUT) ? CCMPC_LGWQ_MID : CCMPC_LGWQ_LARGE;
}

__host__ __device__ inline int lg_waves_per_item(int rb) {
  return rb == 1 ? CCMPC_LG_NW1 : (rb <= 2 ? 2 : CCMPC_LG_NW_BIG);
}

inline int store_lg_chunk(int rb, int64_t n_bound) {
  return lg_waves_per_item(rb) + store_lg_wave_quota(rb, n_bound);
}

inline int64_t max_items(int64_t n_cells, int64_t n_bound, int64_t chunk) {
  return (n_bound + chunk - 1) / chunk + n_cells;
}

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// items of a cell: at least one, so an empty cell is still finalised (to NaN, as np.cov does).
// Chunks are powers of two, so this is a shift (a 64-bit division by a runtime value costs
// ~100 instructions, and locate_item ran it per tree level).
__device__ __forceinline__ int32_t items_of(int64_t n, int lg_chunk) {
  return n > 0 ? static_cast<int32_t>((n + (int64_t(1) << lg_chunk) - 1) >> lg_chunk) : 1;
}
// With whole-cell items: a cell of <= whole particles is ONE item (its workgroup's waves deal
// its load groups round-robin), so its Gram is combined in LDS -- no slabs, no arrival, no
// root gather; larger cells are cut into chunk-sized items as before.  whole = 0: off.
__device__ __forceinline__ int32_t items_of(int64_t n, int lg_chunk, int64_t whole) {
  return n <= whole ? 1 : items_of(n, lg_chunk);
}

constexpr int kFanIn = 16;
constexpr int kLgFanIn = 4;
constexpr int kMaxLevels = 6;  // combine-tree depth bound: 16^6 items per cell

struct ItemLoc {
  int cell;
  int32_t ref_sel;  // cell_ref[cell] (0 when no table is given)
  int32_t chunk_idx;
  int32_t first;    // the cell's first item (= its first level-0 tree node)
  int64_t cnt, off;
};

// Wave-wide inclusive prefix sum of an int32 by DPP row shifts (rows of 16 lanes) and three
// readlanes of the row totals: register moves instead of __shfl_up's six dependent
// ds_bpermute round trips (~0.35 us of every launch's locate).  All 64 lanes must be active.
__device__ __forceinline__ int32_t wave_incl_scan_i32(int32_t x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  const int32_t r0 = __builtin_amdgcn_readlane(x, 15), r1 = __builtin_amdgcn_readlane(x, 31),
                r2 = __builtin_amdgcn_readlane(x, 47);
  const int row = (threadIdx.x & 63) >> 4;
  return x + (row >= 1 ? r0 : 0) + (row >= 2 ? r1 : 0) + (row >= 3 ? r2 : 0);
}
// Lane l's value (l wave-uniform): a scalar readlane instead of a ds_bpermute round trip.
__device__ __forceinline__ int32_t lane_i32(int32_t v, int l) {
  return __builtin_amdgcn_readlane(v, l);
}
__device__ __forceinline__ int64_t lane_i64(int64_t v, int l) {
  const int32_t lo = __builtin_amdgcn_readlane(static_cast<int32_t>(v), l);
  const int32_t hi = __builtin_amdgcn_readlane(static_cast<int32_t>(v >> 32), l);
  return static_cast<int64_t>((static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) |
                              static_cast<uint32_t>(lo));
}

// Item id -> (cell, chunk index, the cell's first item, count, offset, reference selector):
// one wave-parallel prefix scan of the cells' item counts in 32-bit arithmetic (items < 2^31:
// the grid is sized by them), so everything an item needs arrives with one memory round trip.
// The combine tree needs nothing more: its node numbering is closed-form in `first` (see
// tree_next_first).  False for ids past the last item (the grid is sized by an upper bound).
__device__ __forceinline__ bool locate_item(int32_t item, const int64_t *__restrict__ cnt,
                                            const int64_t *__restrict__ off, int n_cells,
                                            int lg_chunk, ItemLoc &loc,
                                            const int32_t *__restrict__ cell_ref = nullptr,
                                            int64_t whole = 0) {
  const int lane = threadIdx.x & 63;
  int32_t before = 0;
  for (int base = 0; base < n_cells; base += 64) {
    const int c = base + lane;
    const int64_t n = (c < n_cells) ? cnt[c] : 0;
    const int64_t o = (c < n_cells) ? off[c] : 0;
    const int32_t rs = (cell_ref && c < n_cells) ? cell_ref[c] : 0;  // same round trip
    const int32_t mine = (c < n_cells) ? items_of(n, lg_chunk, whole) : 0;
    const int32_t incl = wave_incl_scan_i32(mine);
    const int32_t total = lane_i32(incl, 63);
    if (item < before + total) {
      const unsigned long long m = __ballot(before + incl > item);
      const int l = __ffsll(static_cast<long long>(m)) - 1;
      loc.cell = base + l;
      loc.first = before + lane_i32(incl - mine, l);
      loc.chunk_idx = item - loc.first;
      loc.cnt = lane_i64(n, l);
      loc.off = lane_i64(o, l);
      loc.ref_sel = lane_i32(rs, l);
      return true;
    }
    before += total;
  }
  return false;
}

// ---- balanced mode (bandwidth-bound inputs) -------------------------------------------------
// Power-of-two items leave the chip unevenly loaded once the input is large: C4 (640k
// particles in 67 cells) made 693 items of 1024 particles for 768 resident slots, so 181 CUs
// ran 3 items and 75 ran 2, and the launch lasted as long as the 3-item CUs (measured,
// tools/probe_balance.py); smaller power-of-two items pay the per-item combine more often
// (C4 29.6 -> 34.1 -> 45.7 us at 256 -> 128 -> 64 particles per wave).  Slices of equal length
// across cell boundaries balance the stream exactly, but a workgroup holding two cells' segments
// runs two pipelines back to back and its second cell finalises ~5 us late.  Balanced mode keeps
// one item per workgroup: the grid is the device's resident capacity G and the chunk is
// total / (G - n_cells) rounded up to kChunkAlign, computed on the device from the counts.  It
// always fits (sum_c ceil(n_c / chunk) <= total / chunk + n_cells <= G), and no CU streams
// more than its slots x chunk.  (A binary search for the smallest fitting chunk cost ~3 us of
// wave reductions per launch on C4, more than the ~5% shorter stream it bought.)
inline bool balanced_mode(int64_t n_bound) {
  return n_bound > (int64_t(1) << CCMPC_LG_SMALL_INPUT);
}
constexpr int kChunkAlign = 16;  // item boundaries: whole 128-byte f64 lines, aligned quads

// ceil(n / d) for n >= 0, d > 0: 32-bit when both fit (every realistic cell), else 64-bit.
__device__ __forceinline__ int64_t ceil_div_fast(int64_t n, int64_t d) {
  if (n < (int64_t(1) << 31) && d < (int64_t(1) << 31))
    return static_cast<int64_t>((static_cast<uint32_t>(n) + static_cast<uint32_t>(d) - 1u) /
                                static_cast<uint32_t>(d));
  return (n + d - 1) / d;
}

// Wave sum of a double (two 32-bit DPP moves per step; exact for integer-valued inputs).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo =
      __builtin_amdgcn_update_dpp(0u, static_cast<uint32_t>(u), CTRL, 0xf, 0xf, false);
  const uint32_t hi =
      __builtin_amdgcn_update_dpp(0u, static_cast<uint32_t>(u >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, (static_cast<uint64_t>(hi) << 32) | lo);
}
__device__ __forceinline__ double wave_sum_dpp_f64(double v) {
  v += dpp_f64<0x111>(v);
  v += dpp_f64<0x112>(v);
  v += dpp_f64<0x114>(v);
  v += dpp_f64<0x118>(v);
  auto lane_val = [&](int l) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(u), l);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(u >> 32), l);
    return __builtin_bit_cast(double, (static_cast<uint64_t>(hi) << 32) | lo);
  };
  return (lane_val(15) + lane_val(31)) + (lane_val(47) + lane_val(63));
}

// ceil(n / c) for integer-valued 0 <= n < 2^53 and 0 < c, given rc ~ 1/c: one product, then
// two exact corrections (k c and (k - 1) c are exact: both < 2^53).
__device__ __forceinline__ double ceil_div_f64(double n, double c, double rc) {
  double k = ceil(n * rc);
  k = (k - 1.0) * c >= n ? k - 1.0 : k;
  k = k * c < n ? k + 1.0 : k;
  return k;
}

// The balanced chunk.  hi = (floor(total / ((G - n_cells) A)) + 1) A always fits (items =
// sum_c max(1, ceil(n_c / hi)) <= G), but it pays the worst case of every cell's rounding: the
// C4 per-GPU batch (67 cells, G = 512) got 1440-particle items where 1250 is the even share,
// so the CUs holding two full items streamed 15% more than the average.  With the counts of
// cells lane and 64 + lane in registers (n_cells <= 128), a bisection over multiples of A in
// [total / G, hi] finds the SMALLEST fitting chunk: a few uniform steps of one product, two
// corrections and a DPP wave sum each (CCMPC_BAL_SEARCH; the r02 search with a 64-bit
// division per cell and step cost ~3 us).  Every caller with the same counts gets the same
// chunk, so root_finalize_kernel re-derives the dealing exactly.  Measured
// (profiles/r03/s41_bal_search_tail_ab.log, two alternating passes): the C4 per-GPU batch's
// moments launch 27.7 / 27.8 us with the search against 27.7 / 27.9 without, C5 73.5 / 74.9
// against 73.7 / 73.0 -- the shorter items buy nothing (the warm stream is bound by the chip's
// rate from the Infinity Cache, not by the CUs holding two full items), so it stays off.
#ifndef CCMPC_BAL_SEARCH
#define CCMPC_BAL_SEARCH 0
#endif
__device__ __forceinline__ int64_t balanced_chunk(double td, int G, int n_cells, int64_t n0,
                                                  int64_t n1) {
  const int64_t A = kChunkAlign;
  int64_t hi = static_cast<int64_t>(td / (static_cast<double>(G - n_cells) * A)) + 1;  // x A
#if CCMPC_BAL_SEARCH
  if (n_cells <= 128) {  // uniform
    const int lane = threadIdx.x & 63;
    const bool in0 = lane < n_cells, in1 = lane + 64 < n_cells;
    const double d0 = static_cast<double>(n0), d1 = static_cast<double>(n1);
    int64_t lo = static_cast<int64_t>(ceil(td / (static_cast<double>(G) * A)));
    if (lo < 1) lo = 1;
    while (lo < hi) {  // uniform: every quantity below the branch is wave-wide
      const int64_t mid = (lo + hi) >> 1;
      const double c = static_cast<double>(mid * A), rc = 1.0 / c;
      double k = 0.0;
      if (in0) k += n0 > 0 ? ceil_div_f64(d0, c, rc) : 1.0;
      if (in1) k += n1 > 0 ? ceil_div_f64(d1, c, rc) : 1.0;
      if (wave_sum_dpp_f64(k) <= static_cast<double>(G))
        hi = mid;
      else
        lo = mid + 1;
    }
  }
#else
  (void)n0;
  (void)n1;
#endif
  return hi * A;
}

// Item id -> (cell, chunk index, ...) as locate_item, with the balanced chunk (returned in
// *chunk_out).
__device__ __forceinline__ bool locate_balanced(int32_t item, int G,
                                                const int64_t *__restrict__ cnt,
                                                const int64_t *__restrict__ off, int n_cells,
                                                ItemLoc &loc, int64_t *chunk_out,
                                                const int32_t *__restrict__ cell_ref = nullptr) {
  const int lane = threadIdx.x & 63;
  // cells 0..127 (every realistic batch) arrive in ONE round trip and stay in registers;
  // blocks beyond are re-read where needed
  const bool in0 = lane < n_cells, in1 = lane + 64 < n_cells;
  const int64_t n0 = in0 ? cnt[lane] : 0, n1 = in1 ? cnt[lane + 64] : 0;
  const int64_t o0 = in0 ? off[lane] : 0, o1 = in1 ? off[lane + 64] : 0;
  const int32_t rs0 = (cell_ref && in0) ? cell_ref[lane] : 0;
  const int32_t rs1 = (cell_ref && in1) ? cell_ref[lane + 64] : 0;
  auto count_at = [&](int base) -> int64_t {
    return base == 0 ? n0 : base == 64 ? n1 : (base + lane < n_cells ? cnt[base + lane] : 0);
  };
  double part = 0.0;  // exact: counts and their sum < 2^53
  for (int base = 0; base < n_cells; base += 64) part += static_cast<double>(count_at(base));
  const double td = wave_sum_dpp_f64(part);
  // the host keeps 2 n_cells <= G
  const int64_t chunk = balanced_chunk(td, G, n_cells, n0, n1);
  *chunk_out = chunk;
  int32_t before = 0;
  for (int base = 0; base < n_cells; base += 64) {
    const int c = base + lane;
    const bool in = c < n_cells;
    const int64_t n = count_at(base);
    const int64_t o = base == 0 ? o0 : base == 64 ? o1 : (in ? off[c] : 0);
    const int32_t rs = base == 0 ? rs0 : base == 64 ? rs1 : ((cell_ref && in) ? cell_ref[c] : 0);
    const int32_t mine = in ? static_cast<int32_t>(n > 0 ? ceil_div_fast(n, chunk) : 1) : 0;
    // __shfl_up / __shfl here, not wave_incl_scan_i32 / lane_*: the DPP form frees ~8 VGPRs,
    // which lets a third T = 12 balanced Scheme4 workgroup onto each CU, and that layout was
    // measured slower (C4 per-GPU batch 32.1 -> 34.7 us, profiles/r03/s52_dpp_locate_ab.log)
    int32_t incl = mine;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
      const int32_t y = __shfl_up(incl, s, 64);
      if (lane >= s) incl += y;
    }
    const int32_t tot = __shfl(incl, 63, 64);
    if (item < before + tot) {
      const unsigned long long m = __ballot(before + incl > item);
      const int l = __ffsll(static_cast<long long>(m)) - 1;
      loc.cell = base + l;
      loc.first = before + __shfl(incl - mine, l, 64);
      loc.chunk_idx = item - loc.first;
      loc.cnt = __shfl(n, l, 64);
      loc.off = __shfl(o, l, 64);
      loc.ref_sel = __shfl(rs, l, 64);
      return true;
    }
    before += tot;
  }
  return false;
}

// Host: the device's CU count (cached per device).
inline int device_cus() {
  static int cache[64];
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return 256;
  if (cache[d] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || n <= 0)
      n = 256;
    cache[d] = n;
  }
  return cache[d];
}

// Host: balanced-mode grid = resident workgroups of `kernel` at `threads` per workgroup.
template <auto Kernel>
inline int resident_grid(int threads) {
  static int cache[64];
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) d = 0;
  if (cache[d] == 0) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, Kernel, threads, 0) !=
            hipSuccess || per_cu <= 0)
      per_cu = 1;
    cache[d] = per_cu * device_cus();
  }
  return cache[d];
}

// Host: bound on the balanced-mode items of any kernel (<= 2048 threads per CU resident).
inline int64_t balanced_max_items(int threads) {
  return static_cast<int64_t>(device_cus()) * (2048 / threads);
}

// Sum over cells c < cell of f(c), wave-parallel (every wave computes it redundantly).
template <typename F>
__device__ __forceinline__ int64_t wave_prefix(int cell, F f) {
  const int lane = threadIdx.x & 63;
  int64_t s = 0;
  for (int c = lane; c < cell; c += 64) s += f(c);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  return s;
}

// One lane's 4 consecutive particles of a row, in the store's element type: two 16-byte loads
// (f64) or one (f32).  Kept unconverted until the consumer, so a load group has no use before
// its MFMA phase (a convert right after the load would force the wait there).
template <typename P>
struct Quad;
template <>
struct Quad<double> {
  double2 lo, hi;
  __device__ __forceinline__ double operator[](int j) const {
    return j == 0 ? lo.x : j == 1 ? lo.y : j == 2 ? hi.x : hi.y;
  }
};
template <>
struct Quad<float> {
  float4 v;
  __device__ __forceinline__ double operator[](int j) const {
    return static_cast<double>(j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w);
  }
};

// The stream loop's particle loads with the nontemporal hint: the store is read exactly once, so
// it need not displace what the caches hold.  Measured (profiles/r04/ab_nt_loads.log): the
// Scheme4 kernel's 16-byte row loads (load_pair, T = 9..12) gain -- the 64-scene C4 batch 218 ->
// 211 us warm, 211 -> 200 us cold (0.58 -> 0.61 of 8 TB/s), the per-GPU batch 36-37 -> 33.6 us
// cold -- while the 16x16-tile kernel's quad loads lose at T = 40 (C5 80 -> 88 us) and are
// neutral at T = 8: so pairs on, quads off.
#ifndef CCMPC_NT_PAIR
#define CCMPC_NT_PAIR 1
#endif
#ifndef CCMPC_NT_QUAD
#define CCMPC_NT_QUAD 0
#endif
typedef double ccmpc_d2v __attribute__((ext_vector_type(2)));
typedef float ccmpc_f2v __attribute__((ext_vector_type(2)));
typedef float ccmpc_f4v __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ double2 stream_load2(const double *p) {
  if constexpr (NT) {
    const ccmpc_d2v t = __builtin_nontemporal_load(reinterpret_cast<const ccmpc_d2v *>(p));
    return make_double2(t.x, t.y);
  } else {
    return *reinterpret_cast<const double2 *>(p);
  }
}
template <bool NT>
__device__ __forceinline__ float2 stream_load2(const float *p) {
  if constexpr (NT) {
    const ccmpc_f2v t = __builtin_nontemporal_load(reinterpret_cast<const ccmpc_f2v *>(p));
    return make_float2(t.x, t.y);
  } else {
    return *reinterpret_cast<const float2 *>(p);
  }
}
__device__ __forceinline__ void load_quad(const double *__restrict__ p, Quad<double> &q) {
  q.lo = stream_load2<CCMPC_NT_QUAD != 0>(p);
  q.hi = stream_load2<CCMPC_NT_QUAD != 0>(p + 2);
}
__device__ __forceinline__ void load_quad(const float *__restrict__ p, Quad<float> &q) {
  if constexpr (CCMPC_NT_QUAD != 0) {
    const ccmpc_f4v t = __builtin_nontemporal_load(reinterpret_cast<const ccmpc_f4v *>(p));
    q.v = make_float4(t.x, t.y, t.z, t.w);
  } else {
    q.v = *reinterpret_cast<const float4 *>(p);
  }
}

// 16-byte write-through (sc1) buffer accesses: one dwordx4 transaction per lane instead of two
// 8-byte atomic-typed ones.
// aux = 16 selects sc1 on gfx950; word 3 = 0x00020000 is the raw-buffer format for gfx9.
typedef unsigned int b128_t __attribute__((__vector_size__(16)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t slab_rsrc(const double *base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(base), 0, 0x7fffffff, 0x00020000);
}

__device__ __forceinline__ void st2_sc1(__amdgpu_buffer_rsrc_t r, int byte_off, double a,
                                        double b) {
  const double2 v = {a, b};
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(b128_t, v), r, byte_off, 0, 16);
}

__device__ __forceinline__ double2 ld2_sc1(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16));
}

// Slab entry order: tile t, lane l, register k at t*256 + 4 l + k (lane-major, so a lane's 4
// accumulators are two 16-byte stores); then the RB*16 row sums.
__device__ __forceinline__ void decode_entry(int e, int RB, int &i, int &j) {
  const int tile = e >> 8, l = (e >> 2) & 63, k = e & 3;
  const int row = (l >> 4) + 4 * k, col = l & 15;
  int bi = 0, t = tile;
  while (t >= RB - bi) {
    t -= RB - bi;
    ++bi;
  }
  i = 16 * bi + row;
  j = 16 * (bi + t) + col;
}

// Tiles exchanged per round of combine_waves, and the LDS it needs (doubles).  Up to 5 tiles
// per round: T = 40's 15 tiles in 3 rounds, 80 KB of LDS at 8 waves.
#ifndef CCMPC_COMBINE_TPR  // build knob: the most tiles a combine round parks
#define CCMPC_COMBINE_TPR 5
#endif
__host__ __device__ constexpr int combine_tiles_per_round(int rb) {
  return n_tiles(rb) < CCMPC_COMBINE_TPR ? n_tiles(rb) : CCMPC_COMBINE_TPR;
}
__host__ __device__ constexpr int combine_xch_doubles(int rb, int nw) {
  // the tile rounds' park area, then the row sums' (every lane's, parked with the first round)
  return nw * combine_tiles_per_round(rb) * 256 + 64 * rb * nw;
}

// Combine the NW waves' accumulators in a fixed order (wave 0 + 1 + ... + NW-1) and write the
// item's slab: to global memory write-through (to_lds = false) or to the LDS slab `dst`
// (to_lds = true).  Rounds of up to combine_tiles_per_round tiles: every wave parks its tiles
// in `xch` (combine_xch_doubles(RB, NW) doubles), then EVERY thread sums entry pairs over the
// waves and stores them -- the sum and the stores are spread over the whole workgroup (with
// wave 0 alone doing them tile by tile, T = 40's 15 tiles took 28 us); the row sums are parked
// and summed with the first round (two barriers instead of two more per row block).  Every
// thread of the workgroup must call it.
template <int RB, int NACC, int NW>
__device__ __forceinline__ void combine_waves(const d4 (&acc)[NACC][n_tiles(RB)],
                                              const double (&s1)[RB], double *xch, double *dst,
                                              bool to_lds) {
  constexpr int NT = n_tiles(RB);
  constexpr int TB = combine_tiles_per_round(RB);
  constexpr int XR = NW * TB * 256;  // the row sums' park area: [w][RB * 16]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t rs = slab_rsrc(dst);
  // the row sums ride the first round: every lane parks its partial (lane r + 16 g: row r of
  // particle group g) and the summing thread adds the four groups as the xor-16 / xor-32 lane
  // butterfly did, ((g0 + g1) + (g2 + g3)), then the waves in order -- the same bits without
  // two dependent cross-lane round trips per row block before the barrier
#pragma unroll
  for (int b = 0; b < RB; ++b) xch[XR + (w * RB + b) * 64 + lane] = s1[b];
#pragma unroll
  for (int t0 = 0; t0 < NT; t0 += TB) {
    // park: xch[((w TB + tb) 4 + k) 64 + lane] = this wave's register k of tile t0 + tb
#pragma unroll
    for (int tb = 0; tb < TB; ++tb) {
      if (t0 + tb < NT) {
        d4 s = acc[0][t0 + tb];
        if (NACC == 2) s += acc[NACC - 1][t0 + tb];
#pragma unroll
        for (int k = 0; k < 4; ++k) xch[((w * TB + tb) * 4 + k) * 64 + lane] = s[k];
      }
    }
    __syncthreads();
    // slab entry t*256 + 4 l + k <-> (tile t, lane l, register k); pairs (k, k+1), k even
    const int n_e = (NT - t0 < TB ? NT - t0 : TB) * 256;
    for (int e = 2 * threadIdx.x; e < n_e; e += 2 * blockDim.x) {
      const int tb = e >> 8, l = (e >> 2) & 63, k = e & 3;
      const double *x = xch + (tb * 4 + k) * 64 + l;
      double a = x[0], b = x[64];
#pragma unroll
      for (int o = 1; o < NW; ++o) {
        a += x[o * TB * 256];
        b += x[o * TB * 256 + 64];
      }
      const int ge = t0 * 256 + e;
      if (to_lds) {
        dst[ge] = a;
        dst[ge + 1] = b;
      } else {
        st2_sc1(rs, 8 * ge, a, b);
      }
    }
    if (t0 == 0) {
      // row-sum pair (2 i, 2 i + 1) of row block b: wave 0's value, then + waves 1, 2, ...
      const int i = static_cast<int>(blockDim.x) - 1 - static_cast<int>(threadIdx.x);
      if (i < 8 * RB) {
        const int b = i >> 3, r = 2 * (i & 7);
        auto rowsum = [&](int o, int rr) {  // wave o's row rr: ((g0 + g1) + (g2 + g3))
          const double *x = xch + XR + (o * RB + b) * 64 + rr;
          return (x[0] + x[16]) + (x[32] + x[48]);
        };
        double v0 = rowsum(0, r), v1 = rowsum(0, r + 1);
#pragma unroll
        for (int o = 1; o < NW; ++o) {
          v0 += rowsum(o, r);
          v1 += rowsum(o, r + 1);
        }
        const int e = NT * 256 + b * 16 + r;
        if (to_lds) {
          dst[e] = v0;
          dst[e + 1] = v1;
        } else {
          st2_sc1(rs, 8 * e, v0, v1);
        }
      }
    }
    __syncthreads();
  }
}

// Drain the workgroup's slab stores, take a ticket; true (in every thread) for the last of
// `nit` arrivals, which also resets the counter for the next launch.
__device__ __forceinline__ bool arrive_last(int32_t *counter, int64_t nit, int *flag_lds) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    const int ticket =
        __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = static_cast<int64_t>(ticket) == nit - 1;
    if (last) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag_lds = last ? 1 : 0;
  }
  __syncthreads();
  const bool last = *flag_lds != 0;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // keep slab loads below the ticket
  return last;
}

// ---- fixed fan-in combine tree ------------------------------------------------------------
// Items of a cell are the leaves (level 0).  Each group of up to kFanIn consecutive level-l
// nodes has an arrival counter; its last arriver sums the group's slabs into one level-(l+1)
// slab.  When a level has <= kFanIn nodes, the last arriver of that single group is the cell's
// reducer.  Depth = ceil(log16(items)), every combine reads <= 16 slabs with all loads in
// flight at once, and the summation order is fixed by the tree: bitwise reproducible.
struct TreeLayout {
  int32_t *counters[kMaxLevels];  // level l: one counter per group of level-l nodes
  double *slabs[kMaxLevels];      // level l: node slabs (level 0 = work items)
};

// Combine-tree numbering.  A cell's level-l nodes are [F_l, F_l + n_l); its level-(l+1) nodes
// start at F_{l+1} = floor(F_l / 16) + cell.  Collision-free by induction: the next cell
// starts at floor((F_l + n_l) / 16) + cell + 1 >= floor(F_l / 16) + ceil(n_l / 16) + cell, and
// level l+1 never holds more than ceil(n_l / 16) of this cell's nodes.  So every level's first
// node follows from the level-0 prefix alone (no per-level scans), and level l+1 needs at most
// (level-l nodes) / 16 + n_cells + 1 slots (level_capacity).
__device__ __forceinline__ int32_t tree_next_first(int32_t first_l, int cell) {
  return (first_l >> kLgFanIn) + cell;
}

// A level with at most kRootFanIn nodes is combined by ONE last arriver (the root); larger
// levels are reduced in fixed groups of kFanIn first.  Cells up to 64 items thus need a single
// arrival round trip.
#ifndef CCMPC_ROOT_FANIN
#define CCMPC_ROOT_FANIN 64
#endif
constexpr int kRootFanIn = CCMPC_ROOT_FANIN;

// Host: capacity of level l (nodes) for n_cells cells holding <= max_items items in total.
inline int64_t level_capacity(int64_t max_items, int64_t n_cells, int l) {
  int64_t c = max_items;
  for (int i = 0; i < l; ++i) c = c / kFanIn + n_cells;  // sum of ceils <= sum/16 + cells
  return c + 1;
}

inline size_t tree_counter_bytes(int64_t max_items, int64_t n_cells) {
  size_t ctr = 0;
  for (int l = 0; l < kMaxLevels; ++l)
    ctr += static_cast<size_t>(level_capacity(max_items, n_cells, l + 1)) * sizeof(int32_t);
  return (ctr + kCounterAlign - 1) / kCounterAlign * kCounterAlign;
}

inline size_t tree_slab_bytes(int64_t max_items, int64_t n_cells, int E) {
  size_t slab = 0;
  for (int l = 0; l < kMaxLevels; ++l)
    slab += static_cast<size_t>(level_capacity(max_items, n_cells, l)) * E * sizeof(double);
  return slab;
}

// Workspace layout.  The arrival counters live in the first ctr_region(ws_bytes) =
// round_up(ws_bytes / 32, 256) bytes -- a function of the WHOLE buffer only -- and the slabs
// after it.  Calls of different shapes sharing one buffer (e.g. a moments call on a small
// store, then a 1e6-sample rollout) therefore agree on where counters are: a per-call
// counter size would let one call's slabs land on another call's counters, which must be
// zero when a launch starts (every launch leaves them zero).  Counters are <= 1.7 % of the
// slab bytes (E >= 176 doubles per node), so 1/32 of the buffer always holds them.
inline size_t ctr_region(size_t ws_bytes) {
  return (ws_bytes / 32 + kCounterAlign - 1) / kCounterAlign * kCounterAlign;
}

inline size_t tree_bytes(int64_t max_items, int64_t n_cells, int E) {
  const size_t c = tree_counter_bytes(max_items, n_cells);
  const size_t s = tree_slab_bytes(max_items, n_cells, E);
  size_t ws = (c + s) + (c + s) / 31 + 2 * kCounterAlign;  // ws - ctr_region(ws) >= s
  if (ctr_region(ws) < c) ws = 32 * c;                     // never binds at E >= 176
  return (ws + kCounterAlign - 1) / kCounterAlign * kCounterAlign;
}

// False when the buffer cannot hold this call's counters or slabs.
inline bool tree_layout(void *ws, size_t ws_bytes, int64_t max_items, int64_t n_cells, int E,
                        TreeLayout &L) {
  const size_t region = ctr_region(ws_bytes);
  if (tree_counter_bytes(max_items, n_cells) > region ||
      region + tree_slab_bytes(max_items, n_cells, E) > ws_bytes)
    return false;
  int32_t *c = static_cast<int32_t *>(ws);
  for (int l = 0; l < kMaxLevels; ++l) {
    L.counters[l] = c;
    c += level_capacity(max_items, n_cells, l + 1);
  }
  double *s = reinterpret_cast<double *>(static_cast<char *>(ws) + region);
  for (int l = 0; l < kMaxLevels; ++l) {
    L.slabs[l] = s;
    s += level_capacity(max_items, n_cells, l) * E;
  }
  return true;
}


// Sum the entry pair (e, e+1), e even, over n <= kFanIn consecutive slabs: all 16-byte sc1 loads
// issued first (indices clamped, no per-load branch), then a fixed-order sum.
__device__ __forceinline__ double2 sum_group2(const double *__restrict__ slab0, int64_t n, int E,
                                              int e) {
  const __amdgpu_buffer_rsrc_t rs = slab_rsrc(slab0);
  double2 v[kFanIn];
#pragma unroll
  for (int i = 0; i < kFanIn; ++i) {
    const int j = static_cast<int>(i < n ? i : n - 1);
    v[i] = ld2_sc1(rs, 8 * (j * E + e));
  }
  double2 s = v[0];
#pragma unroll
  for (int i = 1; i < kFanIn; ++i) {
    s.x += (i < n) ? v[i].x : 0.0;
    s.y += (i < n) ? v[i].y : 0.0;
  }
  return s;
}

// Climb the tree from a published leaf.  Returns true in the workgroup that must finalise the
// cell; then *root points at the root level's first slab and *root_n is its node count
// (<= kRootFanIn).  first0 is the cell's first item; deeper levels follow tree_next_first.
template <int E>
__device__ bool tree_climb(const TreeLayout &L, int32_t idx, int32_t nit, int32_t first0,
                           int cell, int *flag, const double **root, int32_t *root_n) {
  int32_t n_l = nit, first_l = first0;
  for (int l = 0; l < kMaxLevels; ++l) {
    const int32_t first_up = tree_next_first(first_l, cell);
    const bool is_root = n_l <= kRootFanIn || l + 1 == kMaxLevels;
    const int32_t grp = is_root ? 0 : idx >> kLgFanIn;
    const int32_t gsize = is_root ? n_l : min(n_l - grp * kFanIn, kFanIn);
    if (!arrive_last(L.counters[l] + first_up + grp, gsize, flag)) return false;
    const double *children = L.slabs[l] + static_cast<int64_t>(first_l + grp * kFanIn) * E;
    if (is_root) {
      *root = L.slabs[l] + static_cast<int64_t>(first_l) * E;
      *root_n = n_l;
      return true;
    }
    double *parent = L.slabs[l + 1] + static_cast<int64_t>(first_up + grp) * E;
    const __amdgpu_buffer_rsrc_t rp = slab_rsrc(parent);
    for (int e = 2 * threadIdx.x; e < E; e += 2 * blockDim.x) {
      const double2 s = sum_group2(children, gsize, E, e);
      st2_sc1(rp, 8 * e, s.x, s.y);
    }
    idx = grp;
    n_l = (n_l + kFanIn - 1) >> kLgFanIn;
    first_l = first_up;
  }
  return false;
}

// ---- Gram schemes: how a slab's entries map to Gram positions -------------------------------
// Scheme16<RB>: f64 16x16x4 MFMA tiles (any T <= 40); Scheme4<NB>: f64 4x4x4_4b MFMA blocks of
// 4 rows (T <= 12), which compute 4-row block pairs instead of 16-row tiles -- far less
// padding work when 2T is not a multiple of 16 (T = 12: 21 block pairs = 336 products per
// 16 particles vs 3 tiles = 768), at the same flop rate per cycle.
template <int RB>
struct Scheme16 {
  static constexpr int GRAM = n_tiles(RB) * 256;
  static constexpr int D = 16 * RB;
  static constexpr int E = GRAM + D;
  __device__ static void decode(int e, int &i, int &j) { decode_entry(e, RB, i, j); }
};

__host__ __device__ constexpr int n_pairs(int nb) { return nb * (nb + 1) / 2; }

template <int NB>
struct Scheme4 {
  static constexpr int NP = n_pairs(NB);
  static constexpr int GRAM = NP * 16;  // entry p*16 + 4i + j: G[4I + i][4J + j], pair p = (I, J)
  static constexpr int D = 4 * NB;
  static constexpr int E = GRAM + D;
  __device__ static void decode(int e, int &i, int &j) {
    int p = e >> 4, I = 0;
    while (p >= NB - I) {  // pairs in row-major upper-triangle order
      p -= NB - I;
      ++I;
    }
    i = 4 * I + ((e >> 2) & 3);
    j = 4 * (I + p) + (e & 3);
  }
};

// DPP rotate within 16-lane rows (row_ror:k, dpp_ctrl 0x120 + k) of an f64, as two 32-bit moves.
template <int K>
__device__ __forceinline__ double row_ror(double x) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x120 + K, 0xf, 0xf, false);
  const int hi =
      __builtin_amdgcn_update_dpp(0, static_cast<int>(v >> 32), 0x120 + K, 0xf, 0xf, false);
  return __longlong_as_double((static_cast<long long>(hi) << 32) |
                              static_cast<unsigned int>(lo));
}

// Scheme4 cross-wave combine.  acc[p] holds, in lane c + 4b + 16i, block b's partial of
// G[4I + i][4J + c] (v_mfma_f64_4x4x4_4b layout: D[b][i][j] -> lane j + 4b + 16i); s1[I]
// holds row 4I + c summed over this lane's particles.  The 4 blocks of a 16-lane row fold
// with two DPP row rotations (register moves, no LDS traffic); lanes b == 0 then write one
// E4-vector per wave (Gram entries final, row sums still split over the 4 rows i), and the
// whole workgroup adds the waves (and the row-sum rows) in fixed order into dst -- an LDS slab,
// or a global slab with 16-byte write-through stores.  Ends with a barrier.
template <int NB>
struct Combine4Layout {
  static constexpr int GRAM = n_pairs(NB) * 16;
  static constexpr int XS = GRAM + 16 * NB;  // per-wave exchange vector
};

template <int NB, int NW>
__device__ __forceinline__ void combine4(const double (&acc)[n_pairs(NB)], const double (&s1)[NB],
                                         double *xch, double *dst, bool to_lds) {
  using Sch = Scheme4<NB>;
  constexpr int XS = Combine4Layout<NB>::XS;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool writer = (lane & 12) == 0;  // b == 0
  const int slot = 4 * (lane >> 4) + (lane & 3);  // 4i + c
  double *mine = xch + w * XS;
#pragma unroll
  for (int p = 0; p < Sch::NP; ++p) {
    double v = acc[p];
    v += row_ror<8>(v);
    v += row_ror<4>(v);
    if (writer) mine[p * 16 + slot] = v;
  }
#pragma unroll
  for (int I = 0; I < NB; ++I) {
    double v = s1[I];
    v += row_ror<8>(v);
    v += row_ror<4>(v);
    if (writer) mine[Sch::GRAM + 16 * I + slot] = v;  // row 4I + c, particle row i
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = slab_rsrc(dst);
  for (int e = 2 * threadIdx.x; e < Sch::E; e += 2 * blockDim.x) {
    double a = 0.0, b = 0.0;
    if (e < Sch::GRAM) {
#pragma unroll
      for (int o = 0; o < NW; ++o) {
        a += xch[o * XS + e];
        b += xch[o * XS + e + 1];
      }
    } else {  // row sums: rows r = e - GRAM (block I = r / 4, c = r % 4), summed over i and w
      const int r = e - Sch::GRAM, I = r >> 2, c = r & 3;
      const double *base = xch + Sch::GRAM + 16 * I;
#pragma unroll
      for (int o = 0; o < NW; ++o)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a += base[o * XS + 4 * i + c];
          b += base[o * XS + 4 * i + c + 1];
        }
    }
    if (to_lds) {
      dst[e] = a;
      dst[e + 1] = b;
    } else {
      st2_sc1(rs, 8 * e, a, b);
    }
  }
  __syncthreads();
}

// The last arriver's root combine: every summed entry pair of the n <= 16 root slabs into LDS
// in ONE round of 16-byte sc1 loads (the finaliser then reads LDS only, instead of paying a
// second dependent global round trip for the Gram tiles after the row sums).  Ends with a
// barrier.
template <int E>
__device__ __forceinline__ void gather_root(const double *__restrict__ root, int32_t root_n,
                                            double *dst_lds) {
  for (int e = 2 * threadIdx.x; e < E; e += 2 * blockDim.x) {
    double2 s = sum_group2(root, min(root_n, kFanIn), E, e);
    for (int k = kFanIn; k < root_n; k += kFanIn) {  // fixed order: deterministic
      const double2 t = sum_group2(root + static_cast<int64_t>(k) * E, min(root_n - k, kFanIn),
                                   E, e);
      s.x += t.x;
      s.y += t.y;
    }
    dst_lds[e] = s.x;
    dst_lds[e + 1] = s.y;
  }
  __syncthreads();
}

// The per-cell finalisation: summed slab entries (read through `rd(e)`) -> mean[T][2]
// (+ origin) and cov[2T][2T] (ddof = 1), cov = (G - S S^T / n) / (n - 1) on data shifted by
// shift_lds.  Writes cov to global memory and, when cov_lds != nullptr, to LDS as well (row
// stride 2T) for the fused half-space tail.  Called by every thread of the workgroup; ends
// with a barrier.
template <typename Sch, typename Reader>
__device__ void finalize_cell(Reader rd, int64_t cnt, int T, const double *shift_lds,
                              double *S_lds, double o0, double o1, double *__restrict__ mean,
                              double *__restrict__ cov, double *mean_lds, double *cov_lds,
                              const double *S_in = nullptr) {
  constexpr int GRAM = Sch::GRAM;
  constexpr int D = Sch::D;
  const int tid = threadIdx.x, nth = blockDim.x;
  const int rows = 2 * T;
  const double n = static_cast<double>(cnt);
  // rd(e) returns the summed entry pair (e, e+1), e even.  S_in: the summed row sums already in
  // LDS (a slab there, entries GRAM.. after the caller's barrier) -- no copy, no barrier
  const double *S = S_in;
  if (!S) {
    for (int r = 2 * tid; r < D; r += 2 * nth) {
      const double2 s = r < rows ? rd(GRAM + r) : double2{0.0, 0.0};
      S_lds[r] = s.x;
      S_lds[r + 1] = s.y;
    }
    __syncthreads();
    S = S_lds;
  }
  for (int r = tid; r < rows; r += nth) {
    const double m = (shift_lds[r] + S[r] / n) + ((r & 1) ? o1 : o0);
    mean[r] = m;
    if (mean_lds) mean_lds[r] = m;
  }
  for (int e = 2 * tid; e < GRAM; e += 2 * nth) {
    int i0, j0, i1, j1;
    Sch::decode(e, i0, j0);
    Sch::decode(e + 1, i1, j1);
    const bool use0 = i0 < rows && j0 < rows && i0 <= j0;  // one value per symmetric pair
    const bool use1 = i1 < rows && j1 < rows && i1 <= j1;
    if (!use0 && !use1) continue;
    const double2 g = rd(e);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (!(h ? use1 : use0)) continue;
      const int i = h ? i1 : i0, j = h ? j1 : j0;
      const double c = ((h ? g.y : g.x) - S[i] * S[j] / n) / (n - 1.0);
      cov[i * rows + j] = c;
      cov[j * rows + i] = c;
      if (cov_lds) {
        cov_lds[i * rows + j] = c;
        cov_lds[j * rows + i] = c;
      }
    }
  }
  __syncthreads();
}

}  // namespace ccmpc
