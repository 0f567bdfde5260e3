// Segmented moment (Gram) reduction of particle clouds -- the dominant kernel of the path --
// optionally fused with the Minkowski/MVOE half-space assembly of each finished cell.
//
// Replaces every np.mean / np.cov the reference runs over particle clouds
// (v8ideal/__init__.py:864-875, :896, :907 -> makeconstraint.py:41-70, :1485-1493,
// :2584-2606).  The reference calls np.cov once per (t, tau) pair on a strided 4xN gather;
// every one of those 4x4 matrices is a block of ONE 2T x 2T covariance per cell, so the
// particle cloud is read exactly once.
//
// Design (gfx950), ONE launch per call:
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
//  * Work item = one workgroup of Geo<RB>::NW waves over CHUNK particles of one cell (gram.hpp).
//    A cell that fits one item is combined entirely in LDS; larger cells publish per-item
//    slabs write-through and meet in the fixed fan-in-16 tree.  The cell's finaliser then
//    (cycle variant) builds its T(T-1)/2 half-spaces from the covariance it just produced in
//    LDS -- no kernel boundary between moments and constraints.
#include "constraints.hpp"
#include <algorithm>
#include <type_traits>

#include "gram.hpp"

#ifndef CCMPC_PROBE
#define CCMPC_PROBE 0
#endif

// CCMPC_PROBE & 4 (diagnostic build only): per-workgroup phase timestamps (s_memrealtime,
// 100 MHz) into a device table read back by ccmpc_probe_timestamps.
#if CCMPC_PROBE & 4
constexpr int kProbeSlots = 8, kProbeMaxWG = 8192;
__device__ unsigned long long g_probe_ts[kProbeMaxWG * kProbeSlots];
#define PROBE_TS(k)                                                                            \
  do {                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < kProbeMaxWG)                                          \
      g_probe_ts[blockIdx.x * kProbeSlots + (k)] = __builtin_amdgcn_s_memrealtime();           \
    if ((k) == 0 && !(CCMPC_PROBE & 16) && threadIdx.x == 0 && blockIdx.x < kProbeMaxWG)       \
      g_probe_ts[blockIdx.x * kProbeSlots + 7] =                                               \
          (static_cast<unsigned long long>(__builtin_amdgcn_s_getreg(0xF814)) << 32) |         \
          __builtin_amdgcn_s_getreg(0xF804); /* XCC_ID : HW_ID, slot 7 */                       \
  } while (0)
#else
#define PROBE_TS(k) \
  do {              \
  } while (0)
#endif
// CCMPC_PROBE & 16 (with 4): slot 7 = the root gather's end instead of the hardware ids
#if (CCMPC_PROBE & 4) && (CCMPC_PROBE & 16)
#define PROBE_GATHERED()                                                                       \
  do {                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < kProbeMaxWG)                                          \
      g_probe_ts[blockIdx.x * kProbeSlots + 7] = __builtin_amdgcn_s_memrealtime();             \
  } while (0)
#else
#define PROBE_GATHERED() \
  do {                   \
  } while (0)
#endif

namespace ccmpc {

// Load groups in flight per wave (a ring: DEPTH - 1 groups stream while one is multiplied).
#ifndef CCMPC_DEPTH
#define CCMPC_DEPTH 2
#endif
#ifndef CCMPC_DEPTH4
#define CCMPC_DEPTH4 CCMPC_DEPTH
#endif
constexpr int kDepth = CCMPC_DEPTH;
#ifndef CCMPC_DEPTH_BIG  // the ring at RB >= 3 (T > 24)
#define CCMPC_DEPTH_BIG CCMPC_DEPTH
#endif
#ifndef CCMPC_PRIO
#define CCMPC_PRIO 0
#endif
// Particles per lane per sub-step at RB >= 4 (T > 24): 4 or 2 (LaneVec).  W = 2 with a 4-deep
// ring keeps 15 KB per wave in flight instead of 10 KB at the same 252 VGPRs: C5 moments 75.6 /
// 77.1 us against 77.3 / 74.4 (a 3-deep ring 76.6 / 75.4; 5-deep spills, 91 us;
// profiles/r03/s44_c5_pair_loads_depth_ab.log) -- bytes in flight do not bound C5's stream, so 4.
#ifndef CCMPC_W_BIG
#define CCMPC_W_BIG 4
#endif
constexpr int kWBig = CCMPC_W_BIG;
static_assert(kWBig == 2 || kWBig == 4, "CCMPC_W_BIG must be 2 or 4");
constexpr int kDepth4 = CCMPC_DEPTH4;
#ifndef CCMPC_DEPTH4_BAL  // the Scheme4 ring in balanced mode (one item per resident workgroup):
#define CCMPC_DEPTH4_BAL 3  // C4 per-GPU batch 33.9 -> 32.5 us warm, 38.7 -> 37.0 cold (ab14)
#endif
constexpr int kDepth4Bal = CCMPC_DEPTH4_BAL;
#ifndef CCMPC_DEPTH4_BAL_F32  // the same for the f32 store (64-particle groups, CCMPC_F32_WIDE4)
#define CCMPC_DEPTH4_BAL_F32 CCMPC_DEPTH4_BAL
#endif
constexpr int kDepth4BalF32 = CCMPC_DEPTH4_BAL_F32;

// Progress priority (balanced mode): issue is arbitrated by priority, then age
// (MI355X_MICROARCH.md, two waves per SIMD), so of two co-resident workgroups the older one
// streams ahead and finishes its item at ~14 us while its partner needs ~19 (C4/8, every CU,
// profiles/r03/s29_c4_pairs.txt) and then cannot fill the CU alone.  With the priority
// falling by one per quarter of the wave's groups done, whichever wave is behind outranks the
// one ahead, so the two stay within a quarter of each other.  Arithmetic unchanged: the bits
// are the same.
#ifndef CCMPC_PROGRESS_PRIO
#define CCMPC_PROGRESS_PRIO 0
#endif
__device__ __forceinline__ void progress_prio(int64_t done, int64_t total) {
#if CCMPC_PROGRESS_PRIO
  const int q = __builtin_amdgcn_readfirstlane(
      static_cast<int>(total > 0 ? (4 * done) / total : 4));  // wave-uniform: a scalar branch
  if (q <= 0)
    __builtin_amdgcn_s_setprio(3);
  else if (q == 1)
    __builtin_amdgcn_s_setprio(2);
  else if (q == 2)
    __builtin_amdgcn_s_setprio(1);
  else
    __builtin_amdgcn_s_setprio(0);
#else
  (void)done;
  (void)total;
#endif
}

// Loads are pure loads, branch-free: every lane always issues its 16-byte loads, the address
// clamped to the wave's last aligned W-particle run (addressable because cell offsets and ld are
// multiples of 4).  Masking (out-of-range particles, dead rows) happens in mfma_group, so a
// group's loads have no consumer until its MFMAs run.  A guarded scalar fallback here turned
// the loop into branches, and the waitcnt pass then drained vmcnt(0) before every MFMA group --
// waiting on the NEXT group's loads too, which serialised the double buffer.
//
// W = particles per lane per sub-step: 4 (Quad: two 16-byte f64 loads, a row's 16 particles of
// a sub-step = one 128-byte line) or 2 (Pair: one 16-byte f64 load, 8 particles per sub-step);
// the narrower form halves the registers of a load group, so the same budget keeps twice the
// groups in flight (CCMPC_W_BIG, long horizons).
template <typename P>
struct Pair;
template <>
struct Pair<double> {
  double2 v;
  __device__ __forceinline__ double operator[](int j) const { return j ? v.y : v.x; }
};
template <>
struct Pair<float> {
  float2 v;
  __device__ __forceinline__ double operator[](int j) const {
    return static_cast<double>(j ? v.y : v.x);
  }
};
__device__ __forceinline__ void load_pair(const double *__restrict__ p, Pair<double> &q) {
  q.v = stream_load2<CCMPC_NT_PAIR != 0>(p);
}
__device__ __forceinline__ void load_pair(const float *__restrict__ p, Pair<float> &q) {
  q.v = stream_load2<CCMPC_NT_PAIR != 0>(p);
}

template <typename P, int W>
struct LaneVec;
template <typename P>
struct LaneVec<P, 4> {
  using type = Quad<P>;
  __device__ static void load(const P *p, type &q) { load_quad(p, q); }
};
template <typename P>
struct LaneVec<P, 2> {
  using type = Pair<P>;
  __device__ static void load(const P *p, type &q) { load_pair(p, q); }
};

template <typename P, int RB, int S, int W>
__device__ __forceinline__ void load_group(typename LaneVec<P, W>::type (&v)[S][RB],
                                           const P *const (&rowp)[RB], int64_t gbase, int64_t p1,
                                           int g) {
  const int64_t qlast = (p1 - 1) & ~int64_t(W - 1);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int64_t q = gbase + 4 * W * s + W * g;
    const int64_t qc = q < qlast ? q : qlast;
#pragma unroll
    for (int b = 0; b < RB; ++b) {
#if CCMPC_PROBE & 2  // diagnostic build only: every lane re-reads one cached run
      LaneVec<P, W>::load(rowp[b] + (qc & (W - 1)), v[s][b]);
#else
      LaneVec<P, W>::load(rowp[b] + qc, v[s][b]);
#endif
    }
  }
}

template <typename P, int RB, int S, int NACC, int W>
__device__ __forceinline__ void mfma_group(const typename LaneVec<P, W>::type (&raw)[S][RB],
                                           const double (&sh)[RB], const bool (&live)[RB],
                                           int64_t gbase, int64_t p1, int g,
                                           d4 (&acc)[NACC][n_tiles(RB)], double (&s1)[RB]) {
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int64_t q = gbase + 4 * W * s + W * g;
    double v[RB][W];
#pragma unroll
    for (int b = 0; b < RB; ++b)
#pragma unroll
      for (int j = 0; j < W; ++j)  // shifted; out-of-range slots and dead rows become 0
#if CCMPC_PROBE & 32  // diagnostic build only: no masks (wrong at partial groups; timing bound)
        v[b][j] = raw[s][b][j] - sh[b];
#elif CCMPC_PROBE & 64  // diagnostic build only: neither masks nor the shift
        v[b][j] = raw[s][b][j];
#else
        v[b][j] = (live[b] && q + j < p1) ? raw[s][b][j] - sh[b] : 0.0;
#endif
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const int a = (NACC == 2) ? (j & 1) : 0;
      int t = 0;
#pragma unroll
      for (int bi = 0; bi < RB; ++bi)
#pragma unroll
        for (int bj = bi; bj < RB; ++bj) {
#if CCMPC_PROBE & 1  // diagnostic build only: no matrix-core work
          acc[a][t][0] += v[bi][j] * v[bj][j];
#else
          acc[a][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(v[bi][j], v[bj][j], acc[a][t], 0, 0, 0);
#endif
          ++t;
        }
    }
#pragma unroll
    for (int b = 0; b < RB; ++b)
      s1[b] += W == 4 ? (v[b][0] + v[b][1]) + (v[b][2 % W] + v[b][3 % W]) : v[b][0] + v[b][1];
  }
}

// Everything after a work item's stream loop, shared by both Gram schemes: publish the item's
// partial Gram (publish(dst, to_lds) = the scheme's cross-wave combine), then either finalise
// in LDS (the cell is this one item) or climb the combine tree, and as the cell's last arriver
// gather the root, finalise and (MINK) build the cell's half-spaces.
// Long horizons (16x16 tiles, RB >= 4, i.e. T > 24) in balanced mode, moments only: a cell's
// root gather is up to kRootFanIn slabs of 10-31 KB, ~1 MB on ONE CU for T = 40 (8 us at the
// CU's L2 bandwidth).  Such cells skip the arrival; root_finalize_kernel then sums them in the
// root gather's order, one workgroup per (cell, tile), so the values are the same bits.
#ifndef CCMPC_DEFER_ROOT
#define CCMPC_DEFER_ROOT 1
#endif
__host__ __device__ constexpr bool defer_root(int rb, bool mink, bool bal) {
  return CCMPC_DEFER_ROOT && bal && !mink && rb >= 4;
}

struct EpilogueLds {
  double *slab, *shift, *S, *mean, *cov, *lb, *ref;
  int *flag;
};

template <typename Sch, bool MINK, bool COV_IN_LDS, bool DEFER, typename Publish>
__device__ __forceinline__ void cell_epilogue(Publish publish, const ItemLoc &loc, int32_t nit,
                                              int T, const TreeLayout &tree,
                                              const double *__restrict__ origin,
                                              double *__restrict__ out_mean,
                                              double *__restrict__ out_cov, const MinkParams &mp,
                                              const EpilogueLds &L) {
  constexpr int E = Sch::E;
  const int cell = loc.cell, rows = 2 * T;
  const double o0 = origin ? origin[2 * cell] : 0.0, o1 = origin ? origin[2 * cell + 1] : 0.0;
  double *mean = out_mean + static_cast<int64_t>(cell) * rows;
  double *cov = out_cov + static_cast<int64_t>(cell) * rows * rows;
  if (nit == 1) {
    // the whole cell lives in this workgroup: combine in LDS, no global round trip
    publish(L.slab, true);
    PROBE_TS(3);
    PROBE_TS(4);
  } else {
    publish(tree.slabs[0] + static_cast<int64_t>(loc.first + loc.chunk_idx) * E, false);
    PROBE_TS(3);
    // deferred root: root_finalize_kernel sums this cell's item slabs, spread over workgroups
    if (DEFER && nit <= kRootFanIn) return;
    const double *root;
    int32_t root_n;
    const bool last = tree_climb<E>(tree, loc.chunk_idx, nit, loc.first, cell, L.flag, &root,
                                    &root_n);
    PROBE_TS(4);
    if (!last) return;
    gather_root<E>(root, root_n, L.slab);
    PROBE_GATHERED();
  }
  finalize_cell<Sch>([&](int e) { return double2{L.slab[e], L.slab[e + 1]}; }, loc.cnt, T,
                     L.shift, L.S, o0, o1, mean, cov, L.mean, COV_IN_LDS ? L.cov : nullptr,
                     L.slab + Sch::GRAM);
  PROBE_TS(5);
  if (MINK)
    minkowski_cell(COV_IN_LDS ? L.cov : cov, L.mean, T, cell, L.ref, L.ref[rows],
                   L.ref[rows + 1], L.ref[rows + 2], mp, L.lb, threadIdx.x, blockDim.x);
  PROBE_TS(6);
}

// Per-wave share of an item's particles [a, b): contiguous quota ranges (power-of-two items,
// quota wq) or, in balanced mode, load groups of GS particles dealt round-robin to the NW
// waves (every wave within one group of the others, whatever the chunk).
struct WaveRange {
  int64_t p0, stride, p1, ngroups;
};
template <bool BAL>
__device__ __forceinline__ WaveRange wave_range(int64_t a, int64_t b, int w, int nw, int64_t wq,
                                                int64_t gs) {
  WaveRange r;
  if (BAL) {
    r.p0 = a + static_cast<int64_t>(w) * gs;
    r.stride = nw * gs;
    r.p1 = b;
    r.ngroups = r.p0 < b ? ceil_div(b - r.p0, r.stride) : 0;
  } else {
    r.p0 = a + static_cast<int64_t>(w) * wq;
    r.stride = gs;
    r.p1 = (r.p0 + wq < b) ? r.p0 + wq : b;
    r.ngroups = r.p1 > r.p0 ? ceil_div(r.p1 - r.p0, gs) : 0;
  }
  return r;
}

// The per-cell inputs of the half-space tail: issued at an item's start, landing behind its
// stream loop (thread i < 2T: ref_traj row, then the 3 risk constants).
__device__ __forceinline__ double prefetch_tail(const MinkParams &mp, const ItemLoc &loc,
                                                int rows) {
  if (threadIdx.x < rows) return mp.ref_traj[static_cast<int64_t>(loc.ref_sel) * rows + threadIdx.x];
  if (threadIdx.x < rows + 3) return mp.cell_risk[3 * loc.cell + (threadIdx.x - rows)];
  return 0.0;
}

template <typename P, int RB, bool MINK, bool BAL>
// The fused half-space tail needs a few more registers than the 128 of 4 waves/SIMD at RB = 1.
__global__ __launch_bounds__(Geo<RB>::NW * 64,
                             (MINK && RB == 1) ? 3 : Geo<RB>::MIN_WAVES_PER_SIMD)
void moments_kernel(
    const int64_t *__restrict__ cell_cnt, const int64_t *__restrict__ cell_off,
    const int32_t *__restrict__ cell_ref, int n_cells, const P *__restrict__ pos, int64_t ld,
    int T, const double *__restrict__ origin, int lg_wq, TreeLayout tree,
    double *__restrict__ out_mean, double *__restrict__ out_cov, MinkParams mp,
    int64_t whole) {
  using G = Geo<RB>;
  constexpr int NT = n_tiles(RB);
  constexpr int NACC = G::NACC;
  constexpr int D = 16 * RB;
  constexpr int S = G::S;
  constexpr int W = RB >= 4 ? kWBig : 4;  // particles per lane per sub-step (LaneVec)
  constexpr int E = slab_doubles(RB);
  // the fused tail reads the covariance from LDS; it lives in the cross-wave exchange buffer,
  // which is free once the item is combined (so T = 40 keeps its 80 x 80 covariance on chip too)
  constexpr bool COV_IN_LDS = MINK;
  constexpr bool DEFER = defer_root(RB, MINK, BAL);
  constexpr int XCH = combine_xch_doubles(RB, G::NW) > (MINK ? D * D : 0)
                          ? combine_xch_doubles(RB, G::NW) : D * D;
  __shared__ double xch[XCH];
  __shared__ double slab_lds[E];
  __shared__ double shift_lds[D];
  __shared__ double S_lds[D];
  __shared__ double mean_lds[D];
  __shared__ double lb_s[MINK ? 40 * 39 / 2 : 1];
  __shared__ double ref_lds[MINK ? D + 3 : 1];  // reference trajectory [T][2], then risk[3]
  __shared__ int flag;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int rows = 2 * T;
  const int lg_chunk = lg_wq + lg_waves_per_item(RB);

  // one work item: the cell's particles [a, b) -> partial Gram -> combine tree / finalise
  auto item = [=](const ItemLoc &loc, int32_t nit, int64_t a, int64_t b) {
    const int r = lane & 15;
    const int g = lane >> 4;
    const int64_t cnt = loc.cnt;
    const double pre = MINK ? prefetch_tail(mp, loc, rows) : 0.0;
    // a whole-cell item longer than a chunk deals its load groups round-robin, as balanced
    // items do, so every wave streams ~1/NW of the cell
    const bool rr = BAL || (b - a > (int64_t(1) << lg_chunk));
    const WaveRange wr = rr ? wave_range<true>(a, b, w, G::NW, int64_t(1) << lg_wq, 4 * W * S)
                            : wave_range<false>(a, b, w, G::NW, int64_t(1) << lg_wq, 4 * W * S);
    const int64_t p1 = wr.p1;

    double sh[RB];
    const P *rowp[RB];
    bool live[RB];
#pragma unroll
    for (int bb = 0; bb < RB; ++bb) {
      const int R = 16 * bb + r;
      live[bb] = R < rows;
      rowp[bb] = pos + static_cast<int64_t>(live[bb] ? R : 0) * ld + loc.off;
      sh[bb] = (live[bb] && cnt > 0) ? static_cast<double>(rowp[bb][0]) : 0.0;
    }

    d4 acc[NACC][NT];
#pragma unroll
    for (int x = 0; x < NACC; ++x)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[x][t] = d4{0.0, 0.0, 0.0, 0.0};
    double s1[RB];
#pragma unroll
    for (int bb = 0; bb < RB; ++bb) s1[bb] = 0.0;

    // double-buffered load groups: the next group's loads are in flight during this group's
    // MFMAs.  The prefetch is unconditional (a group past the end is clamped + masked and
    // never multiplied) so there is no divergent join for the waitcnt pass to merge.
    // sched_barrier(0) fences keep the four phases in program order, so each MFMA group waits
    // (vmcnt) only for its own buffer while the other buffer's loads stay in flight.
    const int64_t ngroups = wr.ngroups, st = wr.stride;
#if CCMPC_PRIO  // experiment: static priority for the second-dispatched half (MI355X_MICROARCH.md)
    if (G::NW == 8 && w >= 4) __builtin_amdgcn_s_setprio(CCMPC_PRIO);
#endif
    constexpr int DP = RB >= 3 ? CCMPC_DEPTH_BIG : kDepth;
    typename LaneVec<P, W>::type buf[DP][S][RB];
    if (ngroups > 0) {
      // ring of DP load groups: group g lives in buf[g % DP]; DP - 1 groups are in flight
      // while one is multiplied
#pragma unroll
      for (int d = 0; d < DP - 1; ++d) load_group<P, RB, S, W>(buf[d], rowp, wr.p0 + d * st, p1, g);
      int64_t gi = 0;
      for (; gi + DP <= ngroups; gi += DP) {
        if (BAL) progress_prio(gi, ngroups);
#pragma unroll
        for (int d = 0; d < DP; ++d) {
          load_group<P, RB, S, W>(buf[(d + DP - 1) % DP], rowp, wr.p0 + (gi + d + DP - 1) * st, p1,
                               g);
          __builtin_amdgcn_sched_barrier(0);
          mfma_group<P, RB, S, NACC, W>(buf[d], sh, live, wr.p0 + (gi + d) * st, p1, g, acc, s1);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int d = 0; d < DP - 1; ++d)  // the < DP groups left were loaded ahead
        if (gi + d < ngroups)
          mfma_group<P, RB, S, NACC, W>(buf[d], sh, live, wr.p0 + (gi + d) * st, p1, g, acc, s1);
    }
    PROBE_TS(2);
#if CCMPC_PRIO || CCMPC_PROGRESS_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif

    if (MINK && threadIdx.x < rows + 3) ref_lds[threadIdx.x] = pre;  // read after barriers below
#pragma unroll
    for (int bb = 0; bb < RB; ++bb) {
      if (w == 0 && g == 0) shift_lds[16 * bb + r] = sh[bb];
    }
    const EpilogueLds L{slab_lds, shift_lds, S_lds, mean_lds, xch, lb_s, ref_lds, &flag};
    cell_epilogue<Scheme16<RB>, MINK, COV_IN_LDS, DEFER>(
        [&](double *dst, bool to_lds) {
          combine_waves<RB, NACC, G::NW>(acc, s1, xch, dst, to_lds);
        },
        loc, nit, T, tree, origin, out_mean, out_cov, mp, L);
  };

  PROBE_TS(0);
  if (BAL) {
    ItemLoc loc;
    int64_t chunk;
    if (!locate_balanced(blockIdx.x, gridDim.x, cell_cnt, cell_off, n_cells, loc, &chunk,
                         cell_ref))
      return;  // uniform
    PROBE_TS(1);
    const int64_t i0 = static_cast<int64_t>(loc.chunk_idx) * chunk;
    item(loc, static_cast<int32_t>(loc.cnt > 0 ? ceil_div_fast(loc.cnt, chunk) : 1), i0,
         min(i0 + chunk, loc.cnt));
    return;
  }
  ItemLoc loc;
  if (!locate_item(blockIdx.x, cell_cnt, cell_off, n_cells, lg_chunk, loc,
                   cell_ref, whole))
    return;  // uniform
  PROBE_TS(1);
  const int32_t nit = items_of(loc.cnt, lg_chunk, whole);
  const int64_t i0 = static_cast<int64_t>(loc.chunk_idx) << lg_chunk;
  const int64_t i1 = nit == 1 ? loc.cnt : min(i0 + (int64_t(1) << lg_chunk), loc.cnt);
  item(loc, nit, i0, i1);
}

// ---- Scheme4: f64 4x4x4_4b MFMA over 4-row blocks (T <= 12) -------------------------------
// Lane l holds row 4I + (l & 3) of block I for the 2 consecutive particles base + 2m, +1
// (m = l >> 2; one 16-byte load per block, so a row's 16 lanes read 256 contiguous bytes and
// an instruction covers whole lines).  Sub-step j feeds particle base + 2m + j: m = b + 4k is
// the instruction's A[b][i][k] lane i + 4b + 16k, so ONE register per block is both the A
// and the B operand of every block pair (I, J), as for the 16x16 tiles.  A group is 32
// particles per wave.
// Scheme4's per-lane row load is 16 bytes in either store type: 2 doubles, or 4 floats
// (CCMPC_F32_WIDE4).  A group is then 16 W particles per wave -- 32 (f64) or 64 (f32) -- so a
// load ring of the same depth keeps the same BYTES in flight for both stores.  With f32 pairs
// (8 bytes, 32-particle groups) the f32 store had half the bytes in flight and streamed at half
// the f64 byte rate: the per-GPU C4 batch took as long on half the bytes (r04 verdict).
#ifndef CCMPC_F32_WIDE4
#define CCMPC_F32_WIDE4 1
#endif
template <typename P>
struct Row4 {  // double (and float without CCMPC_F32_WIDE4): one 16 / 8-byte pair per row
  using type = Pair<P>;
  static constexpr int W = 2;
  __device__ static void load(const P *p, type &q) { load_pair(p, q); }
};
#if CCMPC_F32_WIDE4
template <>
struct Row4<float> {
  using type = Quad<float>;
  static constexpr int W = 4;
  __device__ static void load(const float *p, type &q) {
    if constexpr (CCMPC_NT_PAIR != 0) {
      const ccmpc_f4v t = __builtin_nontemporal_load(reinterpret_cast<const ccmpc_f4v *>(p));
      q.v = make_float4(t.x, t.y, t.z, t.w);
    } else {
      q.v = *reinterpret_cast<const float4 *>(p);
    }
  }
};
#endif

template <typename P, int NB>
__device__ __forceinline__ void load_group4(typename Row4<P>::type (&v)[NB],
                                            const P *const (&rowp)[NB], int64_t gbase, int64_t p1,
                                            int m) {
  constexpr int W = Row4<P>::W;
  const int64_t qlast = (p1 - 1) & ~int64_t(W - 1);
  const int64_t q = gbase + W * m;
  const int64_t qc = q < qlast ? q : qlast;
#pragma unroll
  for (int I = 0; I < NB; ++I) Row4<P>::load(rowp[I] + qc, v[I]);
}

// Row-contiguous loads (CCMPC_ROWLOAD4): the matrix-core layout puts 4 rows in every 4
// consecutive lanes, so a load instruction in that layout walks 4 rows megabytes apart lane by
// lane and the address-translation unit sees one request per 16-byte lane (UTCL1 counters,
// profiles/r02/utcl1_counters_C4_C5.txt: 72M requests per C4 launch = one per 13.6 bytes).
// Instead, lane l loads row 4I + (l >> 4), particles 2 (l & 15) + {0, 1}: 16 lanes cover 256
// contiguous bytes of one row.  One ds_bpermute per dword then hands lane (c + 4 m) the value
// of lane (16 c + m).  Measured (profiles/r02/ab10_rowload4.log): the 64-scene C4 batch 212.8
// -> 209.6 us cold, the per-GPU batch at 8 GPUs 33.9 -> 34.9 us warm -- so translation is not
// what holds the stream back; off by default, kept as a build knob.
#ifndef CCMPC_ROWLOAD4
#define CCMPC_ROWLOAD4 0
#endif
__device__ __forceinline__ double bperm_f64(int addr, double x) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = static_cast<uint32_t>(
      __builtin_amdgcn_ds_bpermute(addr, static_cast<int>(static_cast<uint32_t>(u))));
  const uint32_t hi = static_cast<uint32_t>(
      __builtin_amdgcn_ds_bpermute(addr, static_cast<int>(static_cast<uint32_t>(u >> 32))));
  return __builtin_bit_cast(double, (static_cast<uint64_t>(hi) << 32) | lo);
}
__device__ __forceinline__ float bperm_f32(int addr, float x) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_ds_bpermute(addr, __builtin_bit_cast(int, x)));
}
__device__ __forceinline__ Pair<double> bperm_pair(int addr, const Pair<double> &p) {
  Pair<double> r;
  r.v.x = bperm_f64(addr, p.v.x);
  r.v.y = bperm_f64(addr, p.v.y);
  return r;
}
__device__ __forceinline__ Pair<float> bperm_pair(int addr, const Pair<float> &p) {
  Pair<float> r;
  r.v.x = bperm_f32(addr, p.v.x);
  r.v.y = bperm_f32(addr, p.v.y);
  return r;
}

template <typename P, int NB>
__device__ __forceinline__ void mfma_group4(const typename Row4<P>::type (&loaded)[NB],
                                            const double (&sh)[NB], const bool (&live)[NB],
                                            int64_t gbase, int64_t p1, int m, int paddr,
                                            double (&acc)[n_pairs(NB)], double (&s1)[NB]) {
  constexpr int W = Row4<P>::W;
  const int64_t q = gbase + W * m;
#if CCMPC_ROWLOAD4
  static_assert(W == 2, "CCMPC_ROWLOAD4 is the pair layout");
  Pair<P> raw[NB];
#pragma unroll
  for (int I = 0; I < NB; ++I) raw[I] = bperm_pair(paddr, loaded[I]);
#else
  const typename Row4<P>::type(&raw)[NB] = loaded;
  (void)paddr;
#endif
#pragma unroll
  for (int j = 0; j < W; ++j) {
    double v[NB];  // sub-step j: shifted; out-of-range slots and dead rows become 0
#pragma unroll
    for (int I = 0; I < NB; ++I) {
#if CCMPC_PROBE & 32
      v[I] = raw[I][j] - sh[I];
#elif CCMPC_PROBE & 64
      v[I] = raw[I][j];
#else
      v[I] = (live[I] && q + j < p1) ? raw[I][j] - sh[I] : 0.0;
#endif
      s1[I] += v[I];
    }
    int p = 0;
#pragma unroll
    for (int I = 0; I < NB; ++I)
#pragma unroll
      for (int J = I; J < NB; ++J) {
        acc[p] = __builtin_amdgcn_mfma_f64_4x4x4f64(v[I], v[J], acc[p], 0, 0, 0);
        ++p;
      }
  }
}

#ifndef CCMPC_NW4  // waves per Scheme4 work item (build knob)
#define CCMPC_NW4 4
#endif
constexpr int kNW4 = CCMPC_NW4;
#ifndef CCMPC_M4_OCC  // Scheme4 workgroups per CU the register budget must allow (build knob)
#define CCMPC_M4_OCC(NB) (((NB) <= 5 ? 3 : 2) * 4 / kNW4 > 0 ? ((NB) <= 5 ? 3 : 2) * 4 / kNW4 : 1)
#endif
#ifndef CCMPC_M4_OCC_F32  // ... for the f32 store (0: as f64)
#define CCMPC_M4_OCC_F32 0
#endif
template <typename P>
constexpr int m4_occ(int nb) {
  return std::is_same_v<P, float> && CCMPC_M4_OCC_F32 > 0 ? CCMPC_M4_OCC_F32 : CCMPC_M4_OCC(nb);
}

template <typename P, int NB, bool MINK, bool BAL>
__global__ __launch_bounds__(kNW4 * 64, m4_occ<P>(NB)) void moments4_kernel(
    const int64_t *__restrict__ cell_cnt, const int64_t *__restrict__ cell_off,
    const int32_t *__restrict__ cell_ref, int n_cells, const P *__restrict__ pos, int64_t ld,
    int T, const double *__restrict__ origin, int lg_wq, TreeLayout tree,
    double *__restrict__ out_mean, double *__restrict__ out_cov, MinkParams mp) {
  using Sch = Scheme4<NB>;
  constexpr int NP = Sch::NP, D = Sch::D, E = Sch::E;
  __shared__ double xch[kNW4 * Combine4Layout<NB>::XS];
  __shared__ double slab_lds[E];
  __shared__ double shift_lds[D];
  __shared__ double S_lds[D];
  __shared__ double mean_lds[D];
  __shared__ double lb_s[MINK ? 12 * 11 / 2 : 1];
  __shared__ double ref_lds[MINK ? D + 3 : 1];  // reference trajectory [T][2], then risk[3]
  __shared__ int flag;

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  const int rows = 2 * T;
  const int lg_chunk = lg_wq + 2;

  auto item = [=](const ItemLoc &loc, int32_t nit, int64_t a, int64_t b) {
    const int c = lane & 3, m = lane >> 2;
#if CCMPC_ROWLOAD4
    const int rl = lane >> 4, ml = lane & 15;  // the loading lane's row in the block, pair
#else
    const int rl = c, ml = m;
#endif
    const int paddr = 4 * (16 * c + m);        // matrix lane (c, m) <- loading lane 16 c + m
    const int64_t cnt = loc.cnt;
    const double pre = MINK ? prefetch_tail(mp, loc, rows) : 0.0;
    const WaveRange wr = wave_range<BAL>(a, b, w, kNW4, int64_t(1) << lg_wq, 16 * Row4<P>::W);
    const int64_t p1 = wr.p1;

    double sh[NB];
    const P *rowp[NB];  // the loading lane's rows (dead rows clamped to row 0)
    bool live[NB];      // the matrix lane's rows
#pragma unroll
    for (int I = 0; I < NB; ++I) {
      const int R = 4 * I + c, RL = 4 * I + rl;
      live[I] = R < rows;
      rowp[I] = pos + static_cast<int64_t>(RL < rows ? RL : 0) * ld + loc.off;
      sh[I] = (live[I] && cnt > 0)
                  ? static_cast<double>(pos[static_cast<int64_t>(R) * ld + loc.off]) : 0.0;
    }
    double acc[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) acc[p] = 0.0;
    double s1[NB];
#pragma unroll
    for (int I = 0; I < NB; ++I) s1[I] = 0.0;

    const int64_t ngroups = wr.ngroups, st = wr.stride;
    constexpr int DP = BAL ? (std::is_same_v<P, float> ? kDepth4BalF32 : kDepth4Bal) : kDepth4;
    typename Row4<P>::type buf[DP][NB];
    if (ngroups > 0) {
#pragma unroll
      for (int d = 0; d < DP - 1; ++d) load_group4<P, NB>(buf[d], rowp, wr.p0 + d * st, p1, ml);
      int64_t gi = 0;
      for (; gi + DP <= ngroups; gi += DP) {
        if (BAL) progress_prio(gi, ngroups);
#pragma unroll
        for (int d = 0; d < DP; ++d) {
          load_group4<P, NB>(buf[(d + DP - 1) % DP], rowp, wr.p0 + (gi + d + DP - 1) * st, p1, ml);
          __builtin_amdgcn_sched_barrier(0);
          mfma_group4<P, NB>(buf[d], sh, live, wr.p0 + (gi + d) * st, p1, m, paddr, acc, s1);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int d = 0; d < DP - 1; ++d)
        if (gi + d < ngroups)
          mfma_group4<P, NB>(buf[d], sh, live, wr.p0 + (gi + d) * st, p1, m, paddr, acc, s1);
    }
    PROBE_TS(2);
#if CCMPC_PROGRESS_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif

    if (MINK && threadIdx.x < rows + 3) ref_lds[threadIdx.x] = pre;  // read after barriers below
#pragma unroll
    for (int I = 0; I < NB; ++I)
      if (w == 0 && m == 0) shift_lds[4 * I + c] = sh[I];
    // the covariance for the tail reuses the exchange buffer (free after combine4)
    static_assert(kNW4 * Combine4Layout<NB>::XS >= D * D, "xch must hold the covariance");
    const EpilogueLds L{slab_lds, shift_lds, S_lds, mean_lds, xch, lb_s, ref_lds, &flag};
    cell_epilogue<Sch, MINK, MINK, false>(
        [&](double *dst, bool to_lds) { combine4<NB, kNW4>(acc, s1, xch, dst, to_lds); }, loc,
        nit, T, tree, origin, out_mean, out_cov, mp, L);
  };

  PROBE_TS(0);
  if (BAL) {
    ItemLoc loc;
    int64_t chunk;
    if (!locate_balanced(blockIdx.x, gridDim.x, cell_cnt, cell_off, n_cells, loc, &chunk,
                         cell_ref))
      return;  // uniform
    PROBE_TS(1);
    const int64_t i0 = static_cast<int64_t>(loc.chunk_idx) * chunk;
    item(loc, static_cast<int32_t>(loc.cnt > 0 ? ceil_div_fast(loc.cnt, chunk) : 1), i0,
         min(i0 + chunk, loc.cnt));
    return;
  }
  ItemLoc loc;
  if (!locate_item(blockIdx.x, cell_cnt, cell_off, n_cells, lg_chunk, loc,
                   cell_ref))
    return;  // uniform
  PROBE_TS(1);
  const int64_t i0 = static_cast<int64_t>(loc.chunk_idx) << lg_chunk;
  const int64_t i1 = min(i0 + (int64_t(1) << lg_chunk), loc.cnt);
  item(loc, items_of(loc.cnt, lg_chunk), i0, i1);
}

// A balanced launch's cell -> (first item, item count), as locate_balanced deals them (same
// chunk from the same exact count sum).  Every lane of the wave gets the result.
__device__ __forceinline__ void cell_items_balanced(int cell, int G, const int64_t *__restrict__ cnt,
                                                    int n_cells, int32_t &first, int32_t &nit,
                                                    int64_t &n) {
  const int lane = threadIdx.x & 63;
  double part = 0.0;  // exact: counts and their sum < 2^53
  for (int base = 0; base < n_cells; base += 64)
    part += base + lane < n_cells ? static_cast<double>(cnt[base + lane]) : 0.0;
  const double td = wave_sum_dpp_f64(part);
  const int64_t n0 = lane < n_cells ? cnt[lane] : 0, n1 = lane + 64 < n_cells ? cnt[lane + 64] : 0;
  const int64_t chunk = balanced_chunk(td, G, n_cells, n0, n1);
  int32_t before = 0;
  first = 0;
  nit = 0;
  n = 0;
  for (int base = 0; base < n_cells; base += 64) {
    const int c = base + lane;
    const int64_t nn = c < n_cells ? cnt[c] : 0;
    const int32_t mine =
        c < n_cells ? static_cast<int32_t>(nn > 0 ? ceil_div_fast(nn, chunk) : 1) : 0;
    const int32_t incl = wave_incl_scan_i32(mine);
    if (cell < base + 64) {
      const int l = cell - base;
      first = before + lane_i32(incl - mine, l);
      nit = lane_i32(mine, l);
      n = lane_i64(nn, l);
      return;
    }
    before += lane_i32(incl, 63);
  }
}

// The deferred root (defer_root): one workgroup per (cell, 16x16 tile).  The root gather sums
// a cell's slabs in groups of kFanIn (sum_group2) and adds the group sums in order; here each of
// the <= kRootFanIn / kFanIn groups is a thread of its own (group q of entry pair k: thread
// q * 128 + k for the tile's 128 pairs, then the row-sum pairs), every load of the cell in flight
// in one round, and the group sums are added in LDS in the same order: the same bits.  Then the
// tile's covariance entries (and, in tile 0, the mean) by finalize_cell's expressions.  Cells of
// one item were finalised by the moments launch, cells past kRootFanIn items by its combine tree.
constexpr int kRootGroups = kRootFanIn / kFanIn;
static_assert(kRootGroups * kFanIn == kRootFanIn, "root = whole fan-in groups");
template <int RB>
struct RootGeo {
  static constexpr int D = 16 * RB;
  static constexpr int PAIRS = 128 + D / 2;               // tile pairs, then row-sum pairs
  static constexpr int GATHER = kRootGroups * PAIRS;      // gather threads
  static constexpr int THREADS = (GATHER + D + 63) / 64 * 64;  // + the shift loads
  // a CCMPC_ROOT_FANIN build knob too wide for one workgroup must fail here, not at launch
  static_assert(THREADS <= 1024, "deferred root: kRootFanIn too wide for one workgroup");
  static_assert(sizeof(double2) * kRootGroups * PAIRS + 2 * sizeof(double) * D <= 64 * 1024,
                "deferred root: LDS partials exceed the static 64 KiB");
};
template <typename P, int RB>
__global__ __launch_bounds__(RootGeo<RB>::THREADS) void root_finalize_kernel(
    const int64_t *__restrict__ cell_cnt, const int64_t *__restrict__ cell_off, int n_cells, int G,
    const P *__restrict__ pos, int64_t ld, int T, const double *__restrict__ origin,
    const double *__restrict__ slabs0, double *__restrict__ out_mean,
    double *__restrict__ out_cov) {
  using RG = RootGeo<RB>;
  constexpr int NT = n_tiles(RB), D = RG::D, E = slab_doubles(RB), GRAM = NT * 256;
  constexpr int PAIRS = RG::PAIRS;
  __shared__ double2 part[kRootGroups][PAIRS];
  __shared__ double S_lds[D];
  __shared__ double shift_lds[D];
  const int cell = blockIdx.x / NT, tile = blockIdx.x % NT, tid = threadIdx.x;
  const int rows = 2 * T;
  int32_t first, nit;
  int64_t cnt;
  cell_items_balanced(cell, G, cell_cnt, n_cells, first, nit, cnt);
  if (nit <= 1 || nit > kRootFanIn) return;  // uniform
  if (tid < RG::GATHER) {
    const int q = tid / PAIRS, k = tid % PAIRS;
    const int e = k < 128 ? tile * 256 + 2 * k : GRAM + 2 * (k - 128);
    const bool live = q * kFanIn < nit && (k < 128 || 2 * (k - 128) < rows);
    if (live)
      part[q][k] = sum_group2(slabs0 + static_cast<int64_t>(first + q * kFanIn) * E,
                              min(nit - q * kFanIn, kFanIn), E, e);
  } else if (tid < RG::GATHER + D) {
    const int r = tid - RG::GATHER;
    shift_lds[r] = r < rows ? static_cast<double>(pos[static_cast<int64_t>(r) * ld +
                                                      cell_off[cell]])
                            : 0.0;
  }
  __syncthreads();
  const int ng = (nit + kFanIn - 1) / kFanIn;
  auto total = [&](int k) {  // gather_root's order: group 0, then += group 1, 2, ...
    double2 s = part[0][k];
    for (int q = 1; q < ng; ++q) {
      s.x += part[q][k].x;
      s.y += part[q][k].y;
    }
    return s;
  };
  if (tid >= 128 && tid < PAIRS) {
    const int r = 2 * (tid - 128);
    const double2 s = r < rows ? total(tid) : double2{0.0, 0.0};
    S_lds[r] = s.x;
    S_lds[r + 1] = s.y;
  }
  __syncthreads();
  const double n = static_cast<double>(cnt);
  if (tile == 0 && tid < rows) {
    const double o = origin ? origin[2 * cell + (tid & 1)] : 0.0;
    out_mean[static_cast<int64_t>(cell) * rows + tid] = (shift_lds[tid] + S_lds[tid] / n) + o;
  }
  if (tid >= 128) return;
  const int e = tile * 256 + 2 * tid;
  int i0, j0, i1, j1;
  decode_entry(e, RB, i0, j0);
  decode_entry(e + 1, RB, i1, j1);
  const bool use0 = i0 < rows && j0 < rows && i0 <= j0;
  const bool use1 = i1 < rows && j1 < rows && i1 <= j1;
  if (!use0 && !use1) return;
  const double2 g = total(tid);
  double *cov = out_cov + static_cast<int64_t>(cell) * rows * rows;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (!(h ? use1 : use0)) continue;
    const int i = h ? i1 : i0, j = h ? j1 : j0;
    const double c = ((h ? g.y : g.x) - S_lds[i] * S_lds[j] / n) / (n - 1.0);
    cov[i * rows + j] = c;
    cov[j * rows + i] = c;
  }
}

// Whole-cell items (T <= 8, tiny inputs): a cell of up to CCMPC_WHOLE_CELL_MAX particles is
// one workgroup's item, combined in LDS -- no slab, arrival or root gather.  One CU's f64 matrix
// pipes then do the whole cell's Gram (16 x 16 tile per 4 particles, ~1.8 ns per particle), so
// this pays only for small cells (profiles/r05/ab_whole_cell_cap.log, C2 / C3 cycle, us):
//   cap      0      1024   1536   2048   3072   4096
//   C2       11.3   11.4   12.8   13.9   17.6   19.1     (its 5000-particle cell sets the path)
//   C3 1e3   10.5    9.7    9.8    9.7    9.7    9.7
// Build knob (0 = off).
#ifndef CCMPC_WHOLE_CELL_MAX
#define CCMPC_WHOLE_CELL_MAX 1024
#endif
inline int64_t whole_cell_max(int rb, int64_t n_bound) {
  return (rb == 1 && n_bound <= (int64_t(1) << CCMPC_LG_TINY_INPUT)) ? CCMPC_WHOLE_CELL_MAX : 0;
}

template <typename P, int RB, bool MINK>
static int launch(const P *pos, int64_t ld, int T, const double *origin, const int64_t *off,
                  const int64_t *cnt, int n_cells, int64_t n_bound, void *ws, size_t ws_bytes,
                  double *mean, double *cov, const MinkParams &mp, hipStream_t s) {
  constexpr int threads = Geo<RB>::NW * 64;
  const int lg_wq = store_lg_wave_quota(RB, n_bound);
  TreeLayout tree;
  const int grid =
      balanced_mode(n_bound) ? resident_grid<moments_kernel<P, RB, MINK, true>>(threads) : 0;
  if (grid > 0 && 2 * n_cells <= grid) {
    if (!tree_layout(ws, ws_bytes, balanced_max_items(threads), n_cells, slab_doubles(RB),
                     tree))
      return CCMPC_ERR_WORKSPACE;
    hipLaunchKernelGGL((moments_kernel<P, RB, MINK, true>), dim3(static_cast<unsigned>(grid)),
                       dim3(threads), 0, s, cnt, off, MINK ? mp.cell_ref : nullptr, n_cells, pos, ld,
                       T, origin, lg_wq, tree, mean, cov, mp, int64_t(0));
    if (defer_root(RB, MINK, true))
      hipLaunchKernelGGL((root_finalize_kernel<P, RB>),
                         dim3(static_cast<unsigned>(n_cells * n_tiles(RB))), dim3(RootGeo<RB>::THREADS), 0,
                         s, cnt, off, n_cells, grid, pos, ld, T, origin, tree.slabs[0], mean, cov);
    return CCMPC_OK;
  }
  const int64_t items = max_items(n_cells, n_bound, int64_t(1) << store_lg_chunk(RB, n_bound));
  if (!tree_layout(ws, ws_bytes, items, n_cells, slab_doubles(RB), tree)) return CCMPC_ERR_WORKSPACE;
  hipLaunchKernelGGL((moments_kernel<P, RB, MINK, false>), dim3(static_cast<unsigned>(items)),
                     dim3(threads), 0, s, cnt, off, MINK ? mp.cell_ref : nullptr, n_cells, pos, ld, T,
                     origin, lg_wq, tree, mean, cov, mp, whole_cell_max(RB, n_bound));
  return CCMPC_OK;
}

template <typename P, int NB, bool MINK>
static int launch4(const P *pos, int64_t ld, int T, const double *origin, const int64_t *off,
                   const int64_t *cnt, int n_cells, int64_t n_bound, void *ws, size_t ws_bytes,
                   double *mean, double *cov, const MinkParams &mp, hipStream_t s) {
  constexpr int threads = kNW4 * 64;
  const int lg_wq = store_lg_wave_quota(1, n_bound);
  TreeLayout tree;
  const int grid =
      balanced_mode(n_bound) ? resident_grid<moments4_kernel<P, NB, MINK, true>>(threads) : 0;
  if (grid > 0 && 2 * n_cells <= grid) {
    if (!tree_layout(ws, ws_bytes, balanced_max_items(threads), n_cells, Scheme4<NB>::E,
                     tree))
      return CCMPC_ERR_WORKSPACE;
    hipLaunchKernelGGL((moments4_kernel<P, NB, MINK, true>), dim3(static_cast<unsigned>(grid)),
                       dim3(threads), 0, s, cnt, off, MINK ? mp.cell_ref : nullptr, n_cells, pos, ld,
                       T, origin, lg_wq, tree, mean, cov, mp);
    return CCMPC_OK;
  }
  const int64_t items = max_items(n_cells, n_bound, int64_t(1) << (lg_wq + 2));
  if (!tree_layout(ws, ws_bytes, items, n_cells, Scheme4<NB>::E, tree)) return CCMPC_ERR_WORKSPACE;
  hipLaunchKernelGGL((moments4_kernel<P, NB, MINK, false>), dim3(static_cast<unsigned>(items)),
                     dim3(threads), 0, s, cnt, off, MINK ? mp.cell_ref : nullptr, n_cells, pos, ld, T,
                     origin, lg_wq, tree, mean, cov, mp);
  return CCMPC_OK;
}

// Scheme4 (4-row blocks) where 16-row tiles would pad heavily: T = 9..12 (18-24 rows in two
// 16-row blocks; C4 at T = 12: 30 -> 38 us moments-only with Scheme16).  At T <= 8 the 16 rows
// fill one tile exactly and Scheme16's cheaper combine wins (C2: 11.7 vs 12.5 us); above
// T = 12 the block-pair accumulators outgrow the register file.
inline int scheme4_blocks(int64_t T) {
  return (T > 8 && T <= 12) ? static_cast<int>((2 * T + 3) / 4) : 0;
}

template <typename P, bool MINK>
static int dispatch(const P *pos, int64_t ld, int T, const double *origin, const int64_t *off,
                    const int64_t *cnt, int n_cells, int64_t n_bound, void *ws, size_t ws_bytes,
                    double *mean, double *cov, const MinkParams &mp, hipStream_t s) {
#define CCMPC_ARGS pos, ld, T, origin, off, cnt, n_cells, n_bound, ws, ws_bytes, mean, cov, mp, s
  switch (scheme4_blocks(T)) {
    case 1: return launch4<P, 1, MINK>(CCMPC_ARGS);
    case 2: return launch4<P, 2, MINK>(CCMPC_ARGS);
    case 3: return launch4<P, 3, MINK>(CCMPC_ARGS);
    case 4: return launch4<P, 4, MINK>(CCMPC_ARGS);
    case 5: return launch4<P, 5, MINK>(CCMPC_ARGS);
    case 6: return launch4<P, 6, MINK>(CCMPC_ARGS);
    default: break;
  }
  switch (row_blocks(T)) {
    case 1: return launch<P, 1, MINK>(CCMPC_ARGS);
    case 2: return launch<P, 2, MINK>(CCMPC_ARGS);
    case 3: return launch<P, 3, MINK>(CCMPC_ARGS);
    case 4: return launch<P, 4, MINK>(CCMPC_ARGS);
    case 5: return launch<P, 5, MINK>(CCMPC_ARGS);
    default: return CCMPC_ERR_UNSUPPORTED;
  }
#undef CCMPC_ARGS
}

#ifndef CCMPC_SPLIT_TAIL_T  // ccmpc_minkowski_cycle above this T: moments, then the rows launch
#define CCMPC_SPLIT_TAIL_T 24
#endif
constexpr int kSplitTailT = CCMPC_SPLIT_TAIL_T;

template <bool MINK>
static int run(const void *positions, int dtype, int64_t ld, int64_t T, const double *origin,
               const int64_t *cell_off, const int64_t *cell_cnt, int64_t n_cells,
               int64_t n_bound, void *workspace, size_t ws_bytes, double *out_mean,
               double *out_cov, const MinkParams &mp, ccmpc_stream_t stream, const char *who) {
  hipStream_t s = as_stream(stream);
  const int Ti = static_cast<int>(T), nc = static_cast<int>(n_cells);
  if (MINK && T > kSplitTailT) {
    // long horizons: the moments launch, then the half-spaces as a launch of their own with one
    // wave per (cell, t) -- the fused tail runs T(T-1)/2 chains on the cell's one finalising
    // workgroup (T = 40: 780 chains, two rounds, ~12 us), while this runs every row at once.
    // Same device functions on the same covariance values, so the same records.
    const int rc = run<false>(positions, dtype, ld, T, origin, cell_off, cell_cnt, n_cells,
                              n_bound, workspace, ws_bytes, out_mean, out_cov, mp, stream, who);
    if (rc != CCMPC_OK) return rc;
    launch_minkowski_rows(out_mean, out_cov, Ti, nc, mp, s);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      set_error(std::string(who) + ": launch failed: " + hipGetErrorString(e));
      return CCMPC_ERR_LAUNCH;
    }
    return CCMPC_OK;
  }
  int rc;
  if (dtype == CCMPC_F64)
    rc = dispatch<double, MINK>(static_cast<const double *>(positions), ld, Ti, origin, cell_off,
                                cell_cnt, nc, n_bound, workspace, ws_bytes, out_mean, out_cov, mp,
                                s);
  else
    rc = dispatch<float, MINK>(static_cast<const float *>(positions), ld, Ti, origin, cell_off,
                               cell_cnt, nc, n_bound, workspace, ws_bytes, out_mean, out_cov, mp,
                               s);
  if (rc != CCMPC_OK) {
    set_error(std::string(who) + (rc == CCMPC_ERR_WORKSPACE ? ": workspace too small"
                                                            : ": unsupported T"));
    return rc;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(who) + ": launch failed: " + hipGetErrorString(e));
    return CCMPC_ERR_LAUNCH;
  }
  return CCMPC_OK;
}

}  // namespace ccmpc

using namespace ccmpc;

#if CCMPC_PROBE & 4
extern "C" int ccmpc_probe_timestamps(void *host, int reset) {
  const size_t bytes = sizeof(g_probe_ts);
  if (reset) {
    static unsigned long long zeros[kProbeMaxWG * kProbeSlots];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_probe_ts), zeros, bytes) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_probe_ts), bytes) == hipSuccess ? 0 : -1;
}
#endif

extern "C" size_t ccmpc_moments_workspace_bytes(int64_t T, int64_t n_cells,
                                                int64_t n_particles_bound) {
  if (T < 1 || T > kMaxT || n_cells < 0 || n_particles_bound < 0) return 0;
  // balanced mode (<= the resident grid) when the launch picks it, else power-of-two items
  const bool bal = balanced_mode(n_particles_bound);
  const int nb = scheme4_blocks(T);
  if (nb > 0) {
    int64_t items = max_items(n_cells, n_particles_bound,
                              int64_t(1) << (store_lg_wave_quota(1, n_particles_bound) + 2));
    if (bal) items = std::max(items, balanced_max_items(kNW4 * 64));
    return tree_bytes(items, n_cells, n_pairs(nb) * 16 + 4 * nb);
  }
  const int rb = row_blocks(T);
  int64_t items =
      max_items(n_cells, n_particles_bound, int64_t(1) << store_lg_chunk(rb, n_particles_bound));
  if (bal) items = std::max(items, balanced_max_items((1 << lg_waves_per_item(rb)) * 64));
  return tree_bytes(items, n_cells, slab_doubles(rb));
}

#define CHECK_STORE_ARGS()                                                                     \
  CCMPC_REQUIRE(T >= 1 && T <= kMaxT, "T must be in [1, 40]");                                 \
  CCMPC_REQUIRE(n_cells >= 0 && n_cells < (1 << 30), "bad n_cells");                           \
  if (n_cells == 0) return CCMPC_OK;                                                           \
  CCMPC_REQUIRE(positions && cell_off && cell_cnt && out_mean && out_cov, "null pointer");     \
  CCMPC_REQUIRE(ld % 4 == 0 && ld > 0, "ld must be a positive multiple of 4");                 \
  CCMPC_REQUIRE(dtype == CCMPC_F64 || dtype == CCMPC_F32, "bad dtype");                        \
  CCMPC_REQUIRE(aligned(positions, 16), "positions must be 16-byte aligned");                  \
  CCMPC_REQUIRE(workspace && aligned(workspace, 16), "workspace must be 16-byte aligned");     \
  if (workspace_bytes < ccmpc_moments_workspace_bytes(T, n_cells, n_particles_bound)) {        \
    set_error(std::string(__func__) + ": workspace too small");                                \
    return CCMPC_ERR_WORKSPACE;                                                                \
  }

extern "C" int ccmpc_moments(const void *positions, int dtype, int64_t ld, int64_t T,
                             const double *origin, const int64_t *cell_off,
                             const int64_t *cell_cnt, int64_t n_cells,
                             int64_t n_particles_bound, void *workspace, size_t workspace_bytes,
                             double *out_mean, double *out_cov, ccmpc_stream_t stream) {
  CHECK_STORE_ARGS();
  const MinkParams none{};
  return run<false>(positions, dtype, ld, T, origin, cell_off, cell_cnt, n_cells,
                    n_particles_bound, workspace, workspace_bytes, out_mean, out_cov, none, stream,
                    "ccmpc_moments");
}

extern "C" int ccmpc_minkowski_cycle(const void *positions, int dtype, int64_t ld, int64_t T,
                                     const double *origin, const int64_t *cell_off,
                                     const int64_t *cell_cnt, int64_t n_cells,
                                     int64_t n_particles_bound, void *workspace,
                                     size_t workspace_bytes, const double *ref_traj,
                                     const int32_t *cell_ref, const double *cell_risk, double R,
                                     double tol, int32_t maxiter, double *out_mean,
                                     double *out_cov, ccmpc_halfspace *out_rec,
                                     double *out_prob_lower, ccmpc_stream_t stream) {
  CHECK_STORE_ARGS();
  CCMPC_REQUIRE(ref_traj && cell_risk && out_rec && out_prob_lower, "null pointer");
  CCMPC_REQUIRE(maxiter >= 1, "maxiter must be >= 1");
  const MinkParams mp{ref_traj, cell_ref, cell_risk, R, tol, maxiter, out_rec, out_prob_lower};
  return run<true>(positions, dtype, ld, T, origin, cell_off, cell_cnt, n_cells,
                   n_particles_bound, workspace, workspace_bytes, out_mean, out_cov, mp, stream,
                   "ccmpc_minkowski_cycle");
}

extern "C" int ccmpc_minkowski_cycle_args(const ccmpc_cycle_args *a) {
  CCMPC_REQUIRE(a, "null args");
  return ccmpc_minkowski_cycle(a->positions, a->dtype, a->ld, a->T, a->origin, a->cell_off,
                               a->cell_cnt, a->n_cells, a->n_particles_bound, a->workspace,
                               a->workspace_bytes, a->ref_traj, a->cell_ref, a->cell_risk, a->R,
                               a->tol, a->maxiter, a->out_mean, a->out_cov, a->out_rec,
                               a->out_prob_lower, a->stream);
}

extern "C" size_t ccmpc_cycle_args_size(void) { return sizeof(ccmpc_cycle_args); }
