// Sampler + bucketing in one placement pass: the drop-in step's do_prediction -> make_ovehicles
// (prediction.py:81-86, v8ideal/__init__.py:469-505, ovehicle.py:24-117), and the same placement
// for the reference's own predictor output (generate_vehicle_latents' predictions + z,
// prediction.py:93-105) instead of the sampler.
//
// What makes the sampler -> three-kernel bucketing form slow is not work but dependent memory
// round trips: each of bucket.hip's kernels re-reads the particles, exchanges partials through
// memory and ends, and the next starts cold (tools/probe_step.py: ~10 us per kernel).  Here:
//
//  P0 latents  one latent id per particle (Philox + CDF count, the injected z, or the predictor's
//              z, validated: make_ovehicles indexes a list by it) and each 64-particle group's
//              count per category -- kept mode k or "rare" -- plus every 512-particle block's
//              totals and its count of invalid ids.
//  P1 place    per block of 64 NCH particles (512 threads): the category counts before its own
//              groups and in total (the P0 block totals before its block and the few groups
//              before it inside it).  No exchange is needed to know where a kept mode's own
//              particles go: cell k of the OV starts at
//                  region + sum_{j < k} round4(n_j + R)       (R = the OV's rare count)
//              so it can take its n_j natives AND, in the worst case, every rare particle; its
//              natives go to  start_k + (natives of k before this block) + (rank in the block).
//              Then the sampler's two phases (actions in parallel, then the Unicycle chain, one
//              wave per 64 particles) -- or, for the predictor's output, the block's coordinate
//              run staged through LDS; the chain writes a native particle's 2T coordinates
//              straight into its cell, and a rare particle's into a rare list in sample order,
//              with its final position and latent id; and each group's kept-mode sums of the
//              final world positions (= one 64-particle centre group, bucket.hpp).
//  small clouds (N <= 8192 per OV):
//  P2 rares    per block of 256 rare-list slots: the centres in the canonical order (bucket.hpp,
//              so they equal bucket.hip's bit for bit), the key (owner, latent) of EVERY rare
//              particle of the OV -- a few KB of L2 reads -- counted per bin in LDS in total and
//              before the block's first slot, so the block knows each bin's start and its own
//              particles' stable ranks in sample order without any exchange; then the copy of
//              its rare particles' coordinates into the owners' cells after the natives.  Block
//              0 writes cell offsets, counts, pmf and centres.
//  large clouds (every rare key in every block would be R^2 / 256 keys -- 11 M at N = 100 000):
//  P2 keys     per block of 1024 rare-list slots: the centres (each superblock's partial sum
//              by its own thread, then the superblocks left to right: the canonical order), the
//              keys of its slots (kept for P3) and their histogram over the bins.
//  P3 copy     per block of 256 slots: every P2 block's histogram (a few KB) -> each bin's
//              total and its count before this block's P2 block; the keys of the slots before it
//              in that P2 block; then the bin starts, the stable ranks (a scan of each wave's 64
//              keys) and the copy into the owners' cells.  Block 0 writes cell offsets, counts
//              and pmf.
// (A single launch whose last arriving block ranked and copied every rare particle of the OV
// was measured at 120 us: that tail is one CU's serial work.)
//
// Each cell holds exactly what bucket.hip's does, in the same order (natives in sample order,
// then the rare latents ascending, each in sample order), so every later kernel -- whose work
// split is cell-relative -- gives the same bits.  Only where the cells start differs: the OV's
// region must have room for sum_k round4(n_k + R) <= K (N + 4) particles.
#include "bucket.hpp"
#include "sampler.hpp"

namespace ccmpc {

constexpr int kFusedMaxN = 8192;             // P2 rares (every rare key per block) up to here
constexpr int kWideMaxN = 1 << 18;            // the keys + copy form (P2 keys, P3 copy) up to here
constexpr int kFusedMaxBins = 512;
constexpr int kFP = 64;                       // particles per chain wave
constexpr int kFThreads = 512;                // 8 waves
constexpr int kFWaves = kFThreads / 64;
constexpr int kFGroups = kFusedMaxN / kFP;    // centre groups (P1 blocks) per OV at most
constexpr int kParSteps = 16;                 // P1: horizons whose step terms run in parallel
constexpr int kRThreads = 256;                // P2 / P3: rare-list slots per block (per thread 1)
constexpr int kKeySlots = 4 * kRThreads;      // P2 keys: rare-list slots per block
constexpr int kWideMaxSup = (kWideMaxN / kFP + kCentreSuper - 1) / kCentreSuper;
// P2: rare records each thread loads per round (kRThreads x this per round; the first round is
// issued with the kernel's other loads, so a rare list of up to that many takes no further
// round trip)
#ifndef CCMPC_RARE_BATCH
#define CCMPC_RARE_BATCH 8
#endif
constexpr int kRWaves = kRThreads / 64;
// per-OV header: tot[kMaxKept + 1] at h[0..], the int64 cell starts cstart[kMaxKept] at
// h + 2 * kMaxKept
constexpr int kHdrInts = 64;
// per-group / per-P0-block category counts: kept modes 0..K-1, then the rare count; a P0
// block's row also holds its count of invalid latent ids in the last slot
constexpr int kCntStride = 32;
constexpr int kBadSlot = kCntStride - 1;
static_assert(kMaxKept + 1 <= 2 * kMaxKept, "tot[] must end before the cell starts");
static_assert(4 * kMaxKept <= kHdrInts, "cell starts (int64) must fit the per-OV header");
static_assert(kCntStride >= kMaxKept + 2, "counts: one slot per kept mode + rare + invalid");
static_assert(kWideMaxSup <= 64, "P2 keys: the superblock sums of one mode fit one LDS row");
#if defined(CCMPC_PROBE) && (CCMPC_PROBE & 4)
__device__ unsigned long long g_fused_ts[5][kStepProbeWG * kStepProbeSlots];
#define FUSED_TS(kern, k) CCMPC_STEP_TS(g_fused_ts[kern], k)
#else
#define FUSED_TS(kern, k) CCMPC_STEP_TS(nullptr, k)
#endif

constexpr int kActCoef = 64 * 40 * 5 / 4;    // P1: per-latent coefficient floats per OV (P0)
constexpr int kSrcPred = 4;                   // P1's particle source: the predictor's output

// where P0's latent ids come from
constexpr int kZPhilox = 0;  // Philox inverse CDF of latent_cdf (the synthetic sampler mode)
constexpr int kZIn = 1;      // injected int32 z_in[o][N] (the sampler's per-particle mode)
constexpr int kZPred = 2;    // the predictor's z[rows[o]][N], int64 or int32 (list-index rules)

struct FusedArgs {
  // sampler (sampler.hip)
  const double *init_state, *latent_cdf;
  const float *gmm, *eps_in;
  const int32_t *z_in;
  int L, T;
  int64_t N;
  float dt;
  uint64_t seed;
  const uint64_t *seed_dev;
  uint32_t ov_base;
  // the predictor's output (ccmpc_bucket_predictions): pred[row][N][T][2], z[row][N]
  const float *pred;
  const void *zsrc;
  int z_bytes;
  const int32_t *rows;
  const uint64_t *ptrs;  // or in device memory: {pred, z} addresses, read at run time
  // bucketing (bucket.hip)
  const int32_t *keep_map, *n_kept, *cell_base;
  int max_k;
  const double *minpos;
  const int64_t *region;
  // workspace (each written by one launch and read by later ones: the kernel boundaries order
  // them, and nothing needs initialising)
  int32_t *zbuf;   // [n_ov][Npad]: latent ids (P0)
  int32_t *gcnt;   // [n_ov][G][kCntStride]: per 64-particle group category counts (P0)
  int32_t *bsum;   // [n_ov][nb0][kCntStride]: per 512-particle P0 block totals + invalid ids
  int32_t *hdr;    // [n_ov][kHdrInts]: category totals [K + 1], then cell starts (int64) [K]
  double *gpart;   // [n_ov][G][max_k][2]
  float *rinfo;    // [n_ov][Npad][4]: rare particle's final (x, y), latent id (bits), 0
  float *rstore;   // [n_ov][2T][Npad]: rare particles' coordinates, rare-list order
  int32_t *kbuf;   // [n_ov][Npad]: rare-list slot keys (P2 keys)
  int32_t *rhist;  // [n_ov][nkb][kFusedMaxBins]: each P2 keys block's bin histogram
  float *coef;     // [n_ov][kActCoef]: the per-latent GMM coefficient rows (P0 block 0)
  int64_t Npad;
  int G, nb0, nkb;
  // outputs
  int32_t *out_z;  // optional sample-order latent ids
  float *out;
  int64_t ld_out;
  int64_t *cell_off, *cell_cnt;
  double *cell_pmf, *init_center;
  int32_t *z_bad;  // optional [n_ov]: invalid latent ids per OV
  int wt;          // the particle stores may go write-through (every offset < 2^31 bytes)
};


// Particle coordinate stores of place_kernel and rare_copy_kernel (build knob CCMPC_WT_STORES):
// write-through (sc1 buffer stores) when every byte offset from the buffer's base fits the 31-bit
// buffer range (a.wt), plain stores otherwise.  The kernel then ends with none of those lines
// dirty in L2 for the end-of-kernel write-back: at 100 000 particles the gaps after place and
// copy shrank 4.5 -> 1.6 and 3.6 -> 2.5 us while the two kernels took 2.8 and 1.7 us longer
// (4-byte sc1 stores cost more than plain ones); step graph 104.3 -> 101.8 us, record path
// 76.1 -> 74.0 (profiles/r06/README.md)
#ifndef CCMPC_WT_STORES
#define CCMPC_WT_STORES 1
#endif
struct OutStore {
  __amdgpu_buffer_rsrc_t r;
  float *base;
  bool wt;
  __device__ __forceinline__ OutStore(float *b, bool w) : r(slab_rsrc(reinterpret_cast<double *>(b))), base(b), wt(w) {}
  __device__ __forceinline__ void put(int64_t e, float v) const {
    if (CCMPC_WT_STORES && wt)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r,
                                            static_cast<int>(e * 4), 0, 16);
    else
      base[e] = v;
  }
};

__device__ __forceinline__ int64_t *hdr_starts(int32_t *h) {
  return reinterpret_cast<int64_t *>(h + 2 * kMaxKept);
}

// The OV's count of invalid latent ids (P0's per-block counts; one wave of the OV's block 0 of
// the last kernel): z_bad[o].
__device__ __forceinline__ void write_z_bad(const FusedArgs &a, int o) {
  if (threadIdx.x >= 64) return;
  int s = 0;
  for (int b = threadIdx.x; b < a.nb0; b += 64)
    s += a.bsum[(static_cast<int64_t>(o) * a.nb0 + b) * kCntStride + kBadSlot];
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) s += __shfl_xor(s, m, 64);
  if (threadIdx.x == 0) a.z_bad[o] = s;
}

// P0: one latent id per particle (Philox inverse CDF, the injected z, or the predictor's z)
// into the workspace, each 64-particle group's count per category (kept mode k, or K = rare) --
// one wave = one group -- and the block's totals with its count of invalid ids.  The
// predictor's ids index make_ovehicles' per-latent list (v8ideal/__init__.py:488-491): an id in
// [-L, 0) wraps as a Python index does, anything else outside [0, L) is what raises IndexError
// there -- it is counted (and clamped for memory safety); the injected sampler ids must lie in
// [0, L).
template <int ZSRC>
__device__ __forceinline__ void latent_count_block(const FusedArgs &a, int bx, int o) {
  __shared__ double cdf_s[64];
  __shared__ int keep_s[64];
  __shared__ int wc_s[kFWaves][kMaxKept + 2];   // per wave: categories 0..K, then invalid ids
  FUSED_TS(0, 0);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int K = a.n_kept[o], L = a.L;
  const int64_t N = a.N;
  // the seed with the other loads (from the host side of the pack in copy_latent_count_kernel:
  // a PCIe round trip, not to be paid twice)
  const uint64_t seed = ZSRC == kZPhilox ? (a.seed_dev ? *a.seed_dev : a.seed) : 0;
  if (ZSRC == kZPhilox && tid < L) cdf_s[tid] = a.latent_cdf[static_cast<int64_t>(o) * L + tid];
  if (tid < L) keep_s[tid] = a.keep_map[o * L + tid];
  const int64_t i = static_cast<int64_t>(bx) * kFThreads + tid;
  const bool v = i < N;
  int z = 0;
  bool bad = false;
  if (ZSRC == kZIn && v) {
    z = a.z_in[static_cast<int64_t>(o) * N + i];
    bad = z < 0 || z >= L;
    z = z < 0 ? 0 : (z >= L ? L - 1 : z);
  } else if (ZSRC == kZPred && v) {
    const int64_t e = (a.rows ? static_cast<int64_t>(a.rows[o]) : o) * N + i;
    const void *zp = a.ptrs ? reinterpret_cast<const void *>(a.ptrs[1]) : a.zsrc;
    int64_t zz = a.z_bytes == 8 ? static_cast<const int64_t *>(zp)[e]
                                : static_cast<int64_t>(static_cast<const int32_t *>(zp)[e]);
    if (zz < 0 && zz >= -L) zz += L;
    bad = zz < 0 || zz >= L;
    z = bad ? 0 : static_cast<int>(zz);
  }
  __syncthreads();
  if (ZSRC == kZPhilox && v)
    z = draw_latent(i, a.ov_base + static_cast<uint32_t>(o), seed, cdf_s, L);
  if (v) {
    a.zbuf[static_cast<int64_t>(o) * a.Npad + i] = z;
    if (a.out_z) a.out_z[static_cast<int64_t>(o) * N + i] = z;
  }
  const int kk = keep_s[z];
  const int cat = kk >= 0 ? kk : K;
  const int g = bx * kFWaves + w;
  int mine = 0;
  for (int c = 0; c <= K; ++c) {
    const int n = __popcll(__ballot(v && cat == c));
    if (lane == c) mine = n;
  }
  const int nbad = __popcll(__ballot(v && bad));
  if (a.coef && bx == 0)        // the OV's per-latent coefficient rows, for P1
    stage_gmm_coefs(a.gmm + static_cast<int64_t>(o) * L * a.T * 5, L * a.T,
                    a.coef + static_cast<int64_t>(o) * kActCoef, tid, kFThreads);
  if (g < a.G && lane <= K) a.gcnt[(static_cast<int64_t>(o) * a.G + g) * kCntStride + lane] = mine;
  if (lane <= K) wc_s[w][lane] = mine;
  if (lane == 0) wc_s[w][kMaxKept + 1] = nbad;
  __syncthreads();
  int32_t *bs = a.bsum + (static_cast<int64_t>(o) * a.nb0 + bx) * kCntStride;
  if (tid <= K || tid == kBadSlot) {
    const int c = tid <= K ? tid : kMaxKept + 1;
    int s = 0;
#pragma unroll
    for (int u = 0; u < kFWaves; ++u) s += wc_s[u][c];
    bs[tid] = s;
  }
  FUSED_TS(0, 1);
}

template <int ZSRC>
__global__ __launch_bounds__(kFThreads) void latent_count_kernel(FusedArgs a) {
  latent_count_block<ZSRC>(a, blockIdx.x, blockIdx.y);
}

// P0 in the same launch as the step's input copy (ccmpc_*_packed): blocks [0, ncopy) copy the
// pinned host pack to its device side, the others are P0's blocks, whose FusedArgs (rebased by
// the host) read their inputs -- latent CDF, keep map, seed, z -- from the host side of the pack
// directly, so nothing in this launch waits on the copy.  One kernel boundary less on the step.
template <int ZSRC>
__global__ __launch_bounds__(kFThreads) void copy_latent_count_kernel(FusedArgs a, uint4 *dst,
                                                                      const uint4 *src, size_t n,
                                                                      int ncopy) {
  if (static_cast<int>(blockIdx.x) < ncopy) {
    constexpr int U = 4;  // loads in flight per thread before their stores (PCIe latency)
    const size_t stride = static_cast<size_t>(ncopy) * blockDim.x;
    for (size_t base = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; base < n;
         base += U * stride) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // clamped, branch-free: all U loads in flight together
        const size_t i = base + u * stride;
        v[u] = src[i < n ? i : n - 1];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {  // past the end: src[n - 1] again into dst[n - 1], harmless
        const size_t i = base + u * stride;
        dst[i < n ? i : n - 1] = v[u];
      }
    }
    return;
  }
  const int b = static_cast<int>(blockIdx.x) - ncopy;
  latent_count_block<ZSRC>(a, b % a.nb0, b / a.nb0);
}

// The category counts P1 block `blk` needs, into LDS (zeroed by the caller, the first batch of
// loads issued before the caller's barrier): total_s[c] over the OV, before_s[c] over the
// groups before g0 -- the P0 block totals (every row: the total; rows before g0's P0 block: the
// prefix) and the groups of g0's own P0 block before g0.  Integer-exact in any order.
__device__ __forceinline__ int count_elem(const FusedArgs &a, int o, int e, int nA, int E,
                                          int Kp1, int b0, bool &in_total, bool &in_before) {
  in_total = in_before = false;
  if (e < nA) {
    const int row = e / Kp1, c = e - row * Kp1;
    in_total = true;
    in_before = row < b0;
    return a.bsum[(static_cast<int64_t>(o) * a.nb0 + row) * kCntStride + c];
  }
  if (e < E) {
    const int ee = e - nA, gg = b0 * kFWaves + ee / Kp1, c = ee - (ee / Kp1) * Kp1;
    in_before = true;
    return a.gcnt[(static_cast<int64_t>(o) * a.G + gg) * kCntStride + c];
  }
  return 0;
}

template <bool PP, bool EPSIN>
__global__ __launch_bounds__(kFThreads) void sample_place_kernel(FusedArgs a) {
  __shared__ float act[2][40][kFP];
  // T <= kParSteps: the terms of each step's position update, [x / y][term][t][particle]
  __shared__ float terms[2][3][kParSteps][kFP];
  __shared__ float gmm_s[64 * 40 * 5 / 4];
  __shared__ int keep_s[64];
  __shared__ int zs[kFP];
  __shared__ int before_s[kMaxKept + 1], total_s[kMaxKept + 1];
  __shared__ int64_t cstart_s[kMaxKept];
  FUSED_TS(1, 0);
  const int o = blockIdx.y, blk = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int K = a.n_kept[o], L = a.L, T = a.T;
  const int64_t N = a.N;
  const uint64_t seed = a.seed_dev ? *a.seed_dev : a.seed;
  const uint32_t key = a.ov_base + static_cast<uint32_t>(o);
  const int64_t i0 = static_cast<int64_t>(blk) * kFP;
  const double mx = a.minpos[2 * o], my = a.minpos[2 * o + 1];
  // the OV's initial state (x, y, heading, speed), read here with everything else: a global
  // read after the barriers below is a round trip of its own on the chain
  const double4 st0 = {a.init_state[4 * o], a.init_state[4 * o + 1], a.init_state[4 * o + 2],
                       a.init_state[4 * o + 3]};
  // every load issued together: own latent ids, the groups' category counts, the tables
  if (tid < kFP && i0 + tid < N) zs[tid] = a.zbuf[static_cast<int64_t>(o) * a.Npad + i0 + tid];
  const int nu = a.G * (K + 1);
  constexpr int kU = kFGroups * (kMaxKept + 1) / kFThreads + 1;
  int cv[kU];
#pragma unroll
  for (int j = 0; j < kU; ++j) {
    const int u = tid + j * kFThreads;
    cv[j] = u < nu ? a.gcnt[(static_cast<int64_t>(o) * a.G + u / (K + 1)) * kCntStride +
                            u % (K + 1)]
                   : 0;
  }
  if (tid < L) keep_s[tid] = a.keep_map[o * L + tid];
  const int gsz = L * T * 5;
  const bool staged = !PP && gsz <= static_cast<int>(sizeof(gmm_s) / sizeof(float));
  if (staged)
    stage_gmm_coefs(a.gmm + static_cast<int64_t>(o) * gsz, gsz / 5, gmm_s, tid, kFThreads);
  if (tid <= K) before_s[tid] = total_s[tid] = 0;
  __syncthreads();
  // category counts before this block's group and in total (integer-exact in any order)
#pragma unroll
  for (int j = 0; j < kU; ++j) {
    const int u = tid + j * kFThreads;
    if (u < nu && cv[j] != 0) {
      const int c = u % (K + 1);
      atomicAdd(&total_s[c], cv[j]);
      if (u / (K + 1) < blk) atomicAdd(&before_s[c], cv[j]);
    }
  }
  __syncthreads();
  if (tid == 0) {
    int64_t cur = a.region[o];
    const int R = total_s[K];
    for (int k = 0; k < K; ++k) {
      cstart_s[k] = cur;
      cur += (static_cast<int64_t>(total_s[k]) + R + 3) & ~int64_t(3);
    }
  }
  FUSED_TS(1, 1);

  // ---- actions (all waves), then the chain (wave 0) ------------------------------------------
  const int64_t ip = i0 + lane;
  const bool valid = ip < N;
  if (valid)
    for (int t = w; t < T; t += kFWaves)
      draw_action<PP, EPSIN>(t, ip, zs[lane], o, T, L, N, key, seed, a.gmm, gmm_s, staged,
                             a.eps_in, act[0][t][lane], act[1][t][lane]);
  __syncthreads();
  FUSED_TS(1, 2);
  // T <= kParSteps: every step's update terms in parallel over the waves (wave w: steps t = w
  // mod 8).  The heading phi_t and speed v_t are the f32 running sums the chain accumulates
  // (phi += dphi dt at a turning step, v += a dt), recomputed by each wave in the same order;
  // sincos_rn(phi_t) is what unicycle_step evaluates (or carries, unchanged, over a straight
  // step).  What stays on the chain is three adds per coordinate and step, in unicycle_step's
  // association: x + A + B (+ C), y + A + B (turning: y - A + B - C)
  const bool par = T <= kParSteps;
  if (par && valid) {
    const float dt = a.dt;
    float phi = static_cast<float>(st0.z);
    float v = static_cast<float>(st0.w);
    for (int t = 0; t < T; ++t) {
      const float dphi = act[0][t][lane], acc = act[1][t][lane];
      const bool straight = fabsf(dphi) <= 1e-2f;
      const float phi1 = straight ? phi : phi + dphi * dt;
      if (t % kFWaves == w) {
        float s0, c0;
        sincos_rn(phi, s0, c0);
        if (straight) {
          terms[0][0][t][lane] = v * c0 * dt;
          terms[0][1][t][lane] = (acc / 2.0f) * c0 * dt * dt;
          terms[1][0][t][lane] = v * s0 * dt;
          terms[1][1][t][lane] = (acc / 2.0f) * s0 * dt * dt;
        } else {
          float s1, c1;
          sincos_rn(phi1, s1, c1);
          const float dsin = (s1 - s0) / dphi, dcos = (c1 - c0) / dphi;
          const float aw = acc / dphi;
          terms[0][0][t][lane] = aw * dcos;
          terms[0][1][t][lane] = v * dsin;
          terms[0][2][t][lane] = aw * s1 * dt;
          terms[1][0][t][lane] = v * dcos;
          terms[1][1][t][lane] = aw * dsin;
          terms[1][2][t][lane] = aw * c1 * dt;
        }
      }
      phi = phi1;
      v = v + acc * dt;
    }
  }
  __syncthreads();
  FUSED_TS(1, 3);
  if (blk == 0 && tid <= K) {  // the OV's header for P2 (every block computed the same values)
    int32_t *h = a.hdr + static_cast<int64_t>(o) * kHdrInts;
    h[tid] = total_s[tid];
    if (tid < K) hdr_starts(h)[tid] = cstart_s[tid];
  }
  if (w != 0) return;
  const int npad = static_cast<int>(a.Npad);
  float *rst = a.rstore + static_cast<int64_t>(o) * 2 * T * a.Npad;
  const int z = valid ? zs[lane] : 0;
  const int kk = keep_s[z];
  const int cat = kk >= 0 ? kk : K;
  const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int rank = 0;
  for (int c = 0; c <= K; ++c) {
    const unsigned long long m = __ballot(valid && cat == c);
    if (cat == c) rank = __popcll(m & below);
  }
  const bool native = kk >= 0;
  const int64_t dst = native ? cstart_s[kk] + before_s[kk] + rank : 0;
  const int rs = native ? 0 : before_s[K] + rank;  // slot in the rare list
  float x = 0.0f, y = 0.0f;
  if (valid) {
    x = static_cast<float>(st0.x);
    y = static_cast<float>(st0.y);
    float *op = native ? a.out + dst : rst + rs;
    const int64_t ld = native ? a.ld_out : a.Npad;
    if (par) {
      for (int t = 0; t < T; ++t) {
        if (fabsf(act[0][t][lane]) <= 1e-2f) {
          x = x + terms[0][0][t][lane] + terms[0][1][t][lane];
          y = y + terms[1][0][t][lane] + terms[1][1][t][lane];
        } else {
          x = x + terms[0][0][t][lane] + terms[0][1][t][lane] + terms[0][2][t][lane];
          y = y - terms[1][0][t][lane] + terms[1][1][t][lane] - terms[1][2][t][lane];
        }
        op[(2 * t) * ld] = x;
        op[(2 * t + 1) * ld] = y;
      }
    } else {
      float phi = static_cast<float>(st0.z), v = static_cast<float>(st0.w);
      float s0, c0;
      sincos_rn(phi, s0, c0);
      for (int t = 0; t < T; ++t) {
        unicycle_step(x, y, phi, v, s0, c0, act[0][t][lane], act[1][t][lane], a.dt);
        op[(2 * t) * ld] = x;
        op[(2 * t + 1) * ld] = y;
      }
    }
    if (!native) {
      const float4 info = {x, y, __builtin_bit_cast(float, z), 0.0f};
      reinterpret_cast<float4 *>(a.rinfo)[static_cast<int64_t>(o) * npad + rs] = info;
    }
  }
  FUSED_TS(1, 4);
  // this block is centre group blk: its kept-mode sums of the final world positions
  const double xw = static_cast<double>(x) + mx, yw = static_cast<double>(y) + my;
  double2 *gp = reinterpret_cast<double2 *>(a.gpart) + (static_cast<int64_t>(o) * a.G + blk) * a.max_k;
  for (int k = 0; k < K; ++k) {
    const bool mine = valid && cat == k;
    const double sx = group_sum64(mine ? xw : 0.0), sy = group_sum64(mine ? yw : 0.0);
    if (lane == 0) gp[k] = double2{sx, sy};
  }
  FUSED_TS(1, 5);
}

// P1 for the large clouds (the sampler) and for the predictor's output (MODE kSrcPred: the
// block's 64 x 2T coordinate run staged through LDS, no actions).  One chain wave of 64
// particles per block of NW waves (4: a 100 000-particle cloud is 1563 blocks, all resident at
// 7 per CU); the sampler's modes (MODE bit 1 = injected noise, 2 = per-particle parameters) draw
// the block's T x 64 actions over the waves first, with the per-latent coefficient rows P0
// staged (no exp per block).  Measured and not kept: the draws as their own launch at full
// occupancy (one pair per lane, or a grid-stride loop): 15 / 12 us against ~10 us inside this
// kernel, plus a boundary.  Dynamic LDS (floats), sized by T:
//   sampler    act[2T][64], coefficient rows [L T 5] (per-latent, when they fit), T <=
//              kParSteps: sc[2][T + 1][64] (the headings' sin / cos) and terms[2][3][T][64]
//              (each step's position terms)
//   predictor  tile[64][2T + 1]
// The category counts come from P0's block totals (a few hundred ints, not every group's).
template <int MODE, int NW>
__global__ __launch_bounds__(64 * NW, 7) void place_kernel(FusedArgs a) {
  constexpr bool PRED = MODE == kSrcPred, PP = (MODE & 2) != 0, EPSIN = (MODE & 1) != 0;
  constexpr int PB = kFP, NTH = 64 * NW;
  extern __shared__ float dyn[];
  __shared__ int keep_s[64];
  __shared__ int zs[PB];
  __shared__ int before_s[kMaxKept + 1], total_s[kMaxKept + 1];
  __shared__ double st_s[6];                // the OV's initial state (x, y, heading, speed), minpos
  FUSED_TS(1, 0);
  const int o = blockIdx.y, blk = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int K = a.n_kept[o], L = a.L, T = a.T, Kp1 = K + 1;
  const int64_t N = a.N;
  const int64_t i0 = static_cast<int64_t>(blk) * PB;
  const int g0 = blk, b0 = g0 / kFWaves;     // (P0 blocks are kFWaves groups)
  const int64_t reg = a.region[o];
  const int W = 2 * T, S = W + 1;
  const int n = static_cast<int>(N - i0 < PB ? N - i0 : PB);
  // every load that needs nothing from another, issued together: own latent ids, the count
  // rows, the tables, the OV's initial state, the block's actions or coordinate run
  if (tid < PB && i0 + tid < N) zs[tid] = a.zbuf[static_cast<int64_t>(o) * a.Npad + i0 + tid];
  if (tid < L) keep_s[tid] = a.keep_map[o * L + tid];
  const int nA = a.nb0 * Kp1, E = nA + (g0 - b0 * kFWaves) * Kp1;
  constexpr int kC = 4;
  int cv[kC];
  bool ct[kC], cb[kC];
#pragma unroll
  for (int j = 0; j < kC; ++j) cv[j] = count_elem(a, o, tid + j * NTH, nA, E, Kp1, b0, ct[j], cb[j]);
  if (tid < 4) st_s[tid] = PRED ? 0.0 : a.init_state[4 * o + tid];
  else if (tid < 6) st_s[tid] = a.minpos[2 * o + tid - 4];
  const bool par = T <= kParSteps;
  const int gsz = L * T * 5;
  const bool staged = !PRED && !PP && a.coef != nullptr;
  float *act = dyn;                                         // [2T][PB]
  float *sc = act + 2 * T * PB;                             // [2][T + 1][PB] (par)
  float *terms = sc + (par ? 2 * (T + 1) * PB : 0);         // [2][3][T][PB] (par)
  float *coef_s = terms;   // [L T 5] when staged: read only before the terms are written
  if (PRED) {
    const int64_t row = a.rows ? static_cast<int64_t>(a.rows[o]) : o;
    const float *pp = a.ptrs ? reinterpret_cast<const float *>(a.ptrs[0]) : a.pred;
    const float *src = pp + (row * N + i0) * W;
    for (int e = tid; e < n * W; e += NTH) {
      const int p = e / W;
      dyn[p * S + (e - p * W)] = src[e];
    }
  } else if (staged) {
    const float *cg = a.coef + static_cast<int64_t>(o) * kActCoef;
    for (int e = tid; e < gsz; e += NTH) coef_s[e] = cg[e];
  }
  if (tid <= K) before_s[tid] = total_s[tid] = 0;
  __syncthreads();
  FUSED_TS(1, 1);
  // the counts (further rounds only for clouds of > ~500 000 particles)
  for (int e0 = 0; e0 < E; e0 += kC * NTH) {
    if (e0 > 0) {
#pragma unroll
      for (int j = 0; j < kC; ++j)
        cv[j] = count_elem(a, o, e0 + tid + j * NTH, nA, E, Kp1, b0, ct[j], cb[j]);
    }
#pragma unroll
    for (int j = 0; j < kC; ++j) {
      const int e = e0 + tid + j * NTH;
      if (cv[j] == 0) continue;
      const int c = e < nA ? e % Kp1 : (e - nA) % Kp1;
      if (ct[j]) atomicAdd(&total_s[c], cv[j]);
      if (cb[j]) atomicAdd(&before_s[c], cv[j]);
    }
  }
  if (!PRED) {     // the block's actions: step t of particle lane on wave t mod NW
    const uint64_t seed = a.seed_dev ? *a.seed_dev : a.seed;
    const uint32_t key = a.ov_base + static_cast<uint32_t>(o);
    if (!EPSIN && T <= 2 * NW) {
      // at most two Philox pairs per lane: every radius first, then every angle (one set of
      // polynomial coefficients in registers at a time: a loop of whole pairs spilled them)
      double rr[2], uu[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int t = w + j * NW;
        if (lane < n && t < T)
          normal_radius(static_cast<uint32_t>(i0 + lane), static_cast<uint32_t>(t), key,
                        STREAM_SAMPLER_EPS, seed, rr[j], uu[j]);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int t = w + j * NW;
        if (lane < n && t < T) {
          double e0, e1;
          normal_angle(rr[j], uu[j], e0, e1);
          action_from_noise<PP>(t, i0 + lane, zs[lane], o, T, L, N, a.gmm, coef_s, staged,
                                static_cast<float>(e0), static_cast<float>(e1),
                                act[(2 * t) * PB + lane], act[(2 * t + 1) * PB + lane]);
        }
      }
    } else if (lane < n) {
#pragma unroll 1
      for (int t = w; t < T; t += NW)
        draw_action<PP, EPSIN>(t, i0 + lane, zs[lane], o, T, L, N, key, seed, a.gmm, coef_s,
                               staged, a.eps_in, act[(2 * t) * PB + lane],
                               act[(2 * t + 1) * PB + lane]);
    }
  }
  const float dt = a.dt;
  if (!PRED) __syncthreads();     // the actions
  if (!PRED && par) {
    // T <= kParSteps: the sin / cos of every heading phi_0 .. phi_T, step t of particle lane on
    // wave t mod NW.  phi_t is the f32 running sum the chain accumulates (phi += dphi dt at a
    // turning step), recomputed in the same order; sincos_rn(phi_t) is what unicycle_step
    // evaluates at step t (or carries, unchanged, over a straight step: phi_t+1 == phi_t).  One
    // sincos per heading, where evaluating each step's pair took two
    if (lane < n) {
#pragma unroll 1
      for (int t = w; t <= T; t += NW) {
        float phi = static_cast<float>(st_s[2]);
        for (int s = 0; s < t; ++s) {
          const float dphi = act[(2 * s) * PB + lane];
          phi = fabsf(dphi) <= 1e-2f ? phi : phi + dphi * dt;
        }
        sincos_rn(phi, sc[t * PB + lane], sc[(T + 1 + t) * PB + lane]);
      }
    }
    __syncthreads();
    FUSED_TS(1, 2);
    // each step's position terms, in unicycle_step's expressions, in parallel over the waves;
    // the chain keeps its adds in unicycle_step's association: x + A + B (+ C), y + A + B
    // (turning: y - A + B - C)
    if (lane < n) {
#pragma unroll 1
      for (int t = w; t < T; t += NW) {
        float v = static_cast<float>(st_s[3]);
        for (int s = 0; s < t; ++s) v = v + act[(2 * s + 1) * PB + lane] * dt;
        const float dphi = act[(2 * t) * PB + lane], acc = act[(2 * t + 1) * PB + lane];
        const float s0 = sc[t * PB + lane], c0 = sc[(T + 1 + t) * PB + lane];
        float *tx = terms + t * PB + lane, *ty = terms + (3 * T + t) * PB + lane;
        if (fabsf(dphi) <= 1e-2f) {
          tx[0] = v * c0 * dt;
          tx[T * PB] = (acc / 2.0f) * c0 * dt * dt;
          ty[0] = v * s0 * dt;
          ty[T * PB] = (acc / 2.0f) * s0 * dt * dt;
        } else {
          const float s1 = sc[(t + 1) * PB + lane], c1 = sc[(T + 2 + t) * PB + lane];
          const float dsin = (s1 - s0) / dphi, dcos = (c1 - c0) / dphi;
          const float aw = acc / dphi;
          tx[0] = aw * dcos;
          tx[T * PB] = v * dsin;
          tx[2 * T * PB] = aw * s1 * dt;
          ty[0] = v * dcos;
          ty[T * PB] = aw * dsin;
          ty[2 * T * PB] = aw * c1 * dt;
        }
      }
    }
  }
  __syncthreads();
  FUSED_TS(1, 3);
  const int R = total_s[K];
  if (blk == 0 && tid <= K) {  // the OV's header for P2 (every block computed the same values)
    int32_t *h = a.hdr + static_cast<int64_t>(o) * kHdrInts;
    h[tid] = total_s[tid];
    if (tid < K) {
      int64_t cur = reg;
      for (int k = 0; k < tid; ++k) cur += (static_cast<int64_t>(total_s[k]) + R + 3) & ~int64_t(3);
      hdr_starts(h)[tid] = cur;
    }
  }
  if (w != 0) return;
  // ---- the chain wave: particle i0 + lane ----------------------------------------------------
  const bool valid = lane < n;
  const int kk = valid ? keep_s[zs[lane]] : -1;
  const int cat = kk >= 0 ? kk : K;
  const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int rank = 0;
  for (int c = 0; c <= K; ++c) {
    const unsigned long long m = __ballot(valid && cat == c);
    if (cat == c) rank = __popcll(m & below);
  }
  const bool native = cat < K;
  int64_t dst = 0;
  if (native) {
    dst = reg;
    for (int k = 0; k < cat; ++k) dst += (static_cast<int64_t>(total_s[k]) + R + 3) & ~int64_t(3);
    dst += before_s[cat] + rank;
  }
  const int rs = native ? 0 : before_s[K] + rank;  // slot in the rare list
  const int npad = static_cast<int>(a.Npad);
  float x = 0.0f, y = 0.0f;
  // both destinations' stores from uniform bases (a.out, the OV's rare list)
  const OutStore so(a.out, a.wt != 0), sr(a.rstore + static_cast<int64_t>(o) * W * a.Npad, a.wt != 0);
  if (valid) {
    const OutStore &st = native ? so : sr;
    const int64_t e0 = native ? dst : rs;
    const int64_t ld = native ? a.ld_out : a.Npad;
    if (PRED) {
      const float *tp = dyn + lane * S;
      for (int r = 0; r < W; ++r) st.put(e0 + r * ld, tp[r]);
      x = tp[W - 2];
      y = tp[W - 1];
    } else if (par) {
      x = static_cast<float>(st_s[0]);
      y = static_cast<float>(st_s[1]);
      for (int t = 0; t < T; ++t) {
        const float *tx = terms + t * PB + lane, *ty = terms + (3 * T + t) * PB + lane;
        if (fabsf(act[(2 * t) * PB + lane]) <= 1e-2f) {
          x = x + tx[0] + tx[T * PB];
          y = y + ty[0] + ty[T * PB];
        } else {
          x = x + tx[0] + tx[T * PB] + tx[2 * T * PB];
          y = y - ty[0] + ty[T * PB] - ty[2 * T * PB];
        }
        st.put(e0 + (2 * t) * ld, x);
        st.put(e0 + (2 * t + 1) * ld, y);
      }
    } else {
      x = static_cast<float>(st_s[0]);
      y = static_cast<float>(st_s[1]);
      float phi = static_cast<float>(st_s[2]), v = static_cast<float>(st_s[3]);
      float s0, c0;
      sincos_rn(phi, s0, c0);
      for (int t = 0; t < T; ++t) {
        unicycle_step(x, y, phi, v, s0, c0, act[(2 * t) * PB + lane],
                      act[(2 * t + 1) * PB + lane], dt);
        st.put(e0 + (2 * t) * ld, x);
        st.put(e0 + (2 * t + 1) * ld, y);
      }
    }
    if (!native) {
      const float4 info = {x, y, __builtin_bit_cast(float, zs[lane]), 0.0f};
      reinterpret_cast<float4 *>(a.rinfo)[static_cast<int64_t>(o) * npad + rs] = info;
    }
  }
  FUSED_TS(1, 4);
  // this block is centre group g0: its kept-mode sums of the final world positions
  const double xw = static_cast<double>(x) + st_s[4], yw = static_cast<double>(y) + st_s[5];
  double2 *gp = reinterpret_cast<double2 *>(a.gpart) + (static_cast<int64_t>(o) * a.G + g0) * a.max_k;
  for (int k = 0; k < K; ++k) {
    const bool mine = valid && cat == k;
    const double sx = group_sum64(mine ? xw : 0.0), sy = group_sum64(mine ? yw : 0.0);
    if (lane == 0) gp[k] = double2{sx, sy};
  }
  FUSED_TS(1, 5);
}

// VR: the coordinate rows a thread holds (2T <= VR); KB: rare records per thread and round of
// the key pass (T <= 8: 16 rows leave room for 16 records, a C2-shape rare list in one round)
template <int VR, int KB>
__global__ __launch_bounds__(kRThreads) void rare_place_kernel(FusedArgs a) {
  __shared__ double2 gp_s[kFGroups * kMaxKept + 1];  // the OV's centre partials [g][k], -0.0
  __shared__ int hist[kFusedMaxBins];             // rare particles per bin in slots >= r0
  __shared__ int pre[kFusedMaxBins];              // ... in rare-list slots before this block's
  __shared__ int bstart[kFusedMaxBins];           // bin start relative to the region
  __shared__ int wcnt[kRWaves][kFusedMaxBins];
  __shared__ __attribute__((aligned(16))) int okey[kRThreads];
  __shared__ int keep_s[64], tot_s[kMaxKept + 1];
  __shared__ int64_t cst_s[kMaxKept];
  __shared__ double cen_s[kMaxKept][2];
  FUSED_TS(2, 0);
  const int o = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int K = a.n_kept[o], L = a.L, T = a.T, rows = 2 * T;
  const int r0 = blockIdx.x * kRThreads;
  const int npad = static_cast<int>(a.Npad);
  // every load that needs nothing from another is issued at once: the header, the tables, this
  // thread's rare-slot coordinates (slot clamped into the list's storage, used only if < R) and
  // the centre partials
  const int32_t *h = a.hdr + static_cast<int64_t>(o) * kHdrInts;
  // (a load issued after a __syncthreads is a fresh round trip the next barrier waits for)
  const int64_t reg = a.region[o];
  const double mx = a.minpos[2 * o], my = a.minpos[2 * o + 1];
  if (tid <= K) tot_s[tid] = h[tid];
  if (tid < K) cst_s[tid] = hdr_starts(const_cast<int32_t *>(h))[tid];
  if (tid < L) keep_s[tid] = a.keep_map[o * L + tid];
  const int r = r0 + tid;
  const float *src = a.rstore + static_cast<int64_t>(o) * 2 * T * a.Npad + (r < npad ? r : npad - 1);
  float v[VR];
#pragma unroll
  for (int rr = 0; rr < VR; ++rr)
    if (rr < rows) v[rr] = src[static_cast<int64_t>(rr) * npad];
  const int ng = a.G * K;
  const double2 *gp = reinterpret_cast<const double2 *>(a.gpart) + static_cast<int64_t>(o) * a.G * a.max_k;
  for (int u = tid; u < ng; u += kRThreads) gp_s[u] = gp[(u / K) * a.max_k + u % K];
  if (tid == 0) gp_s[kFGroups * kMaxKept] = double2{-0.0, -0.0};  // superblock_sum's sentinel
  // the first batch of rare records too: R is not known yet, so the slots are clamped into the
  // list's storage (a launch's first kB * 256 records cover the C2 shape's whole rare list)
  const float4 *info = reinterpret_cast<const float4 *>(a.rinfo) + static_cast<int64_t>(o) * npad;
  constexpr int kB = KB;
  float4 f[kB];
#pragma unroll
  for (int j = 0; j < kB; ++j) {
    const int q = j * kRThreads + tid;
    f[j] = info[q < npad ? q : npad - 1];
  }
  const int nbins = K * (L + 1);
  for (int b = tid; b < nbins; b += kRThreads) hist[b] = pre[b] = 0;
  okey[tid] = -1;                                 // not one of this block's rare slots
  __syncthreads();
  FUSED_TS(2, 1);
  const int R = tot_s[K];
  if (r0 >= R && blockIdx.x != 0) return;  // uniform: no rare slots here (block 0 writes cells)
  const bool own = r < R;
  auto load_batch = [&](int q0) {
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      const int q = q0 + j * kRThreads + tid;
      f[j] = info[q < R ? q : (R > 0 ? R - 1 : 0)];
    }
  };
  // centres, canonical order (bucket.hpp): superblocks, then left to right
  if (tid < K) {
    const int k = tid;
    double2 tot = {0.0, 0.0};
#if defined(CCMPC_PROBE) && (CCMPC_PROBE & 128)  // timing probe: the centre sums left out
    if (a.G < 0)
#endif
    for (int j = 0; j * kCentreSuper < a.G; ++j) {
      const double2 s = superblock_sum(
          j, a.G, [&](int g, bool in) { return gp_s[in ? g * K + k : kFGroups * kMaxKept]; });
      tot.x += s.x;
      tot.y += s.y;
    }
    const double nk = static_cast<double>(tot_s[k]);
    cen_s[k][0] = tot.x / nk;
    cen_s[k][1] = tot.y / nk;
  }
  __syncthreads();
  FUSED_TS(2, 2);
  // every rare particle's key (owner (L + 1) + 1 + z), counted per bin before this block's
  // first slot (pre) and from it on (hist): one LDS atomic per key; this block's own keys kept
  for (int q0 = 0; q0 < R; q0 += kB * kRThreads) {
    if (q0 > 0) load_batch(q0);
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      const int q = q0 + j * kRThreads + tid;
      if (q < R) {
        const int kq = key_staged(__builtin_bit_cast(int, f[j].z), static_cast<double>(f[j].x) + mx,
                                  static_cast<double>(f[j].y) + my, keep_s, cen_s, K, L);
        atomicAdd(q < r0 ? &pre[kq] : &hist[kq], 1);
        if (q >= r0 && q < r0 + kRThreads) okey[q - r0] = kq;
      }
    }
  }
  for (int b = tid; b < kRWaves * nbins; b += kRThreads) wcnt[b / nbins][b % nbins] = 0;
  __syncthreads();
  FUSED_TS(2, 3);
  // bins of kept mode k start after its natives, latents ascending (one thread per bin, its
  // prefix summed over independent LDS reads); block 0: the cells' outputs
  for (int b = tid; b < nbins; b += kRThreads) {
    const int k = b / (L + 1), gi = b - k * (L + 1), hb = k * (L + 1) + 1;
    const int upto = gi == 0 ? L : gi - 1;  // gi == 0 (the natives' bin): every rare bin of k
    int s = 0;
#pragma unroll 8
    for (int zz = 0; zz < upto; ++zz) s += hist[hb + zz] + pre[hb + zz];
    if (gi > 0) {
      bstart[b] = static_cast<int>(cst_s[k] - reg) + tot_s[k] + s;
    } else if (blockIdx.x == 0) {
      const int64_t n = tot_s[k] + s;
      const int cell = a.cell_base[o] + k;
      a.cell_off[cell] = cst_s[k];
      a.cell_cnt[cell] = n;
      a.cell_pmf[cell] = static_cast<double>(n) / static_cast<double>(a.N);
      a.init_center[2 * cell] = cen_s[k][0];
      a.init_center[2 * cell + 1] = cen_s[k][1];
    }
  }
  if (blockIdx.x == 0 && a.z_bad) write_z_bad(a, o);
  FUSED_TS(2, 4);
  // this block's stable ranks: lanes in order within a wave, waves in order.  Every lane scans
  // its wave's 64 keys (broadcast LDS reads, 16 bytes at a time): the same-key lanes before it
  // (its rank) and in all (the wave's count, written by the last such lane) -- a fixed 16
  // reads, where a ballot round per distinct key took up to ~30 dependent rounds
  const int kr = okey[tid];
  int rank = 0, cnt = 0;
  {
    const int4 *wk = reinterpret_cast<const int4 *>(okey + w * 64);
#pragma unroll
    for (int j4 = 0; j4 < 16; ++j4) {
      const int4 k4 = wk[j4];
      const int kk[4] = {k4.x, k4.y, k4.z, k4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool same = kk[e] == kr;
        rank += (same && 4 * j4 + e < lane) ? 1 : 0;
        cnt += same ? 1 : 0;
      }
    }
  }
  if (own && rank == cnt - 1) wcnt[w][kr] = cnt;
  __syncthreads();
  FUSED_TS(2, 5);
  if (own) {
    int before = pre[kr] + rank;
    for (int u = 0; u < w; ++u) before += wcnt[u][kr];
    float *out = a.out + reg + bstart[kr] + before;
#pragma unroll
    for (int rr = 0; rr < VR; ++rr)
      if (rr < rows) out[static_cast<int64_t>(rr) * a.ld_out] = v[rr];
  }
  FUSED_TS(2, 6);
}

// P2 keys (N > kFusedMaxN): per block of kKeySlots rare-list slots, the centres and the keys.
// Centres in the canonical order (bucket.hpp): thread (k, j) sums superblock j of mode k's group
// partials left to right (S_j = 0.0 + P_64j + P_64j+1 + ...), then thread k adds the S_j left to
// right -- the same additions in the same order as every other form, so the same bits.  Block 0
// writes the centres (init_center) even when the OV has no rare particle.
__global__ __launch_bounds__(kRThreads) void rare_key_kernel(FusedArgs a) {
  __shared__ double2 sup_s[kMaxKept][kWideMaxSup + 16];  // padded to rounds of 16 with -0.0
  __shared__ int hist[kFusedMaxBins];
  __shared__ int keep_s[64], tot_s[kMaxKept + 1];
  __shared__ double cen_s[kMaxKept][2];
  FUSED_TS(3, 0);
  const int o = blockIdx.y, tid = threadIdx.x;
  const int K = a.n_kept[o], L = a.L;
  const int s0 = blockIdx.x * kKeySlots;
  const int npad = static_cast<int>(a.Npad);
  const int32_t *h = a.hdr + static_cast<int64_t>(o) * kHdrInts;
  const double mx = a.minpos[2 * o], my = a.minpos[2 * o + 1];
  if (tid <= K) tot_s[tid] = h[tid];
  if (tid < L) keep_s[tid] = a.keep_map[o * L + tid];
  // this thread's four rare records (slots clamped into the list's storage; R is not known yet)
  const float4 *info = reinterpret_cast<const float4 *>(a.rinfo) + static_cast<int64_t>(o) * npad;
  float4 f[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = s0 + j * kRThreads + tid;
    f[j] = info[r < npad ? r : npad - 1];
  }
  const int nbins = K * (L + 1);
  for (int b = tid; b < nbins; b += kRThreads) hist[b] = 0;
  __syncthreads();
  FUSED_TS(3, 1);
  const int R = tot_s[K];
  if (s0 >= R && blockIdx.x != 0) return;  // uniform: no slots here (block 0 writes centres)
  // the superblock sums: thread (k, j) sums superblock j of mode k's group partials left to
  // right from global (S_j = 0.0 + P_64j + P_64j+1 + ...), then thread k adds the S_j left to
  // right.  Measured and not kept: staging the partials through LDS first (3.8 us against 3.0),
  // and P1's last arriving block per superblock summing it (keys 8.1 -> 5.5 us, but P1 25.6 ->
  // 34.9 us: its blocks slowed down throughout, profiles/r06/README.md)
  const int G = a.G, nsup = (G + kCentreSuper - 1) / kCentreSuper;
  {
    const double2 *gp = reinterpret_cast<const double2 *>(a.gpart) + static_cast<int64_t>(o) * G * a.max_k;
    for (int u = tid; u < K * nsup; u += kRThreads) {
      const int k = u / nsup, jj = u - k * nsup;
      const int ga = jj * kCentreSuper, gb = min(G, ga + kCentreSuper);
      double2 acc = {0.0, 0.0};
      for (int g = ga; g < gb; g += 16) {
        double2 v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = gp[static_cast<int64_t>(g + q < gb ? g + q : gb - 1) * a.max_k + k];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const bool in = g + q < gb;
          acc.x += in ? v[q].x : -0.0;      // x + -0.0 == x: bucket.hpp's sentinel
          acc.y += in ? v[q].y : -0.0;
        }
      }
      sup_s[k][jj] = acc;
    }
  }
  for (int u = tid; u < K * 16; u += kRThreads) {
    const int k = u / 16, j = nsup + (u - k * 16);
    sup_s[k][j] = double2{-0.0, -0.0};
  }
  __syncthreads();
  FUSED_TS(3, 2);
  if (tid < K) {
    double2 tot = {0.0, 0.0};
    lds_row_sum(tot, sup_s[tid], nsup);
    const double nk = static_cast<double>(tot_s[tid]);
    cen_s[tid][0] = tot.x / nk;
    cen_s[tid][1] = tot.y / nk;
    if (blockIdx.x == 0) {
      const int cell = a.cell_base[o] + tid;
      a.init_center[2 * cell] = cen_s[tid][0];
      a.init_center[2 * cell + 1] = cen_s[tid][1];
    }
  }
  __syncthreads();
  FUSED_TS(3, 3);
  int32_t *kb = a.kbuf + static_cast<int64_t>(o) * npad;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = s0 + j * kRThreads + tid;
    if (r < R) {
      const int kq = key_staged(__builtin_bit_cast(int, f[j].z), static_cast<double>(f[j].x) + mx,
                                static_cast<double>(f[j].y) + my, keep_s, cen_s, K, L);
      kb[r] = kq;
      atomicAdd(&hist[kq], 1);
    }
  }
  __syncthreads();
  if (s0 < R) {
    int32_t *rh = a.rhist + (static_cast<int64_t>(o) * a.nkb + blockIdx.x) * kFusedMaxBins;
    for (int b = tid; b < nbins; b += kRThreads) rh[b] = hist[b];
  }
  FUSED_TS(3, 4);
}

// P3 copy (N > kFusedMaxN): per block of kRThreads rare-list slots (one per thread), in the P2
// keys block B = r0 / kKeySlots.  Every P2 block's histogram gives each bin's total (-> the bin
// starts) and its count in the P2 blocks before B; the keys of B's slots before r0 add the rest
// of the count before this block; a scan of each wave's 64 keys gives the stable ranks.  Block 0
// writes the cells' offsets, counts and pmf (and the invalid-id count).
template <int VR>  // the coordinate rows a thread holds (2T <= VR), as rare_place_kernel
__global__ __launch_bounds__(kRThreads) void rare_copy_kernel(FusedArgs a) {
  __shared__ int binsum[kFusedMaxBins];   // rare particles per bin, whole OV
  __shared__ int pre[kFusedMaxBins];      // ... in rare-list slots before this block's
  __shared__ int bstart[kFusedMaxBins];   // bin start relative to the region
  __shared__ int wcnt[kRWaves][kFusedMaxBins];
  __shared__ __attribute__((aligned(16))) int okey[kRThreads];
  __shared__ int tot_s[kMaxKept + 1];
  __shared__ int64_t cst_s[kMaxKept];
  FUSED_TS(4, 0);
  const int o = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int K = a.n_kept[o], L = a.L, T = a.T, rows = 2 * T;
  const int r0 = blockIdx.x * kRThreads, B = r0 / kKeySlots;
  const int npad = static_cast<int>(a.Npad);
  const int32_t *h = a.hdr + static_cast<int64_t>(o) * kHdrInts;
  const int64_t reg = a.region[o];
  if (tid <= K) tot_s[tid] = h[tid];
  if (tid < K) cst_s[tid] = hdr_starts(const_cast<int32_t *>(h))[tid];
  const int r = r0 + tid;
  const int rc = r < npad ? r : npad - 1;
  const int32_t *kb = a.kbuf + static_cast<int64_t>(o) * npad;
  const int kown = kb[rc];
  const float *src = a.rstore + static_cast<int64_t>(o) * rows * a.Npad + rc;
  float v[VR];
#pragma unroll
  for (int rr = 0; rr < VR; ++rr)
    if (rr < rows) v[rr] = src[static_cast<int64_t>(rr) * npad];
  constexpr int kPre = kKeySlots / kRThreads - 1;  // B's slots before r0: up to 3 per thread
  int pk[kPre];
#pragma unroll
  for (int j = 0; j < kPre; ++j) {
    const int sl = B * kKeySlots + j * kRThreads + tid;
    pk[j] = sl < r0 ? kb[sl] : -1;
  }
  const int nbins = K * (L + 1);
  for (int b = tid; b < nbins; b += kRThreads) binsum[b] = pre[b] = 0;
  for (int b = tid; b < kRWaves * nbins; b += kRThreads) wcnt[b / nbins][b % nbins] = 0;
  __syncthreads();
  FUSED_TS(4, 1);
  const int R = tot_s[K];
  if (r0 >= R && blockIdx.x != 0) return;  // uniform: no rare slots here (block 0 writes cells)
  const bool own = r < R;
  const int nkb = (R + kKeySlots - 1) / kKeySlots;
  const int32_t *rh = a.rhist + static_cast<int64_t>(o) * a.nkb * kFusedMaxBins;
  for (int e0 = 0; e0 < nkb * nbins; e0 += 4 * kRThreads) {
    int hv[4], hb[4], hr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = e0 + j * kRThreads + tid;
      hr[j] = e / nbins;
      hb[j] = e - hr[j] * nbins;
      hv[j] = e < nkb * nbins ? rh[static_cast<int64_t>(hr[j]) * kFusedMaxBins + hb[j]] : 0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (hv[j] == 0) continue;
      atomicAdd(&binsum[hb[j]], hv[j]);
      if (hr[j] < B) atomicAdd(&pre[hb[j]], hv[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < kPre; ++j)
    if (pk[j] >= 0) atomicAdd(&pre[pk[j]], 1);
  okey[tid] = own ? kown : -1;
  __syncthreads();
  FUSED_TS(4, 2);
  // bins of kept mode k start after its natives, latents ascending (one thread per bin, its
  // prefix summed over independent LDS reads); block 0: the cells' outputs
  for (int b = tid; b < nbins; b += kRThreads) {
    const int k = b / (L + 1), gi = b - k * (L + 1), hb = k * (L + 1) + 1;
    const int upto = gi == 0 ? L : gi - 1;  // gi == 0 (the natives' bin): every rare bin of k
    int s = 0;
#pragma unroll 8
    for (int zz = 0; zz < upto; ++zz) s += binsum[hb + zz];
    if (gi > 0) {
      bstart[b] = static_cast<int>(cst_s[k] - reg) + tot_s[k] + s;
    } else if (blockIdx.x == 0) {
      const int64_t n = tot_s[k] + s;
      const int cell = a.cell_base[o] + k;
      a.cell_off[cell] = cst_s[k];
      a.cell_cnt[cell] = n;
      a.cell_pmf[cell] = static_cast<double>(n) / static_cast<double>(a.N);
    }
  }
  if (blockIdx.x == 0 && a.z_bad) write_z_bad(a, o);
  // this block's stable ranks (rare_place's scan of each wave's 64 keys)
  const int kr = okey[tid];
  int rank = 0, cnt = 0;
  {
    const int4 *wk = reinterpret_cast<const int4 *>(okey + w * 64);
#pragma unroll
    for (int j4 = 0; j4 < 16; ++j4) {
      const int4 k4 = wk[j4];
      const int kk[4] = {k4.x, k4.y, k4.z, k4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool same = kk[e] == kr;
        rank += (same && 4 * j4 + e < lane) ? 1 : 0;
        cnt += same ? 1 : 0;
      }
    }
  }
  if (own && rank == cnt - 1) wcnt[w][kr] = cnt;
  __syncthreads();
  FUSED_TS(4, 3);
  if (own) {
    int before = pre[kr] + rank;
    for (int u = 0; u < w; ++u) before += wcnt[u][kr];
    const OutStore so(a.out, a.wt != 0);
    const int64_t e0 = reg + bstart[kr] + before;
#pragma unroll
    for (int rr = 0; rr < VR; ++rr)
      if (rr < rows) so.put(e0 + static_cast<int64_t>(rr) * a.ld_out, v[rr]);
  }
  FUSED_TS(4, 4);
}

struct FusedWs {
  size_t zbuf, gcnt, bsum, hdr, gpart, rinfo, rstore, kbuf, rhist, coef, total;
  int64_t G, nb0, nkb, Npad;
};

inline size_t a256(size_t b) { return (b + 255) / 256 * 256; }

inline FusedWs fused_ws(int64_t n_ov, int64_t N, int64_t T, int64_t max_k) {
  FusedWs w;
  w.G = (N + kFP - 1) / kFP;
  w.Npad = (N + 3) & ~int64_t(3);
  w.nb0 = (N + kFThreads - 1) / kFThreads;
  w.nkb = (w.Npad + kKeySlots - 1) / kKeySlots;
  size_t o = 0;
  w.zbuf = o;
  o += a256(sizeof(int32_t) * n_ov * w.Npad);
  w.gcnt = o;
  o += a256(sizeof(int32_t) * n_ov * w.G * kCntStride);
  w.bsum = o;
  o += a256(sizeof(int32_t) * n_ov * w.nb0 * kCntStride);
  w.hdr = o;
  o += a256(sizeof(int32_t) * kHdrInts * n_ov);
  w.gpart = o;
  o += a256(sizeof(double) * 2 * n_ov * w.G * max_k);
  w.rinfo = o;
  o += a256(sizeof(float) * 4 * n_ov * w.Npad);
  w.rstore = o;
  o += a256(sizeof(float) * n_ov * 2 * T * w.Npad);
  w.kbuf = o;
  o += a256(sizeof(int32_t) * n_ov * w.Npad);
  w.rhist = o;
  o += a256(sizeof(int32_t) * n_ov * w.nkb * kFusedMaxBins);
  const bool wide = N > kFusedMaxN;       // P0's coefficient rows for the large clouds' P1
  w.coef = o;
  o += wide ? a256(sizeof(float) * n_ov * kActCoef) : 0;
  w.total = o;
  return w;
}

// The rare stage: one pass (rare_place) up to kFusedMaxN, the keys + copy pair above (measured
// at C2's shape the pair cost 18.2 us against rare_place's 16.7, profiles/r06/README.md)
inline bool rare_two_pass(int64_t N) { return N > kFusedMaxN; }

// Raise a kernel's dynamic LDS limit above the 48 KiB default when a launch needs it (the
// attribute is per device: set on every such launch; a failure is reported, not launched)
template <typename Kern>
inline bool lds_fits(Kern k, size_t bytes) {
  if (bytes <= 48 * 1024) return true;
  return hipFuncSetAttribute(reinterpret_cast<const void *>(k),
                             hipFuncAttributeMaxDynamicSharedMemorySize,
                             static_cast<int>(bytes)) == hipSuccess;
}

template <int MODE>
inline int launch_place(const FusedArgs &a, int64_t n_ov, hipStream_t s) {
  // four waves: 7 blocks per CU (72 VGPRs, LDS 21 KB), so all 1563 blocks of a 100 000-particle
  // cloud are resident at once.  The sampler's f64 draws spill 16 VGPRs there (scratch
  // traffic: the PMC write bytes are ~4x the placement's); two-wave blocks at 80 VGPRs spill
  // 3 but measured no faster (span 26.0 vs 25.6 us, record path 80.4 vs 77.6 us,
  // profiles/r06/README.md)
  constexpr int NW = 4;
  const int T = a.T;
  const bool par = T <= kParSteps;
  const size_t coef = a.coef ? static_cast<size_t>(a.L) * T * 5 : 0;
  const size_t floats =
      MODE == kSrcPred ? static_cast<size_t>(kFP) * (2 * T + 1)
                       : static_cast<size_t>(kFP) * (2 * T + (par ? 2 * T + 2 : 0)) +
                             std::max(par ? static_cast<size_t>(kFP) * 6 * T : 0, coef);
  const size_t lds = floats * sizeof(float);
  if (!lds_fits(&place_kernel<MODE, NW>, lds)) {
    set_error("ccmpc_sample_bucket: hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
    return CCMPC_ERR_LAUNCH;
  }
  const dim3 grid(static_cast<unsigned>(a.G), static_cast<unsigned>(n_ov));
  hipLaunchKernelGGL((place_kernel<MODE, NW>), grid, dim3(64 * NW), lds, s, a);
  return CCMPC_OK;
}

// P0 -> P1 -> the rare stage, for either particle source (pred != nullptr: the predictor's).
// Small sampler clouds: P1 = sample_place_kernel (8-wave blocks, a few per CU); large ones and
// the predictor's: place_kernel
// The step's input pack: n 16-byte words from the pinned host side src to the device side dst
struct PackCopy {
  uint4 *dst;
  const uint4 *src;
  size_t n;
};

// p itself, or its image on the host side when it points into the pack's device side
template <typename T>
inline T *pack_host_image(T *p, const PackCopy &k) {
  const char *c = reinterpret_cast<const char *>(p), *lo = reinterpret_cast<const char *>(k.dst);
  if (!p || c < lo || c >= lo + 16 * k.n) return p;
  return reinterpret_cast<T *>(
      const_cast<char *>(reinterpret_cast<const char *>(k.src) + (c - lo)));
}

template <int ZSRC>
inline void launch_latents(const FusedArgs &a, int64_t n_ov, const PackCopy *pk, hipStream_t s) {
  if (!pk || pk->n == 0) {
    const dim3 zgrid(static_cast<unsigned>(a.nb0), static_cast<unsigned>(n_ov));
    hipLaunchKernelGGL(latent_count_kernel<ZSRC>, zgrid, dim3(kFThreads), 0, s, a);
    return;
  }
  FusedArgs ah = a;  // P0's inputs from the host side of the pack
  ah.latent_cdf = pack_host_image(a.latent_cdf, *pk);
  ah.gmm = pack_host_image(a.gmm, *pk);
  ah.z_in = pack_host_image(a.z_in, *pk);
  ah.zsrc = pack_host_image(a.zsrc, *pk);
  ah.rows = pack_host_image(a.rows, *pk);
  ah.ptrs = pack_host_image(a.ptrs, *pk);
  ah.seed_dev = pack_host_image(a.seed_dev, *pk);
  ah.keep_map = pack_host_image(a.keep_map, *pk);
  ah.n_kept = pack_host_image(a.n_kept, *pk);
  const size_t per = static_cast<size_t>(kFThreads) * 4;
  const int ncopy = static_cast<int>(std::min<size_t>(64, (pk->n + per - 1) / per));
  const unsigned grid = static_cast<unsigned>(ncopy + a.nb0 * n_ov);
  hipLaunchKernelGGL(copy_latent_count_kernel<ZSRC>, dim3(grid), dim3(kFThreads), 0, s, ah,
                     pk->dst, pk->src, pk->n, ncopy);
}

inline int fused_launch(FusedArgs &a, int64_t n_ov, bool pp, hipStream_t s,
                        const PackCopy *pk = nullptr) {
  // write-through particle stores need every byte offset within the 31-bit buffer range
  a.wt = (int64_t(8) * a.T * a.ld_out < (int64_t(1) << 31)) &&
         (int64_t(8) * a.T * a.Npad < (int64_t(1) << 31));
  if (a.pred)
    launch_latents<kZPred>(a, n_ov, pk, s);
  else if (a.z_in)
    launch_latents<kZIn>(a, n_ov, pk, s);
  else
    launch_latents<kZPhilox>(a, n_ov, pk, s);
  const bool eps = a.eps_in != nullptr;
  const dim3 grid(static_cast<unsigned>(a.G), static_cast<unsigned>(n_ov));
  int rc = CCMPC_OK;
  if (a.pred) {
    rc = launch_place<kSrcPred>(a, n_ov, s);
  } else if (a.N > kFusedMaxN) {
    switch ((pp ? 2 : 0) | (eps ? 1 : 0)) {
      case 0: rc = launch_place<0>(a, n_ov, s); break;
      case 1: rc = launch_place<1>(a, n_ov, s); break;
      case 2: rc = launch_place<2>(a, n_ov, s); break;
      default: rc = launch_place<3>(a, n_ov, s); break;
    }
  } else {
#define CCMPC_FUSED(PP, EPSIN) \
  hipLaunchKernelGGL((sample_place_kernel<PP, EPSIN>), grid, dim3(kFThreads), 0, s, a)
    switch ((pp ? 2 : 0) | (eps ? 1 : 0)) {
      case 0: CCMPC_FUSED(false, false); break;
      case 1: CCMPC_FUSED(false, true); break;
      case 2: CCMPC_FUSED(true, false); break;
      default: CCMPC_FUSED(true, true); break;
    }
#undef CCMPC_FUSED
  }
  if (rc != CCMPC_OK) return rc;
  if (rare_two_pass(a.N)) {
    const dim3 kgrid(static_cast<unsigned>(a.nkb), static_cast<unsigned>(n_ov));
    hipLaunchKernelGGL(rare_key_kernel, kgrid, dim3(kRThreads), 0, s, a);
    const dim3 cgrid(static_cast<unsigned>((a.Npad + kRThreads - 1) / kRThreads),
                     static_cast<unsigned>(n_ov));
    if (a.T <= 8)
      hipLaunchKernelGGL(rare_copy_kernel<16>, cgrid, dim3(kRThreads), 0, s, a);
    else
      hipLaunchKernelGGL(rare_copy_kernel<80>, cgrid, dim3(kRThreads), 0, s, a);
  } else {
    const dim3 rgrid(static_cast<unsigned>((a.N + kRThreads - 1) / kRThreads),
                     static_cast<unsigned>(n_ov));
    if (a.T <= 8)
      hipLaunchKernelGGL((rare_place_kernel<16, 2 * CCMPC_RARE_BATCH>), rgrid, dim3(kRThreads), 0,
                         s, a);
    else
      hipLaunchKernelGGL((rare_place_kernel<80, CCMPC_RARE_BATCH>), rgrid, dim3(kRThreads), 0, s,
                         a);
  }
  return CCMPC_OK;
}

inline void fused_args_ws(FusedArgs &a, const FusedWs &L, void *workspace) {
  char *ws = static_cast<char *>(workspace);
  a.zbuf = reinterpret_cast<int32_t *>(ws + L.zbuf);
  a.gcnt = reinterpret_cast<int32_t *>(ws + L.gcnt);
  a.bsum = reinterpret_cast<int32_t *>(ws + L.bsum);
  a.hdr = reinterpret_cast<int32_t *>(ws + L.hdr);
  a.gpart = reinterpret_cast<double *>(ws + L.gpart);
  a.rinfo = reinterpret_cast<float *>(ws + L.rinfo);
  a.rstore = reinterpret_cast<float *>(ws + L.rstore);
  a.kbuf = reinterpret_cast<int32_t *>(ws + L.kbuf);
  a.rhist = reinterpret_cast<int32_t *>(ws + L.rhist);
  a.coef = nullptr;                      // set by ccmpc_sample_bucket for the per-latent P1
  a.Npad = L.Npad;
  a.G = static_cast<int>(L.G);
  a.nb0 = static_cast<int>(L.nb0);
  a.nkb = static_cast<int>(L.nkb);
}

}  // namespace ccmpc

using namespace ccmpc;

#if defined(CCMPC_PROBE) && (CCMPC_PROBE & 4)
// which 0: P0 latents (slots 0 start, 1 done); 1: P1 place (0 start, 1 counted, 2 sampled +
// published; place_kernel: 0 start, 1 loaded, 2 acted, 3 sincos, 4 chained, 5 summed); 2: P2
// rares (0 start, 1 loaded, 2 centres, 3 keyed, 4 bin starts, 5 ranked, 6 copied); 3: P2 keys
// (0 start, 1 loaded, 2 superblocks, 3 centres, 4 keyed); 4: P3 copy (0 start, 1 loaded, 2
// counted, 3 ranked, 4 copied)  (tools/probe_step.py)
extern "C" int ccmpc_probe_fused_timestamps(void *host, int which, int reset) {
  if (which < 0 || which > 4) return -1;
  const size_t bytes = sizeof(g_fused_ts[0]);
  if (reset) {
    static unsigned long long zeros[kStepProbeWG * kStepProbeSlots];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_fused_ts), zeros, bytes, which * bytes) == hipSuccess
               ? 0 : -1;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fused_ts), bytes, which * bytes) == hipSuccess
             ? 0 : -1;
}
#endif

extern "C" size_t ccmpc_sample_bucket_workspace_bytes(int64_t n_ov, int64_t N, int64_t T,
                                                      int64_t max_k) {
  if (n_ov < 0 || N < 1 || N > kWideMaxN || T < 1 || T > 40 || max_k < 1 || max_k > kMaxKept)
    return 0;
  return fused_ws(n_ov, N, T, max_k).total;
}

// The pack arguments of the *_packed entry points, checked
static bool pack_args(void *pack_dev, const void *pack_host, size_t pack_bytes, PackCopy &pk) {
  if (!pack_dev || !pack_host || pack_bytes % 16 != 0 || !aligned(pack_dev, 16) ||
      !aligned(pack_host, 16)) {
    set_error("pack: null, or bytes and pointers not 16-byte aligned");
    return false;
  }
  pk = PackCopy{static_cast<uint4 *>(pack_dev), static_cast<const uint4 *>(pack_host),
                pack_bytes / 16};
  return true;
}

static int sample_bucket_impl(const double *init_state, const double *latent_cdf,
                              int64_t n_latent, const float *gmm, int32_t gmm_layout,
                              const int32_t *z_in, const float *eps_in, int64_t n_ov, int64_t N,
                              int64_t T, double dt, uint64_t seed, const uint64_t *seed_dev,
                              int64_t ov_base, const int32_t *keep_map, const int32_t *n_kept,
                              const int32_t *cell_base, int64_t max_k, const double *minpos,
                              const int64_t *region, void *workspace, size_t workspace_bytes,
                              int32_t *out_z, float *pos_out, int64_t ld_out, int64_t *cell_off,
                              int64_t *cell_cnt, double *cell_pmf, double *init_center,
                              ccmpc_stream_t stream, const PackCopy *pk) {
  CCMPC_REQUIRE(T >= 1 && T <= 40, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_latent >= 1 && n_latent <= 64, "n_latent must be in [1, 64]");
  CCMPC_REQUIRE(N >= 1 && N <= kWideMaxN, "N must be in [1, 262144] (bucket.hip beyond)");
  CCMPC_REQUIRE(max_k >= 1 && max_k <= kMaxKept && max_k * (n_latent + 1) <= kFusedMaxBins,
                "max_k out of range");
  CCMPC_REQUIRE(n_ov >= 0 && n_ov < 65536, "bad n_ov");
  CCMPC_REQUIRE(ov_base >= 0 && ov_base + n_ov <= (int64_t(1) << 32), "bad ov_base");
  CCMPC_REQUIRE(gmm_layout == CCMPC_GMM_PER_LATENT || gmm_layout == CCMPC_GMM_PER_PARTICLE,
                "bad gmm_layout");
  const bool pp = gmm_layout == CCMPC_GMM_PER_PARTICLE;
  CCMPC_REQUIRE(!pp || z_in, "per-particle GMM parameters need the injected z_in");
  if (n_ov == 0) return CCMPC_OK;
  CCMPC_REQUIRE(init_state && gmm && keep_map && n_kept && cell_base && minpos && region &&
                    pos_out && cell_off && cell_cnt && cell_pmf && init_center,
                "null pointer");
  CCMPC_REQUIRE(z_in || latent_cdf, "latent_cdf is needed when z is drawn here");
  CCMPC_REQUIRE(ld_out >= 1 && ld_out * 2 * T < (int64_t(1) << 40), "bad ld_out");
  const FusedWs L = fused_ws(n_ov, N, T, max_k);
  if (!workspace || workspace_bytes < L.total || !aligned(workspace, 256)) {
    set_error("ccmpc_sample_bucket: workspace too small or not 256-byte aligned");
    return CCMPC_ERR_WORKSPACE;
  }
  FusedArgs a = {};
  a.init_state = init_state;
  a.latent_cdf = latent_cdf;
  a.gmm = gmm;
  a.eps_in = eps_in;
  a.z_in = z_in;
  a.L = static_cast<int>(n_latent);
  a.T = static_cast<int>(T);
  a.N = N;
  a.dt = static_cast<float>(dt);
  a.seed = seed;
  a.seed_dev = seed_dev;
  a.ov_base = static_cast<uint32_t>(ov_base);
  a.keep_map = keep_map;
  a.n_kept = n_kept;
  a.cell_base = cell_base;
  a.max_k = static_cast<int>(max_k);
  a.minpos = minpos;
  a.region = region;
  fused_args_ws(a, L, workspace);
  a.out_z = out_z;
  a.out = pos_out;
  a.ld_out = ld_out;
  a.cell_off = cell_off;
  a.cell_cnt = cell_cnt;
  a.cell_pmf = cell_pmf;
  a.init_center = init_center;
  if (N > kFusedMaxN && !pp && n_latent * T * 5 <= kActCoef)
    a.coef = reinterpret_cast<float *>(static_cast<char *>(workspace) + L.coef);
  const int rc = fused_launch(a, n_ov, pp, as_stream(stream), pk);
  if (rc != CCMPC_OK) return rc;
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}

#define CCMPC_SAMPLE_BUCKET_PARAMS                                                             \
  const double *init_state, const double *latent_cdf, int64_t n_latent, const float *gmm,      \
      int32_t gmm_layout, const int32_t *z_in, const float *eps_in, int64_t n_ov, int64_t N,   \
      int64_t T, double dt, uint64_t seed, const uint64_t *seed_dev, int64_t ov_base,          \
      const int32_t *keep_map, const int32_t *n_kept, const int32_t *cell_base, int64_t max_k, \
      const double *minpos, const int64_t *region, void *workspace, size_t workspace_bytes,    \
      int32_t *out_z, float *pos_out, int64_t ld_out, int64_t *cell_off, int64_t *cell_cnt,    \
      double *cell_pmf, double *init_center, ccmpc_stream_t stream
#define CCMPC_SAMPLE_BUCKET_ARGS                                                               \
  init_state, latent_cdf, n_latent, gmm, gmm_layout, z_in, eps_in, n_ov, N, T, dt, seed,       \
      seed_dev, ov_base, keep_map, n_kept, cell_base, max_k, minpos, region, workspace,        \
      workspace_bytes, out_z, pos_out, ld_out, cell_off, cell_cnt, cell_pmf, init_center, stream

extern "C" int ccmpc_sample_bucket(CCMPC_SAMPLE_BUCKET_PARAMS) {
  return sample_bucket_impl(CCMPC_SAMPLE_BUCKET_ARGS, nullptr);
}

extern "C" int ccmpc_sample_bucket_packed(void *pack_dev, const void *pack_host,
                                          size_t pack_bytes, CCMPC_SAMPLE_BUCKET_PARAMS) {
  PackCopy pk;
  if (!pack_args(pack_dev, pack_host, pack_bytes, pk)) return CCMPC_ERR_ARG;
  return sample_bucket_impl(CCMPC_SAMPLE_BUCKET_ARGS, &pk);
}

static int bucket_predictions_impl(const float *pred, const void *z, const uint64_t *ptrs,
                                   int z_bytes, const int32_t *rows, int64_t n_ov, int64_t N,
                                   int64_t T, int64_t n_latent, const int32_t *keep_map,
                                   const int32_t *n_kept, const int32_t *cell_base,
                                   int64_t max_k, const double *minpos, const int64_t *region,
                                   void *workspace, size_t workspace_bytes, float *pos_out,
                                   int64_t ld_out, int64_t *cell_off, int64_t *cell_cnt,
                                   double *cell_pmf, double *init_center, int32_t *z_bad,
                                   ccmpc_stream_t stream, const PackCopy *pk = nullptr) {
  CCMPC_REQUIRE(T >= 1 && T <= 40, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_latent >= 1 && n_latent <= 64, "n_latent must be in [1, 64]");
  CCMPC_REQUIRE(N >= 1 && N <= kWideMaxN, "N must be in [1, 262144] (ccmpc_load_predictions + "
                "ccmpc_bucket beyond)");
  CCMPC_REQUIRE(z_bytes == 4 || z_bytes == 8, "z must be int32 or int64");
  CCMPC_REQUIRE(max_k >= 1 && max_k <= kMaxKept && max_k * (n_latent + 1) <= kFusedMaxBins,
                "max_k out of range");
  CCMPC_REQUIRE(n_ov >= 0 && n_ov < 65536, "bad n_ov");
  if (n_ov == 0) return CCMPC_OK;
  CCMPC_REQUIRE(((pred && z) || ptrs) && keep_map && n_kept && cell_base && minpos && region &&
                    pos_out && cell_off && cell_cnt && cell_pmf && init_center,
                "null pointer");
  CCMPC_REQUIRE(ld_out >= 1 && ld_out * 2 * T < (int64_t(1) << 40), "bad ld_out");
  const FusedWs L = fused_ws(n_ov, N, T, max_k);
  if (!workspace || workspace_bytes < L.total || !aligned(workspace, 256)) {
    set_error("ccmpc_bucket_predictions: workspace too small or not 256-byte aligned");
    return CCMPC_ERR_WORKSPACE;
  }
  FusedArgs a = {};
  a.pred = ptrs ? reinterpret_cast<const float *>(ptrs) : pred;  // (non-null: the source)
  a.zsrc = z;
  a.ptrs = ptrs;
  a.z_bytes = z_bytes;
  a.rows = rows;
  a.L = static_cast<int>(n_latent);
  a.T = static_cast<int>(T);
  a.N = N;
  a.keep_map = keep_map;
  a.n_kept = n_kept;
  a.cell_base = cell_base;
  a.max_k = static_cast<int>(max_k);
  a.minpos = minpos;
  a.region = region;
  fused_args_ws(a, L, workspace);
  a.out = pos_out;
  a.ld_out = ld_out;
  a.cell_off = cell_off;
  a.cell_cnt = cell_cnt;
  a.cell_pmf = cell_pmf;
  a.init_center = init_center;
  a.z_bad = z_bad;
  const int rc = fused_launch(a, n_ov, false, as_stream(stream), pk);
  if (rc != CCMPC_OK) return rc;
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}

extern "C" int ccmpc_bucket_predictions(const float *pred, const void *z, int z_bytes,
                                        const int32_t *rows, int64_t n_ov, int64_t N, int64_t T,
                                        int64_t n_latent, const int32_t *keep_map,
                                        const int32_t *n_kept, const int32_t *cell_base,
                                        int64_t max_k, const double *minpos,
                                        const int64_t *region, void *workspace,
                                        size_t workspace_bytes, float *pos_out, int64_t ld_out,
                                        int64_t *cell_off, int64_t *cell_cnt, double *cell_pmf,
                                        double *init_center, int32_t *z_bad,
                                        ccmpc_stream_t stream) {
  return bucket_predictions_impl(pred, z, nullptr, z_bytes, rows, n_ov, N, T, n_latent, keep_map,
                                 n_kept, cell_base, max_k, minpos, region, workspace,
                                 workspace_bytes, pos_out, ld_out, cell_off, cell_cnt, cell_pmf,
                                 init_center, z_bad, stream);
}

extern "C" int ccmpc_bucket_predictions_indirect(const uint64_t *ptrs, int z_bytes,
                                                 const int32_t *rows, int64_t n_ov, int64_t N,
                                                 int64_t T, int64_t n_latent,
                                                 const int32_t *keep_map, const int32_t *n_kept,
                                                 const int32_t *cell_base, int64_t max_k,
                                                 const double *minpos, const int64_t *region,
                                                 void *workspace, size_t workspace_bytes,
                                                 float *pos_out, int64_t ld_out,
                                                 int64_t *cell_off, int64_t *cell_cnt,
                                                 double *cell_pmf, double *init_center,
                                                 int32_t *z_bad, ccmpc_stream_t stream) {
  CCMPC_REQUIRE(ptrs, "null ptrs");
  return bucket_predictions_impl(nullptr, nullptr, ptrs, z_bytes, rows, n_ov, N, T, n_latent,
                                 keep_map, n_kept, cell_base, max_k, minpos, region, workspace,
                                 workspace_bytes, pos_out, ld_out, cell_off, cell_cnt, cell_pmf,
                                 init_center, z_bad, stream);
}

extern "C" int ccmpc_bucket_predictions_packed(
    void *pack_dev, const void *pack_host, size_t pack_bytes, const float *pred, const void *z,
    int z_bytes, const int32_t *rows, int64_t n_ov, int64_t N, int64_t T, int64_t n_latent,
    const int32_t *keep_map, const int32_t *n_kept, const int32_t *cell_base, int64_t max_k,
    const double *minpos, const int64_t *region, void *workspace, size_t workspace_bytes,
    float *pos_out, int64_t ld_out, int64_t *cell_off, int64_t *cell_cnt, double *cell_pmf,
    double *init_center, int32_t *z_bad, ccmpc_stream_t stream) {
  PackCopy pk;
  if (!pack_args(pack_dev, pack_host, pack_bytes, pk)) return CCMPC_ERR_ARG;
  return bucket_predictions_impl(pred, z, nullptr, z_bytes, rows, n_ov, N, T, n_latent, keep_map,
                                 n_kept, cell_base, max_k, minpos, region, workspace,
                                 workspace_bytes, pos_out, ld_out, cell_off, cell_cnt, cell_pmf,
                                 init_center, z_bad, stream, &pk);
}

extern "C" int ccmpc_bucket_predictions_indirect_packed(
    void *pack_dev, const void *pack_host, size_t pack_bytes, const uint64_t *ptrs, int z_bytes,
    const int32_t *rows, int64_t n_ov, int64_t N, int64_t T, int64_t n_latent,
    const int32_t *keep_map, const int32_t *n_kept, const int32_t *cell_base, int64_t max_k,
    const double *minpos, const int64_t *region, void *workspace, size_t workspace_bytes,
    float *pos_out, int64_t ld_out, int64_t *cell_off, int64_t *cell_cnt, double *cell_pmf,
    double *init_center, int32_t *z_bad, ccmpc_stream_t stream) {
  CCMPC_REQUIRE(ptrs, "null ptrs");
  PackCopy pk;
  if (!pack_args(pack_dev, pack_host, pack_bytes, pk)) return CCMPC_ERR_ARG;
  return bucket_predictions_impl(nullptr, nullptr, ptrs, z_bytes, rows, n_ov, N, T, n_latent,
                                 keep_map, n_kept, cell_base, max_k, minpos, region, workspace,
                                 workspace_bytes, pos_out, ld_out, cell_off, cell_cnt, cell_pmf,
                                 init_center, z_bad, stream, &pk);
}
