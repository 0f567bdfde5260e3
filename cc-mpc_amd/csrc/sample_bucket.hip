// Sampler + bucketing for small clouds (N <= 8192 particles per OV): the drop-in step's
// do_prediction -> make_ovehicles (prediction.py:81-86, v8ideal/__init__.py:469-505,
// ovehicle.py:24-117) in three short launches instead of the sampler and bucket.hip's three.
//
// What makes the four-launch form slow is not work but dependent memory round trips: each of
// bucket.hip's kernels re-reads the particles, exchanges partials through memory and ends, and
// the next starts cold (tools/probe_step.py: ~10 us per kernel).  Here:
//
//  P0 latents  one latent id per particle (Philox + CDF count, or the injected z) and each
//              64-particle group's count per category -- kept mode k or "rare".
//  P1 place    per block of 64 particles (512 threads): the category counts of the groups before
//              its own and in total (a few KB of reads summed in LDS; an earlier form redrew every
//              latent of the OV in every block: 13-20 us of Philox).  No exchange is needed to
//              know where a kept mode's own particles go: cell k of the OV starts at
//                  region + sum_{j < k} round4(n_j + R)       (R = the OV's rare count)
//              so it can take its n_j natives AND, in the worst case, every rare particle; its
//              natives go to  start_k + (natives of k before this block) + (rank in the block).
//              Then the sampler's two phases (actions in parallel, then the Unicycle chain on
//              one wave); the chain writes a native particle's 2T coordinates straight into its
//              cell, and a rare particle's into a rare list in sample order, with its final
//              position and latent id; and the block's kept-mode sums of the final world
//              positions (= one 64-particle centre group, bucket.hpp).
//  P2 rares    per block of 256 rare-list slots: the centres in the canonical order (bucket.hpp,
//              so they equal bucket.hip's bit for bit), the key (owner, latent) of EVERY rare
//              particle of the OV -- a few KB of L2 reads -- counted per bin in LDS in total and
//              before the block's first slot, so the block knows each bin's start and its own
//              particles' stable ranks in sample order without any exchange; then the copy of
//              its rare particles' coordinates into the owners' cells after the natives.  Block
//              0 writes cell offsets, counts, pmf and centres.
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

constexpr int kFusedMaxN = 8192;
constexpr int kFusedMaxBins = 512;
constexpr int kFP = 64;                       // particles per P1 block (the chain wave)
constexpr int kFThreads = 512;                // 8 waves
constexpr int kFWaves = kFThreads / 64;
constexpr int kFGroups = kFusedMaxN / kFP;    // centre groups (P1 blocks) per OV at most
constexpr int kParSteps = 16;                 // P1: horizons whose step terms run in parallel
constexpr int kRThreads = 256;                // P2: rare-list slots per block
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
// per-group category counts: kept modes 0..K-1, then the rare count
constexpr int kCntStride = 32;
static_assert(kMaxKept + 1 <= 2 * kMaxKept, "tot[] must end before the cell starts");
static_assert(4 * kMaxKept <= kHdrInts, "cell starts (int64) must fit the per-OV header");
static_assert(kCntStride >= kMaxKept + 1, "group counts: one slot per kept mode + rare");
#if defined(CCMPC_PROBE) && (CCMPC_PROBE & 4)
__device__ unsigned long long g_fused_ts[3][kStepProbeWG * kStepProbeSlots];
#define FUSED_TS(kern, k) CCMPC_STEP_TS(g_fused_ts[kern], k)
#else
#define FUSED_TS(kern, k) CCMPC_STEP_TS(nullptr, k)
#endif

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
  // bucketing (bucket.hip)
  const int32_t *keep_map, *n_kept, *cell_base;
  int max_k;
  const double *minpos;
  const int64_t *region;
  // workspace (written by P1, read by P2; the kernel boundary orders them)
  int32_t *zbuf;   // [n_ov][Npad]: latent ids (P0)
  int32_t *gcnt;   // [n_ov][G][kCntStride]: per 64-particle group category counts (P0)
  int32_t *hdr;    // [n_ov][kHdrInts]: category totals [K + 1], then cell starts (int64) [K]
  double *gpart;   // [n_ov][G][max_k][2]
  float *rinfo;    // [n_ov][Npad][4]: rare particle's final (x, y), latent id (bits), 0
  float *rstore;   // [n_ov][2T][Npad]: rare particles' coordinates, rare-list order
  int64_t Npad;
  int G;
  // outputs
  int32_t *out_z;  // optional sample-order latent ids
  float *out;
  int64_t ld_out;
  int64_t *cell_off, *cell_cnt;
  double *cell_pmf, *init_center;
};

__device__ __forceinline__ int64_t *hdr_starts(int32_t *h) {
  return reinterpret_cast<int64_t *>(h + 2 * kMaxKept);
}

// P0: one latent id per particle (Philox inverse CDF, or the injected z) into the workspace, and
// each 64-particle group's count per category (kept mode k, or K = rare) -- one wave = one group.
template <bool ZIN>
__global__ __launch_bounds__(kFThreads) void latent_count_kernel(FusedArgs a) {
  __shared__ double cdf_s[64];
  __shared__ int keep_s[64];
  FUSED_TS(0, 0);
  const int o = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int K = a.n_kept[o], L = a.L;
  const int64_t N = a.N;
  if (!ZIN && tid < L) cdf_s[tid] = a.latent_cdf[static_cast<int64_t>(o) * L + tid];
  if (tid < L) keep_s[tid] = a.keep_map[o * L + tid];
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kFThreads + tid;
  const bool v = i < N;
  int z = 0;
  if (ZIN && v) {
    z = a.z_in[static_cast<int64_t>(o) * N + i];
    z = z < 0 ? 0 : (z >= L ? L - 1 : z);  // memory safety; the host validates
  }
  __syncthreads();
  if (!ZIN && v)
    z = draw_latent(i, a.ov_base + static_cast<uint32_t>(o), a.seed_dev ? *a.seed_dev : a.seed,
                    cdf_s, L);
  if (v) {
    a.zbuf[static_cast<int64_t>(o) * a.Npad + i] = z;
    if (a.out_z) a.out_z[static_cast<int64_t>(o) * N + i] = z;
  }
  const int kk = keep_s[z];
  const int cat = kk >= 0 ? kk : K;
  const int g = blockIdx.x * kFWaves + w;
  int mine = 0;
  for (int c = 0; c <= K; ++c) {
    const int n = __popcll(__ballot(v && cat == c));
    if (lane == c) mine = n;
  }
  if (g < a.G && lane <= K) a.gcnt[(static_cast<int64_t>(o) * a.G + g) * kCntStride + lane] = mine;
  FUSED_TS(0, 1);
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
    for (int e = tid; e < gsz; e += kFThreads) gmm_s[e] = a.gmm[static_cast<int64_t>(o) * gsz + e];
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
  float v[80];
#pragma unroll
  for (int rr = 0; rr < 80; ++rr)
    if (rr < rows) v[rr] = src[static_cast<int64_t>(rr) * npad];
  const int ng = a.G * K;
  const double2 *gp = reinterpret_cast<const double2 *>(a.gpart) + static_cast<int64_t>(o) * a.G * a.max_k;
  for (int u = tid; u < ng; u += kRThreads) gp_s[u] = gp[(u / K) * a.max_k + u % K];
  if (tid == 0) gp_s[kFGroups * kMaxKept] = double2{-0.0, -0.0};  // superblock_sum's sentinel
  // the first batch of rare records too: R is not known yet, so the slots are clamped into the
  // list's storage (a launch's first kB * 256 records cover the C2 shape's whole rare list)
  const float4 *info = reinterpret_cast<const float4 *>(a.rinfo) + static_cast<int64_t>(o) * npad;
  constexpr int kB = CCMPC_RARE_BATCH;
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
    for (int rr = 0; rr < 80; ++rr)
      if (rr < rows) out[static_cast<int64_t>(rr) * a.ld_out] = v[rr];
  }
  FUSED_TS(2, 6);
}

struct FusedWs {
  size_t zbuf, gcnt, hdr, gpart, rinfo, rstore, total;
};

inline size_t a256(size_t b) { return (b + 255) / 256 * 256; }

inline FusedWs fused_ws(int64_t n_ov, int64_t N, int64_t T, int64_t max_k) {
  const int64_t G = (N + kFP - 1) / kFP, Npad = (N + 3) & ~int64_t(3);
  FusedWs w;
  size_t o = 0;
  w.zbuf = o;
  o += a256(sizeof(int32_t) * n_ov * Npad);
  w.gcnt = o;
  o += a256(sizeof(int32_t) * n_ov * G * kCntStride);
  w.hdr = o;
  o += a256(sizeof(int32_t) * kHdrInts * n_ov);
  w.gpart = o;
  o += a256(sizeof(double) * 2 * n_ov * G * max_k);
  w.rinfo = o;
  o += a256(sizeof(float) * 4 * n_ov * Npad);
  w.rstore = o;
  o += a256(sizeof(float) * n_ov * 2 * T * Npad);
  w.total = o;
  return w;
}

}  // namespace ccmpc

using namespace ccmpc;

#if defined(CCMPC_PROBE) && (CCMPC_PROBE & 4)
// which 0: P0 latents (slots 0 start, 1 done); 1: P1 place (0 start, 1 counted, 2 sampled +
// published); 2: P2 rares (0 start, 1 loaded, 2 centres, 3 keyed, 4 bin starts, 5 ranked,
// 6 copied)  (tools/probe_step.py)
extern "C" int ccmpc_probe_fused_timestamps(void *host, int which, int reset) {
  if (which < 0 || which > 2) return -1;
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
  if (n_ov < 0 || N < 1 || N > kFusedMaxN || T < 1 || T > 40 || max_k < 1 || max_k > kMaxKept)
    return 0;
  return fused_ws(n_ov, N, T, max_k).total;
}

extern "C" int ccmpc_sample_bucket(const double *init_state, const double *latent_cdf,
                                   int64_t n_latent, const float *gmm, int32_t gmm_layout,
                                   const int32_t *z_in, const float *eps_in, int64_t n_ov,
                                   int64_t N, int64_t T, double dt, uint64_t seed,
                                   const uint64_t *seed_dev, int64_t ov_base,
                                   const int32_t *keep_map, const int32_t *n_kept,
                                   const int32_t *cell_base, int64_t max_k, const double *minpos,
                                   const int64_t *region, void *workspace,
                                   size_t workspace_bytes, int32_t *out_z, float *pos_out,
                                   int64_t ld_out, int64_t *cell_off, int64_t *cell_cnt,
                                   double *cell_pmf, double *init_center, ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T >= 1 && T <= 40, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_latent >= 1 && n_latent <= 64, "n_latent must be in [1, 64]");
  CCMPC_REQUIRE(N >= 1 && N <= kFusedMaxN, "N must be in [1, 8192] (bucket.hip beyond)");
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
  char *ws = static_cast<char *>(workspace);
  FusedArgs a;
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
  a.zbuf = reinterpret_cast<int32_t *>(ws + L.zbuf);
  a.gcnt = reinterpret_cast<int32_t *>(ws + L.gcnt);
  a.hdr = reinterpret_cast<int32_t *>(ws + L.hdr);
  a.gpart = reinterpret_cast<double *>(ws + L.gpart);
  a.rinfo = reinterpret_cast<float *>(ws + L.rinfo);
  a.rstore = reinterpret_cast<float *>(ws + L.rstore);
  a.Npad = (N + 3) & ~int64_t(3);
  a.G = static_cast<int>((N + kFP - 1) / kFP);
  a.out_z = out_z;
  a.out = pos_out;
  a.ld_out = ld_out;
  a.cell_off = cell_off;
  a.cell_cnt = cell_cnt;
  a.cell_pmf = cell_pmf;
  a.init_center = init_center;
  hipStream_t s = as_stream(stream);
  const dim3 zgrid(static_cast<unsigned>((N + kFThreads - 1) / kFThreads),
                   static_cast<unsigned>(n_ov));
  if (z_in)
    hipLaunchKernelGGL(latent_count_kernel<true>, zgrid, dim3(kFThreads), 0, s, a);
  else
    hipLaunchKernelGGL(latent_count_kernel<false>, zgrid, dim3(kFThreads), 0, s, a);
  const dim3 grid(static_cast<unsigned>(a.G), static_cast<unsigned>(n_ov));
  const int mode = (pp ? 2 : 0) | (eps_in ? 1 : 0);
#define CCMPC_FUSED(PP, EPSIN) \
  hipLaunchKernelGGL((sample_place_kernel<PP, EPSIN>), grid, dim3(kFThreads), 0, s, a)
  switch (mode) {
    case 0: CCMPC_FUSED(false, false); break;
    case 1: CCMPC_FUSED(false, true); break;
    case 2: CCMPC_FUSED(true, false); break;
    default: CCMPC_FUSED(true, true); break;
  }
#undef CCMPC_FUSED
  const dim3 rgrid(static_cast<unsigned>((N + kRThreads - 1) / kRThreads),
                   static_cast<unsigned>(n_ov));
  hipLaunchKernelGGL(rare_place_kernel, rgrid, dim3(kRThreads), 0, s, a);
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}
