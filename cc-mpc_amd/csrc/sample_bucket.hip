// Fused sampler + bucketing for small clouds (N <= 8192 particles per OV): the drop-in step's
// do_prediction -> make_ovehicles (prediction.py:81-86, v8ideal/__init__.py:469-505,
// ovehicle.py:24-117) in ONE launch instead of the sampler and bucket.hip's three kernels.
//
// What made the four-launch form slow was not work but dependent memory round trips: each of
// bucket.hip's kernels re-reads the particles, exchanges partials through memory and ends, and
// the next starts cold (measured, tools/probe_step.py: ~10 us per kernel, 35 us for the three).
// Here the bucketing rides on the sampler's blocks (64 particles, 512 threads each):
//
//   counts   every block redraws the latent ids of its whole OV (one Philox + CDF search per
//            particle; or reads the injected z) and counts them per category -- kept mode k or
//            "rare" -- before its own first particle and in total.  No exchange is needed to know
//            where a kept mode's own particles go: cell k of the OV starts at
//                region + sum_{j < k} round4(n_j + R)       (R = the OV's rare count)
//            so it can take its n_j natives AND, in the worst case, every rare particle; its
//            natives go to  start_k + (natives of k before this block) + (rank in the block).
//   sample   the sampler's two phases (actions in parallel, then the Unicycle chain on one wave);
//            the chain writes a native particle's 2T coordinates straight into its cell, and a
//            rare particle's into a rare list in sample order (write-through), with its final
//            position and latent id.
//   centres  per block (= one 64-particle centre group, bucket.hpp), the kept-mode sums of the
//            final world positions, published write-through.
//   rares    the OV's last arriving block: centres in the canonical order (bucket.hpp, so they
//            equal bucket.hip's bit for bit), the owner of every rare particle, a stable counting
//            sort of the rare list by (owner, latent) in sample order, and the copy of each rare
//            particle's coordinates into its owner's cell after the natives; cell offsets,
//            counts, pmf and centres.
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
constexpr int kFP = 64;                       // particles per block (the chain wave)
constexpr int kFThreads = 512;                // 8 waves
constexpr int kFWaves = kFThreads / 64;
constexpr int kFGroups = kFusedMaxN / kFP;    // centre groups (blocks) per OV at most
#if defined(CCMPC_PROBE) && (CCMPC_PROBE & 4)
__device__ unsigned long long g_fused_ts[kStepProbeWG * kStepProbeSlots];
#endif
#define FUSED_TS(k) CCMPC_STEP_TS(g_fused_ts, k)

constexpr int kFPrefetch = 32;                // rare-copy elements per thread loaded up front

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
  // workspace
  int32_t *ctr;    // [n_ov] arrival counters (zero between calls)
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

union FusedSmem {
  struct {
    float act[2][40][kFP];
    float gmm[64 * 40 * 5 / 4];
  } s;                                  // sampling
  double2 gp[kFGroups * kMaxKept];      // last arriver: the centre groups' partials
  struct {
    int32_t rk[kFusedMaxN];             // rare r: its key, then key << 16 | rank in its bin
    int32_t run[kFusedMaxBins];         // rare particles of each bin in earlier rounds
    int32_t wcnt[kFWaves][kFusedMaxBins];
    int32_t bstart[kFusedMaxBins];      // bin start relative to the region
  } r;                                  // rare ranking
};

template <bool PP, bool ZIN, bool EPSIN>
__global__ __launch_bounds__(kFThreads) void sample_bucket_kernel(FusedArgs a) {
  __shared__ FusedSmem sm;
  __shared__ double cdf_s[64];
  __shared__ int keep_s[64];
  __shared__ int zs[kFP];
  __shared__ int wc[kFWaves][2][kMaxKept + 1];
  __shared__ int before_s[kMaxKept + 1], total_s[kMaxKept + 1];
  __shared__ int64_t cstart_s[kMaxKept];
  __shared__ double cen_s[kMaxKept][2];
  __shared__ int flag;
  FUSED_TS(0);
  const int o = blockIdx.y, blk = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int K = a.n_kept[o], L = a.L, T = a.T;
  const int64_t N = a.N;
  const uint64_t seed = a.seed_dev ? *a.seed_dev : a.seed;
  const uint32_t key = a.ov_base + static_cast<uint32_t>(o);
  const int64_t i0 = static_cast<int64_t>(blk) * kFP;
  const double mx = a.minpos[2 * o], my = a.minpos[2 * o + 1];
  if (!ZIN && tid < L) cdf_s[tid] = a.latent_cdf[static_cast<int64_t>(o) * L + tid];
  if (tid < L) keep_s[tid] = a.keep_map[o * L + tid];
  const int gsz = L * T * 5;
  const bool staged = !PP && gsz <= static_cast<int>(sizeof(sm.s.gmm) / sizeof(float));
  if (staged)
    for (int e = tid; e < gsz; e += kFThreads) sm.s.gmm[e] = a.gmm[static_cast<int64_t>(o) * gsz + e];
  __syncthreads();

  // ---- counts: the OV's latent ids, per category, before this block and in total ------------
  if (tid < kFWaves * 2 * (kMaxKept + 1)) (&wc[0][0][0])[tid] = 0;
  __syncthreads();
  for (int64_t base = 0; base < N; base += kFThreads) {
    const int64_t i = base + tid;
    const bool v = i < N;
    int z = 0;
    if (v) {
      if (ZIN) {
        z = a.z_in[static_cast<int64_t>(o) * N + i];
        z = z < 0 ? 0 : (z >= L ? L - 1 : z);  // memory safety; the host validates
      } else {
        z = draw_latent(i, key, seed, cdf_s, L);
      }
      if (i >= i0 && i < i0 + kFP) {
        zs[i - i0] = z;
        if (a.out_z) a.out_z[static_cast<int64_t>(o) * N + i] = z;
      }
    }
    const int kk = keep_s[z];
    const int cat = kk >= 0 ? kk : K;
    for (int c = 0; c <= K; ++c) {  // wave counts by ballot, kept in this wave's LDS row
      const int nt = __popcll(__ballot(v && cat == c));
      const int nb = __popcll(__ballot(v && cat == c && i < i0));
      if (lane == 0) {
        wc[w][0][c] += nb;
        wc[w][1][c] += nt;
      }
    }
  }
  __syncthreads();
  if (tid <= K) {
    int b = 0, t = 0;
    for (int u = 0; u < kFWaves; ++u) {
      b += wc[u][0][tid];
      t += wc[u][1][tid];
    }
    before_s[tid] = b;
    total_s[tid] = t;
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

  FUSED_TS(1);
  // ---- actions (all waves), then the chain (wave 0) ------------------------------------------
  const int64_t ip = i0 + lane;
  const bool valid = ip < N;
  if (valid)
    for (int t = w; t < T; t += kFWaves)
      draw_action<PP, EPSIN>(t, ip, zs[lane], o, T, L, N, key, seed, a.gmm, sm.s.gmm, staged,
                             a.eps_in, sm.s.act[0][t][lane], sm.s.act[1][t][lane]);
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rrs = raw_rsrc(a.rstore + static_cast<int64_t>(o) * 2 * T * a.Npad);
  const __amdgpu_buffer_rsrc_t rri = raw_rsrc(a.rinfo + static_cast<int64_t>(o) * a.Npad * 4);
  const __amdgpu_buffer_rsrc_t rg =
      slab_rsrc(a.gpart + static_cast<int64_t>(o) * a.G * a.max_k * 2);
  const int npad = static_cast<int>(a.Npad);
  if (w == 0) {
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
      const double *st = a.init_state + 4 * o;
      x = static_cast<float>(st[0]);
      y = static_cast<float>(st[1]);
      float phi = static_cast<float>(st[2]), v = static_cast<float>(st[3]);
      float s0, c0;
      sincos_rn(phi, s0, c0);
      float *op = a.out + dst;
      for (int t = 0; t < T; ++t) {
        unicycle_step(x, y, phi, v, s0, c0, sm.s.act[0][t][lane], sm.s.act[1][t][lane], a.dt);
        if (native) {
          op[(2 * t) * a.ld_out] = x;
          op[(2 * t + 1) * a.ld_out] = y;
        } else {
          stf_sc1(rrs, 4 * ((2 * t) * npad + rs), x);
          stf_sc1(rrs, 4 * ((2 * t + 1) * npad + rs), y);
        }
      }
      if (!native) {
        const float4 info = {x, y, __builtin_bit_cast(float, z), 0.0f};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(b128_t, info), rri, 16 * rs, 0,
                                               16);
      }
    }
    // this block is centre group blk: its kept-mode sums of the final world positions
    const double xw = static_cast<double>(x) + mx, yw = static_cast<double>(y) + my;
    for (int k = 0; k < K; ++k) {
      const bool mine = valid && cat == k;
      const double sx = group_sum64(mine ? xw : 0.0), sy = group_sum64(mine ? yw : 0.0);
      if (lane == 0) st2_sc1(rg, 16 * (blk * a.max_k + k), sx, sy);
    }
  }
  FUSED_TS(2);
  if (!arrive_last(a.ctr + o, a.G, &flag)) return;
  FUSED_TS(3);

  // ---- the OV's last arriver: centres, then the rare particles --------------------------------
  const int R = total_s[K];
  const int rows = 2 * T;
  const int E = R * rows;
  // every load the rest needs is issued here: the centre partials, and the first kFPrefetch
  // copy elements of this thread (element e = row * R + r, e = tid + 512 j)
  const int ng = a.G * K;
  double2 gpv[kFGroups * kMaxKept / kFThreads];
#pragma unroll
  for (int q = 0; q < kFGroups * kMaxKept / kFThreads; ++q) {
    const int u = tid + q * kFThreads;  // u = g K + k
    if (u < ng) gpv[q] = ld2_sc1(rg, 16 * ((u / K) * a.max_k + u % K));
  }
  const int dr = R > 0 ? kFThreads % R : 0, drow = R > 0 ? kFThreads / R : 0;
  int row0 = R > 0 ? tid / R : rows, r0 = R > 0 ? tid % R : 0;
  float v[kFPrefetch];
  {
    int row = row0, r = r0;
#pragma unroll
    for (int j = 0; j < kFPrefetch; ++j) {
      v[j] = row < rows ? ldf_sc1(rrs, 4 * (row * npad + r)) : 0.0f;
      r += dr;
      row += drow;
      if (r >= R) {
        r -= R;
        ++row;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < kFGroups * kMaxKept / kFThreads; ++q) {
    const int u = tid + q * kFThreads;
    if (u < ng) sm.gp[u] = gpv[q];
  }
  __syncthreads();
  // centres, canonical order (bucket.hpp): superblocks (at most 2 here), then left to right
  if (tid < K) {
    const int k = tid;
    double2 tot = {0.0, 0.0};
    for (int j = 0; j * kCentreSuper < a.G; ++j) {
      const double2 s = superblock_sum(j, a.G, [&](int g) { return sm.gp[g * K + k]; });
      tot.x += s.x;
      tot.y += s.y;
    }
    const double nk = static_cast<double>(total_s[k]);
    cen_s[k][0] = tot.x / nk;
    cen_s[k][1] = tot.y / nk;
  }
  __syncthreads();  // sm.gp is dead from here
  FUSED_TS(4);
  // keys of the rare list: owner (L + 1) + 1 + z
  const int nbins = K * (L + 1);
  for (int r = tid; r < R; r += kFThreads) {
    const float4 info = __builtin_bit_cast(
        float4, __builtin_amdgcn_raw_buffer_load_b128(rri, 16 * r, 0, 16));
    const int z = __builtin_bit_cast(int, info.z);
    sm.r.rk[r] = key_staged(z, static_cast<double>(info.x) + mx,
                            static_cast<double>(info.y) + my, keep_s, cen_s, K, L);
  }
  for (int b = tid; b < nbins; b += kFThreads) sm.r.run[b] = 0;
  // stable ranks in sample order: rounds of 512 rare particles, waves in order
  const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (int base = 0; base < R; base += kFThreads) {
    for (int b = tid; b < kFWaves * nbins; b += kFThreads) sm.r.wcnt[b / nbins][b % nbins] = 0;
    __syncthreads();
    const int r = base + tid;
    const bool ok = r < R;
    const int kr = ok ? sm.r.rk[r] : -1;
    int rank = 0;
    unsigned long long todo = __ballot(ok);
    while (todo) {
      const int leader = __ffsll(static_cast<long long>(todo)) - 1;
      const int kl = __shfl(kr, leader, 64);
      const unsigned long long m = __ballot(ok && kr == kl);
      if (ok && kr == kl) rank = __popcll(m & below);
      if (lane == leader) sm.r.wcnt[w][kl] = __popcll(m);
      todo &= ~m;
    }
    __syncthreads();
    if (ok) {
      int before = sm.r.run[kr];
      for (int u = 0; u < w; ++u) before += sm.r.wcnt[u][kr];
      sm.r.rk[r] = (kr << 16) | (before + rank);
    }
    __syncthreads();
    for (int b = tid; b < nbins; b += kFThreads) {
      int s = sm.r.run[b];
      for (int u = 0; u < kFWaves; ++u) s += sm.r.wcnt[u][b];
      sm.r.run[b] = s;
    }
    __syncthreads();  // before the next round clears wcnt
  }
  FUSED_TS(5);
  // bins of kept mode k start after its natives; the cells' outputs
  if (tid < K) {
    const int k = tid;
    const int64_t reg = a.region[o];
    int s = static_cast<int>(cstart_s[k] - reg) + total_s[k];
    for (int z = 0; z < L; ++z) {
      const int b = k * (L + 1) + 1 + z;
      sm.r.bstart[b] = s;
      s += sm.r.run[b];
    }
    const int64_t n = s - (cstart_s[k] - reg);
    const int cell = a.cell_base[o] + k;
    a.cell_off[cell] = cstart_s[k];
    a.cell_cnt[cell] = n;
    a.cell_pmf[cell] = static_cast<double>(n) / static_cast<double>(N);
    a.init_center[2 * cell] = cen_s[k][0];
    a.init_center[2 * cell + 1] = cen_s[k][1];
  }
  __syncthreads();
  // the copy: element (row, r) -> row `row` of the owner's cell, slot bstart + rank
  float *out = a.out + a.region[o];
  auto dst_of = [&](int r) {
    const int p = sm.r.rk[r];
    return static_cast<int64_t>(sm.r.bstart[p >> 16] + (p & 0xffff));
  };
  {
    int row = row0, r = r0;
#pragma unroll
    for (int j = 0; j < kFPrefetch; ++j) {
      if (row < rows) out[row * a.ld_out + dst_of(r)] = v[j];
      r += dr;
      row += drow;
      if (r >= R) {
        r -= R;
        ++row;
      }
    }
  }
  for (int e = tid + kFPrefetch * kFThreads; e < E; e += kFThreads) {  // beyond the prefetch
    const int row = e / R, r = e % R;
    out[row * a.ld_out + dst_of(r)] = ldf_sc1(rrs, 4 * (row * npad + r));
  }
  FUSED_TS(6);
}

struct FusedWs {
  size_t ctr, gpart, rinfo, rstore, total;
};

inline size_t a256(size_t b) { return (b + 255) / 256 * 256; }

inline FusedWs fused_ws(int64_t n_ov, int64_t N, int64_t T, int64_t max_k) {
  const int64_t G = (N + kFP - 1) / kFP, Npad = (N + 3) & ~int64_t(3);
  FusedWs w;
  size_t o = 0;
  w.ctr = o;  // arrival counters first: the zero-filled head of the workspace
  o += a256(sizeof(int32_t) * n_ov);
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
// slots: 0 start, 1 counted, 2 sampled + published, 3 last arriver, 4 centres, 5 ranked,
// 6 copied (tools/probe_step.py)
extern "C" int ccmpc_probe_fused_timestamps(void *host, int reset) {
  const size_t bytes = sizeof(g_fused_ts);
  if (reset) {
    static unsigned long long zeros[kStepProbeWG * kStepProbeSlots];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_fused_ts), zeros, bytes) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fused_ts), bytes) == hipSuccess ? 0 : -1;
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
  a.ctr = reinterpret_cast<int32_t *>(ws + L.ctr);
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
  const dim3 grid(static_cast<unsigned>(a.G), static_cast<unsigned>(n_ov));
  hipStream_t s = as_stream(stream);
  const int mode = (pp ? 4 : 0) | (z_in ? 2 : 0) | (eps_in ? 1 : 0);
#define CCMPC_FUSED(PP, ZIN, EPSIN) \
  hipLaunchKernelGGL((sample_bucket_kernel<PP, ZIN, EPSIN>), grid, dim3(kFThreads), 0, s, a)
  switch (mode) {
    case 0: CCMPC_FUSED(false, false, false); break;
    case 1: CCMPC_FUSED(false, false, true); break;
    case 2: CCMPC_FUSED(false, true, false); break;
    case 3: CCMPC_FUSED(false, true, true); break;
    case 6: CCMPC_FUSED(true, true, false); break;
    default: CCMPC_FUSED(true, true, true); break;
  }
#undef CCMPC_FUSED
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}
