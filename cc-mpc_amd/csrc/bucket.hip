// Particle bucketing by latent mode: v8ideal/__init__.py:469-505 (make_ovehicles: per-particle
// append into veh_latent_predictions[z]) + ovehicle.py:24-117 (OVehicle.from_trajectron).
//
// Per OV, on the sampler's sample-order store:
//   kept modes   = latents with p(z|x) > filter (host decides: latent_probs are host data)
//   centre_k     = mean final (t = T-1) world position of kept mode k's own particles
//   rare z       -> owner = argmin_k ||final position - centre_k|| (first minimum on ties,
//                   scipy.spatial.distance_matrix + np.argmin)
//   bucket order = kept mode k's own particles in sample order, then for each rare latent value
//                  in ascending order its particles owned by k in sample order -- exactly the
//                  reference's np.concatenate order
//   pmf_k        = N_k / N
// This is a stable counting sort on key = owner * (L + 1) + group, group = 0 for the native
// mode and 1 + z for a rare latent.  Three short kernels:
//   B1 stats   per block: latent counts (LDS int atomics, exact) and, per wave, the kept-mode
//              sums of its 64 final positions (bucket.hpp's centre groups), published
//              write-through -> centres
//   B2 keys    per block: key histogram (LDS int atomics, exact), published write-through ->
//              per chunk of 16 blocks the bin starts, 4-aligned cell offsets
//   B3 scatter per block: stable rank inside the block (wave ballots, waves in order) -> copy
//              the particle's 2T coordinates to its bucket slot
// B1 and B2 meet in two hand-off levels: a chunk of kChunkRows = 16 blocks is exactly one centre
// superblock (64 groups of 64 particles), so the chunk's last arriving block sums its superblock
// in the canonical order (bucket.hpp) and its latent counts / bin totals, every load in flight at
// once; the OV's last arriving chunk then combines the chunk results (one more round of loads).
// A single OV-level arriver walking every block's partials was ~8 dependent round trips of
// fresh data (10 us per kernel at N = 100 000, profiles/r03/s13_probe_step_c1_100k.log).
// The last-arriver hand-off is the one of the moment reduction (gram.hpp: sc1 stores, drain,
// agent-scope ticket, sc1 loads); its counters live at the head of the workspace, which must be
// zero-filled once (every call leaves them zero).
// Everything is integer-exact except the centre sums, whose fixed order makes them
// deterministic; the bucketed store is bit-identical across runs, and to the fused sampler +
// bucketing kernel's (sample_bucket.hip) up to where each cell starts.
#include "bucket.hpp"

namespace ccmpc {

constexpr int kBucketBlock = 256;
constexpr int kPerThread = 1;  // one round per block: many short blocks (C2 shape: 80, not 20)
constexpr int kSpan = kBucketBlock * kPerThread;  // particles per block, in sample order
constexpr int kChunkRows = 16;  // blocks per chunk of the bin-offset scan

#if defined(CCMPC_PROBE) && (CCMPC_PROBE & 4)
__device__ unsigned long long g_bkt_ts[3][kStepProbeWG * kStepProbeSlots];
#define BKT_TS(kern, k) CCMPC_STEP_TS(g_bkt_ts[kern], k)
#else
#define BKT_TS(kern, k) CCMPC_STEP_TS(nullptr, k)
#endif

struct BucketArgs {
  const int32_t *z;        // [n_ov][N]
  const float *pos;        // sample-order store, OV o at o * S_in
  int64_t ld_in, S_in;
  int T, L, n_ov, max_k;
  int64_t N;
  const int32_t *keep_map;  // [n_ov][L] kept index or -1
  const int32_t *n_kept;    // [n_ov]
  const int32_t *cell_base; // [n_ov] first global cell of the OV
  const int64_t *region;    // [n_ov] first particle slot of the OV's region in the output
  const double *minpos;     // [n_ov][2]
  int nb;                   // blocks per OV
  // workspace
  int32_t *ctr;             // [2][n_ov] OV arrival counters, then [2][n_ov][nch] chunk counters
                            // (zero between calls)
  int nch;                  // chunks of kChunkRows blocks per OV
  int32_t *bcnt;            // [n_ov][nb][L]: each block's latent counts
  int32_t *ccnt;            // [n_ov][nch][L]: each chunk's latent counts
  double *gpart;            // [n_ov][G][max_k][2]: per 64-particle group kept-mode sums
  int G;                    // groups per OV = ceil(N / 64)
  double *csup;             // [n_ov][nch][max_k][2]: each chunk's superblock sums (bucket.hpp)
  double *centre;           // [n_ov][max_k][2]
  int32_t *hist;            // [n_ov][nb][nbins]
  int32_t *ctot;            // [n_ov][nch][nbins]: each chunk's bin totals
  int64_t *chunk_off;       // [n_ov][nch][nbins]: each chunk's bin starts
  // outputs
  float *out;
  int64_t ld_out;
  int64_t *cell_off, *cell_cnt;
  double *cell_pmf, *init_center;
};

__device__ __forceinline__ void final_world(const BucketArgs &a, int o, int64_t i, double &x,
                                            double &y) {
  const float *p = a.pos + o * a.S_in + i;
  x = static_cast<double>(p[(2 * (a.T - 1)) * a.ld_in]) + a.minpos[2 * o];
  y = static_cast<double>(p[(2 * (a.T - 1) + 1) * a.ld_in]) + a.minpos[2 * o + 1];
}

static_assert(kChunkRows * (kBucketBlock / kCentreGroup) == kCentreSuper,
              "a chunk of blocks is one centre superblock");

// The chunk's and OV's arrival counters (stats: which = 0, hist: which = 1).
__device__ __forceinline__ int32_t *chunk_ctr(const BucketArgs &a, int which, int o, int ch) {
  return a.ctr + 2 * a.n_ov + (static_cast<int64_t>(which) * a.n_ov + o) * a.nch + ch;
}
__device__ __forceinline__ int32_t *ov_ctr(const BucketArgs &a, int which, int o) {
  return a.ctr + which * a.n_ov + o;
}
// The OV level of the hand-off: the OV's last arriving chunk goes on.  An OV of one chunk has
// no second level (its chunk's last arriver is the OV's), but still drains its stores, which it
// reads back below.
__device__ __forceinline__ bool ov_last(const BucketArgs &a, int which, int o, int *flag) {
  if (a.nch > 1) return arrive_last(ov_ctr(a, which, o), a.nch, flag);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  return true;
}

__global__ __launch_bounds__(kBucketBlock) void bucket_stats(BucketArgs a) {
  BKT_TS(0, 0);
  __shared__ int cnt[64];
  __shared__ int flag;
  __shared__ int keep_s[64];
  __shared__ int zv_s[kMaxKept];
  __shared__ int nk_s[kMaxKept];
  __shared__ double2 sup_s[kMaxKept][kCentreSuper];  // a superblock's partials / chunk sums
  const int o = blockIdx.y, blk = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int K = a.n_kept[o];
  const int64_t i0 = static_cast<int64_t>(blk) * kSpan;
  static_assert(kPerThread == 1 && kBucketBlock % kCentreGroup == 0, "one group per wave");
  const int64_t i = i0 + threadIdx.x;
  int zv = -1;
  double xf = 0.0, yf = 0.0;
  if (i < a.N) {
    zv = a.z[o * a.N + i];
    final_world(a, o, i, xf, yf);
  }
  for (int l = threadIdx.x; l < a.L; l += blockDim.x) {
    cnt[l] = 0;
    keep_s[l] = a.keep_map[o * a.L + l];
  }
  if (threadIdx.x < kMaxKept) nk_s[threadIdx.x] = 0;
  __syncthreads();
  BKT_TS(0, 1);
  if (zv >= 0) atomicAdd(&cnt[zv], 1);
  // this wave's 64 particles are centre group g (bucket.hpp): its kept-mode sums
  const int g = blk * (kBucketBlock / kCentreGroup) + (threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t rg =
      slab_rsrc(a.gpart + static_cast<int64_t>(o) * a.G * a.max_k * 2);
  for (int k = 0; k < K; ++k) {
    const bool mine = zv >= 0 && keep_s[zv] == k;
    const double sx = group_sum64(mine ? xf : 0.0), sy = group_sum64(mine ? yf : 0.0);
    if (lane == 0 && g < a.G) st2_sc1(rg, 16 * (g * a.max_k + k), sx, sy);
  }
  __syncthreads();
  // latent counts, published write-through
  const __amdgpu_buffer_rsrc_t rb = raw_rsrc(a.bcnt + static_cast<int64_t>(o) * a.nb * a.L);
  for (int l = threadIdx.x; l < a.L; l += blockDim.x) st1_sc1(rb, 4 * (blk * a.L + l), cnt[l]);
  BKT_TS(0, 2);
  // ---- chunk level: the chunk's last arriving block -----------------------------------------
  const int ch = blk / kChunkRows, r0 = ch * kChunkRows, nr = min(kChunkRows, a.nb - r0);
  if (!arrive_last(chunk_ctr(a, 0, o, ch), nr, &flag)) return;
  BKT_TS(0, 3);
  // (1) the superblock's K x 64 group partials into LDS and (2) the chunk's latent counts, every
  // load in flight together
  const int g0 = ch * kCentreSuper, ng = min(kCentreSuper, a.G - g0);
  constexpr int kPartRounds = kMaxKept * kCentreSuper / kBucketBlock;
  double2 pv[kPartRounds];
#pragma unroll
  for (int r = 0; r < kPartRounds; ++r) {
    const int t = threadIdx.x + r * kBucketBlock, k = t / kCentreSuper, q = t % kCentreSuper;
    const int kc = k < K ? k : (K > 0 ? K - 1 : 0), qc = q < ng ? q : ng - 1;  // valid addresses
    pv[r] = ld2_sc1(rg, 16 * ((g0 + qc) * a.max_k + kc));
  }
  int32_t cv[kChunkRows];
  const bool counter = threadIdx.x < a.L;
#pragma unroll
  for (int j = 0; j < kChunkRows; ++j)
    cv[j] = counter ? ld1_sc1(rb, 4 * ((r0 + (j < nr ? j : nr - 1)) * a.L + threadIdx.x)) : 0;
#pragma unroll
  for (int r = 0; r < kPartRounds; ++r) {
    const int t = threadIdx.x + r * kBucketBlock, k = t / kCentreSuper, q = t % kCentreSuper;
    if (k < K) sup_s[k][q] = q < ng ? pv[r] : double2{-0.0, -0.0};  // lds_row_sum's padding
  }
  int32_t csum = 0;
#pragma unroll
  for (int j = 0; j < kChunkRows; ++j) csum += j < nr ? cv[j] : 0;
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = slab_rsrc(a.csup + static_cast<int64_t>(o) * a.nch * a.max_k * 2);
  const __amdgpu_buffer_rsrc_t rc = raw_rsrc(a.ccnt + static_cast<int64_t>(o) * a.nch * a.L);
  if (threadIdx.x < K) {  // S_ch = 0.0 + P_{64 ch} + P_{64 ch + 1} + ... (bucket.hpp)
    double2 acc = {0.0, 0.0};
    lds_row_sum(acc, sup_s[threadIdx.x], ng);
    st2_sc1(rs, 16 * (ch * a.max_k + threadIdx.x), acc.x, acc.y);
  }
  if (counter) st1_sc1(rc, 4 * (ch * a.L + threadIdx.x), csum);
  BKT_TS(0, 4);
  // ---- OV level: the OV's last arriving chunk ------------------------------------------------
  if (!ov_last(a, 0, o, &flag)) return;
  BKT_TS(0, 5);
  for (int l = threadIdx.x; l < a.L; l += blockDim.x) {
    const int k = keep_s[l];
    if (k >= 0) zv_s[k] = l;
  }
  __syncthreads();
  // n_k: kept mode k's own particles, summed over the chunks (integer-exact in any order); the
  // chunk sums S_ch in windows of kCentreSuper chunks, added left to right (bucket.hpp)
  double2 tot = {0.0, 0.0};  // thread k's running sum of mode k
  for (int c0 = 0; c0 < a.nch; c0 += kCentreSuper) {
    const int nc = min(kCentreSuper, a.nch - c0);
    double2 sv[kPartRounds];
    int32_t nv[kPartRounds];
#pragma unroll
    for (int r = 0; r < kPartRounds; ++r) {
      const int t = threadIdx.x + r * kBucketBlock, k = t / kCentreSuper, q = t % kCentreSuper;
      const int kc = k < K ? k : (K > 0 ? K - 1 : 0), qc = q < nc ? q : nc - 1;
      sv[r] = ld2_sc1(rs, 16 * ((c0 + qc) * a.max_k + kc));
      nv[r] = K > 0 ? ld1_sc1(rc, 4 * ((c0 + qc) * a.L + zv_s[kc])) : 0;
    }
#pragma unroll
    for (int r = 0; r < kPartRounds; ++r) {
      const int t = threadIdx.x + r * kBucketBlock, k = t / kCentreSuper, q = t % kCentreSuper;
      if (k < K) sup_s[k][q] = q < nc ? sv[r] : double2{-0.0, -0.0};
      if (k < K && q < nc) atomicAdd(&nk_s[k], nv[r]);
    }
    __syncthreads();
    if (threadIdx.x < K) lds_row_sum(tot, sup_s[threadIdx.x], nc);
    __syncthreads();
  }
  if (threadIdx.x < K) {
    const int k = threadIdx.x;
    const double n = static_cast<double>(nk_s[k]);
    const double cx = tot.x / n, cy = tot.y / n;
    a.centre[(o * a.max_k + k) * 2] = cx;
    a.centre[(o * a.max_k + k) * 2 + 1] = cy;
    const int cell = a.cell_base[o] + k;
    a.init_center[2 * cell] = cx;
    a.init_center[2 * cell + 1] = cy;
  }
  BKT_TS(0, 6);
}

// Chunk bin totals the OV's last arriver keeps in LDS for the chunk starts (beyond: re-read)
constexpr int kHistKeep = 4096;  // 16 KB: N <= ~200 000 at 78 bins

__global__ __launch_bounds__(kBucketBlock) void bucket_hist(BucketArgs a) {
  BKT_TS(1, 0);
  __shared__ int h[kMaxBins];
  __shared__ int64_t start[kMaxBins];
  __shared__ int flag;
  __shared__ int keep_s[64];
  __shared__ double cen_s[kMaxKept][2];
  __shared__ int32_t pre_s[kHistKeep];  // [chunk][bin]: the bin's count in the chunks before
  const int o = blockIdx.y, blk = blockIdx.x;
  const int K = a.n_kept[o];
  const int G = a.L + 1;
  const int nbins = K * G;
  const int64_t i0 = static_cast<int64_t>(blk) * kSpan;
  int zs[kPerThread];
  double xs[kPerThread], ys[kPerThread];
#pragma unroll
  for (int r = 0; r < kPerThread; ++r) {  // every load of the block issued together
    const int64_t i = i0 + r * kBucketBlock + threadIdx.x;
    zs[r] = -1;
    xs[r] = ys[r] = 0.0;
    if (i < a.N) {
      zs[r] = a.z[o * a.N + i];
      final_world(a, o, i, xs[r], ys[r]);
    }
  }
  for (int l = threadIdx.x; l < a.L; l += blockDim.x) keep_s[l] = a.keep_map[o * a.L + l];
  for (int j = threadIdx.x; j < 2 * K; j += blockDim.x)
    cen_s[j >> 1][j & 1] = a.centre[(o * a.max_k + (j >> 1)) * 2 + (j & 1)];
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) h[b] = 0;
  __syncthreads();
  BKT_TS(1, 1);
#pragma unroll
  for (int r = 0; r < kPerThread; ++r)
    if (zs[r] >= 0) atomicAdd(&h[key_staged(zs[r], xs[r], ys[r], keep_s, cen_s, K, a.L)], 1);
  __syncthreads();
  const int64_t stride = static_cast<int64_t>(a.max_k) * G;
  const __amdgpu_buffer_rsrc_t rh = raw_rsrc(a.hist + static_cast<int64_t>(o) * a.nb * stride);
  for (int b = threadIdx.x; b < nbins; b += blockDim.x)
    st1_sc1(rh, 4 * static_cast<int>(blk * stride + b), h[b]);
  BKT_TS(1, 2);
  // ---- chunk level: the chunk's bin totals (every row's load in flight together) ------------
  const int ch = blk / kChunkRows, r0 = ch * kChunkRows, nr = min(kChunkRows, a.nb - r0);
  if (!arrive_last(chunk_ctr(a, 1, o, ch), nr, &flag)) return;
  BKT_TS(1, 3);
  const __amdgpu_buffer_rsrc_t rt = raw_rsrc(a.ctot + static_cast<int64_t>(o) * a.nch * stride);
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) {
    int32_t v[kChunkRows];
#pragma unroll
    for (int j = 0; j < kChunkRows; ++j)
      v[j] = ld1_sc1(rh, 4 * static_cast<int>((r0 + (j < nr ? j : nr - 1)) * stride + b));
    int32_t sum = 0;
#pragma unroll
    for (int j = 0; j < kChunkRows; ++j) sum += j < nr ? v[j] : 0;
    st1_sc1(rt, 4 * static_cast<int>(ch * stride + b), sum);
  }
  BKT_TS(1, 4);
  // ---- OV level: bin totals, cell offsets, every chunk's start in every bin -----------------
  if (!ov_last(a, 1, o, &flag)) return;
  BKT_TS(1, 5);
  // pass 1 (thread per bin): running counts over the chunks, 32 loads in flight
  const bool keep = static_cast<int64_t>(a.nch) * nbins <= kHistKeep;
  constexpr int kBatch = 32;
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) {
    int64_t run = 0;
    for (int c0 = 0; c0 < a.nch; c0 += kBatch) {
      int32_t v[kBatch];
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const int c = c0 + j < a.nch ? c0 + j : a.nch - 1;
        v[j] = ld1_sc1(rt, 4 * static_cast<int>(c * stride + b));
      }
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        if (c0 + j < a.nch) {
          if (keep) pre_s[(c0 + j) * nbins + b] = static_cast<int32_t>(run);
          run += v[j];
        }
      }
    }
    start[b] = run;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t cur = a.region[o];
    for (int k = 0; k < K; ++k) {
      int64_t n = 0;
      for (int gi = 0; gi < G; ++gi) {
        const int64_t c = start[k * G + gi];
        start[k * G + gi] = cur + n;
        n += c;
      }
      const int cell = a.cell_base[o] + k;
      a.cell_off[cell] = cur;
      a.cell_cnt[cell] = n;
      a.cell_pmf[cell] = static_cast<double>(n) / static_cast<double>(a.N);
      cur += (n + 3) & ~int64_t(3);
    }
  }
  __syncthreads();
  // pass 2: each chunk's start in every bin (plain stores: read by the next launch)
  int64_t *coff = a.chunk_off + static_cast<int64_t>(o) * a.nch * stride;
  if (keep) {
    for (int t = threadIdx.x; t < a.nch * nbins; t += blockDim.x) {
      const int c = t / nbins, b = t - c * nbins;
      coff[c * stride + b] = start[b] + pre_s[t];
    }
  } else {
    for (int b = threadIdx.x; b < nbins; b += blockDim.x) {
      int64_t run = start[b];
      for (int c0 = 0; c0 < a.nch; c0 += kBatch) {
        int32_t v[kBatch];
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
          const int c = c0 + j < a.nch ? c0 + j : a.nch - 1;
          v[j] = ld1_sc1(rt, 4 * static_cast<int>(c * stride + b));
        }
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
          if (c0 + j < a.nch) {
            coff[(c0 + j) * stride + b] = run;
            run += v[j];
          }
        }
      }
    }
  }
  BKT_TS(1, 6);
}

__global__ __launch_bounds__(kBucketBlock) void bucket_scatter(BucketArgs a) {
  BKT_TS(2, 0);
  __shared__ int run[kMaxBins];        // particles of each bin in earlier rounds of this block
  __shared__ int wcnt[4][kMaxBins];    // per wave counts of the current round
  __shared__ int keep_s[64];
  __shared__ double cen_s[kMaxKept][2];
  __shared__ int64_t boff_s[kMaxBins];
  const int o = blockIdx.y, blk = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int K = a.n_kept[o];
  const int nbins = K * (a.L + 1);
  const int64_t stride = static_cast<int64_t>(a.max_k) * (a.L + 1);
  // this block's start in every bin: its chunk's start (bucket_hist) + the histograms of the
  // blocks before it in the chunk
  const int ch = blk / kChunkRows;
  const int64_t *coff = a.chunk_off + (static_cast<int64_t>(o) * a.nch + ch) * stride;
  const int32_t *hist0 = a.hist + static_cast<int64_t>(o) * a.nb * stride;
  const int64_t i0 = static_cast<int64_t>(blk) * kSpan;
  // kPerThread == 1: this thread's particle, its key inputs and its 2T coordinates, every load
  // issued together with the block's tables
  static_assert(kPerThread == 1, "one particle per thread");
  const int64_t i = i0 + threadIdx.x;  // sample order = (wave, lane)
  const bool valid = i < a.N;
  int zv = 0;
  double xf = 0.0, yf = 0.0;
  if (valid) {
    zv = a.z[o * a.N + i];
    final_world(a, o, i, xf, yf);
  }
  const int rows = 2 * a.T;
  const float *src = a.pos + o * a.S_in + (valid ? i : 0);
  float v[80];
#pragma unroll
  for (int rr = 0; rr < 80; ++rr)
    if (rr < rows) v[rr] = src[static_cast<int64_t>(rr) * a.ld_in];
  for (int l = threadIdx.x; l < a.L; l += blockDim.x) keep_s[l] = a.keep_map[o * a.L + l];
  for (int j = threadIdx.x; j < 2 * K; j += blockDim.x)
    cen_s[j >> 1][j & 1] = a.centre[(o * a.max_k + (j >> 1)) * 2 + (j & 1)];
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) {
    run[b] = 0;
    int32_t v[kChunkRows - 1];
    const int r0 = ch * kChunkRows, nr = blk - r0;  // rows of this chunk before the block
#pragma unroll
    for (int j = 0; j < kChunkRows - 1; ++j)
      v[j] = hist0[static_cast<int64_t>(r0 + (j < nr ? j : 0)) * stride + b];
    int64_t s = coff[b];
#pragma unroll
    for (int j = 0; j < kChunkRows - 1; ++j) s += j < nr ? v[j] : 0;
    boff_s[b] = s;
  }
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int r = 0; r < kPerThread; ++r) {
    for (int b = threadIdx.x; b < 4 * nbins; b += blockDim.x) wcnt[b / nbins][b % nbins] = 0;
    __syncthreads();
    BKT_TS(2, 1);
    const int key = valid ? key_staged(zv, xf, yf, keep_s, cen_s, K, a.L) : -1;
    // rank among equal keys of this wave (lanes in order)
    int rank = 0;
    unsigned long long todo = __ballot(valid);
    while (todo) {
      const int leader = __ffsll(static_cast<long long>(todo)) - 1;
      const int k = __shfl(key, leader, 64);
      const unsigned long long m = __ballot(valid && key == k);
      if (valid && key == k) rank = __popcll(m & below);
      if (lane == leader) wcnt[w][k] = __popcll(m);
      todo &= ~m;
    }
    __syncthreads();
    if (valid) {
      int before = run[key];
      for (int u = 0; u < w; ++u) before += wcnt[u][key];
      const int64_t dst = boff_s[key] + before + rank;
#pragma unroll
      for (int rr = 0; rr < 80; ++rr)
        if (rr < rows) a.out[static_cast<int64_t>(rr) * a.ld_out + dst] = v[rr];
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nbins; b += blockDim.x)
      run[b] += wcnt[0][b] + wcnt[1][b] + wcnt[2][b] + wcnt[3][b];
    __syncthreads();
  }
  BKT_TS(2, 2);
}

inline size_t align256(size_t b) { return (b + 255) / 256 * 256; }

struct WsLayout {
  size_t ctr, bcnt, ccnt, gpart, csup, centre, hist, ctot, chunk_off, total;
  int G, nch;
};

inline WsLayout bucket_ws(int64_t n_ov, int64_t N, int64_t L, int64_t max_k) {
  const int64_t nb = (N + kSpan - 1) / kSpan, nch = (nb + kChunkRows - 1) / kChunkRows;
  WsLayout w;
  w.G = static_cast<int>((N + kCentreGroup - 1) / kCentreGroup);
  w.nch = static_cast<int>(nch);
  size_t o = 0;
  w.ctr = o;  // arrival counters first: the zero-filled head of the workspace
  o += align256(sizeof(int32_t) * 2 * n_ov * (1 + nch));
  w.bcnt = o;
  o += align256(sizeof(int32_t) * n_ov * nb * L);
  w.ccnt = o;
  o += align256(sizeof(int32_t) * n_ov * nch * L);
  w.gpart = o;
  o += align256(sizeof(double) * n_ov * w.G * max_k * 2);
  w.csup = o;
  o += align256(sizeof(double) * n_ov * nch * max_k * 2);
  w.centre = o;
  o += align256(sizeof(double) * n_ov * max_k * 2);
  w.hist = o;
  o += align256(sizeof(int32_t) * n_ov * nb * max_k * (L + 1));
  w.ctot = o;
  o += align256(sizeof(int32_t) * n_ov * nch * max_k * (L + 1));
  w.chunk_off = o;
  o += align256(sizeof(int64_t) * n_ov * nch * max_k * (L + 1));
  w.total = o;
  return w;
}

}  // namespace ccmpc

using namespace ccmpc;

#if defined(CCMPC_PROBE) && (CCMPC_PROBE & 4)
// which: 0 stats (slots 0 start, 1 loaded, 2 published, 3 chunk's last arriver, 4 chunk
// published, 5 OV's last arriver, 6 done), 1 hist (same), 2 scatter (0 start, 1 loaded, 2 done)
// (tools/probe_step.py)
extern "C" int ccmpc_probe_bucket_timestamps(void *host, int which, int reset) {
  if (which < 0 || which > 2) return -1;
  const size_t bytes = sizeof(g_bkt_ts[0]);
  if (reset) {
    static unsigned long long zeros[kStepProbeWG * kStepProbeSlots];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_bkt_ts), zeros, bytes, which * bytes) == hipSuccess
               ? 0 : -1;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bkt_ts), bytes, which * bytes) == hipSuccess
             ? 0 : -1;
}
#endif

extern "C" size_t ccmpc_bucket_workspace_bytes(int64_t n_ov, int64_t N, int64_t n_latent,
                                               int64_t max_k) {
  if (n_ov < 0 || N < 1 || n_latent < 1 || n_latent > 64 || max_k < 1 || max_k > kMaxKept)
    return 0;
  return bucket_ws(n_ov, N, n_latent, max_k).total;
}

extern "C" int ccmpc_bucket(const int32_t *z, const float *pos_in, int64_t ld_in, int64_t T,
                            int64_t n_ov, int64_t N, int64_t n_latent, const int32_t *keep_map,
                            const int32_t *n_kept, const int32_t *cell_base, int64_t max_k,
                            const double *minpos, const int64_t *region, void *workspace,
                            size_t workspace_bytes, float *pos_out, int64_t ld_out,
                            int64_t *cell_off, int64_t *cell_cnt, double *cell_pmf,
                            double *init_center, ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T >= 1 && T <= 40, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_latent >= 1 && n_latent <= 64, "n_latent must be in [1, 64]");
  CCMPC_REQUIRE(max_k >= 1 && max_k <= kMaxKept && max_k * (n_latent + 1) <= kMaxBins,
                "max_k out of range");
  CCMPC_REQUIRE(n_ov >= 0 && n_ov < 65536 && N >= 1 && N < (int64_t(1) << 31), "bad sizes");
  // the per-OV histogram / chunk-offset tables are addressed with 32-bit buffer offsets
  CCMPC_REQUIRE(8 * ((N + kSpan - 1) / kSpan) * max_k * (n_latent + 1) < (int64_t(1) << 31),
                "N x kept modes x latents too large for one bucketing call");
  if (n_ov == 0) return CCMPC_OK;
  CCMPC_REQUIRE(z && pos_in && keep_map && n_kept && cell_base && minpos && region && pos_out &&
                    cell_off && cell_cnt && cell_pmf && init_center,
                "null pointer");
  const WsLayout L = bucket_ws(n_ov, N, n_latent, max_k);
  if (!workspace || workspace_bytes < L.total) {
    set_error("ccmpc_bucket: workspace too small");
    return CCMPC_ERR_WORKSPACE;
  }
  char *ws = static_cast<char *>(workspace);
  BucketArgs a;
  a.z = z;
  a.pos = pos_in;
  a.ld_in = ld_in;
  a.S_in = (N + 3) & ~int64_t(3);
  a.T = static_cast<int>(T);
  a.L = static_cast<int>(n_latent);
  a.n_ov = static_cast<int>(n_ov);
  a.max_k = static_cast<int>(max_k);
  a.N = N;
  a.keep_map = keep_map;
  a.n_kept = n_kept;
  a.cell_base = cell_base;
  a.region = region;
  a.minpos = minpos;
  a.nb = static_cast<int>((N + kSpan - 1) / kSpan);
  a.ctr = reinterpret_cast<int32_t *>(ws + L.ctr);
  a.nch = L.nch;
  a.bcnt = reinterpret_cast<int32_t *>(ws + L.bcnt);
  a.ccnt = reinterpret_cast<int32_t *>(ws + L.ccnt);
  a.gpart = reinterpret_cast<double *>(ws + L.gpart);
  a.G = L.G;
  a.csup = reinterpret_cast<double *>(ws + L.csup);
  a.centre = reinterpret_cast<double *>(ws + L.centre);
  a.hist = reinterpret_cast<int32_t *>(ws + L.hist);
  a.ctot = reinterpret_cast<int32_t *>(ws + L.ctot);
  a.chunk_off = reinterpret_cast<int64_t *>(ws + L.chunk_off);
  a.out = pos_out;
  a.ld_out = ld_out;
  a.cell_off = cell_off;
  a.cell_cnt = cell_cnt;
  a.cell_pmf = cell_pmf;
  a.init_center = init_center;
  hipStream_t s = as_stream(stream);
  const dim3 grid(static_cast<unsigned>(a.nb), static_cast<unsigned>(n_ov));
  hipLaunchKernelGGL(bucket_stats, grid, dim3(kBucketBlock), 0, s, a);
  hipLaunchKernelGGL(bucket_hist, grid, dim3(kBucketBlock), 0, s, a);
  hipLaunchKernelGGL(bucket_scatter, grid, dim3(kBucketBlock), 0, s, a);
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}

// ---- the reference's own prediction boundary ---------------------------------------------
// generate_vehicle_latents (prediction.py:93-105) hands make_ovehicles (v8ideal/__init__.py:
// 469-505) predictions[node][N][T][2] float32 (scene-relative; particle-major, as numpy's
// swapaxes(predictions, 0, 1) leaves them) and z[node][N] (int64 argmax of the one-hot sample).
// load_predictions_kernel gathers the OV rows (rows[o]: the non-ego nodes) into the plane-major
// sample-order store ccmpc_bucket reads, pos[(2t + c) * ld + o * ov_stride + i], and the latent
// ids into int32.  A workgroup moves kLoadChunk particles: the chunk's 2T * kLoadChunk floats
// are one contiguous run of the source, read coalesced into LDS (padded rows: 2T + 1 floats),
// then written plane by plane, kLoadChunk consecutive floats per plane.
constexpr int kLoadChunk = 128;

__global__ __launch_bounds__(256) void load_predictions_kernel(
    const float *__restrict__ pred, const void *__restrict__ z, int z_bytes,
    const int32_t *__restrict__ rows, int64_t N, int T, int64_t n_latent,
    float *__restrict__ pos, int64_t ld, int64_t ov_stride, int32_t *__restrict__ z_out,
    int32_t *__restrict__ z_bad) {
  extern __shared__ float tile[];
  int bad = 0;
  const int o = blockIdx.y;
  const int64_t row = rows ? rows[o] : o;
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * kLoadChunk;
  const int n = static_cast<int>(N - b0 < kLoadChunk ? N - b0 : kLoadChunk);
  const int W = 2 * T, S = W + 1;
  const float *src = pred + (row * N + b0) * W;
  for (int e = threadIdx.x; e < n * W; e += 256) {
    const int p = e / W;
    tile[p * S + (e - p * W)] = src[e];
  }
  if (threadIdx.x < n) {
    const int64_t i = row * N + b0 + threadIdx.x;
    int64_t v = z_bytes == 8 ? static_cast<const int64_t *>(z)[i]
                             : static_cast<int64_t>(static_cast<const int32_t *>(z)[i]);
    // make_ovehicles indexes a list by it (v8ideal/__init__.py:488-491): [-L, 0) wraps as a
    // Python index, anything else outside [0, L) raises IndexError there -- counted in z_bad,
    // clamped here for memory safety
    if (v < 0 && v >= -n_latent) v += n_latent;
    bad = v < 0 || v >= n_latent;
    v = v < 0 ? 0 : (v >= n_latent ? n_latent - 1 : v);
    z_out[o * N + b0 + threadIdx.x] = static_cast<int32_t>(v);
  }
  const int nbad = __syncthreads_count(bad);
  if (threadIdx.x == 0 && nbad > 0 && z_bad) atomicAdd(z_bad + o, nbad);
  float *dst = pos + o * ov_stride + b0;
  for (int e = threadIdx.x; e < W * kLoadChunk; e += 256) {
    const int r = e / kLoadChunk, p = e % kLoadChunk;
    if (p < n) dst[r * ld + p] = tile[p * S + r];
  }
}

extern "C" int ccmpc_load_predictions(const float *pred, const void *z, int z_bytes,
                                      const int32_t *rows, int64_t n_ov, int64_t N, int64_t T,
                                      int64_t n_latent, float *pos_out, int64_t ld_out,
                                      int64_t ov_stride, int32_t *z_out, int32_t *z_bad,
                                      ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T >= 1 && T <= 40, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_ov >= 0 && N >= 0 && n_ov < 65536, "bad n_ov / N");
  CCMPC_REQUIRE(z_bytes == 4 || z_bytes == 8, "z must be int32 or int64");
  CCMPC_REQUIRE(n_latent >= 1, "n_latent must be >= 1");
  if (n_ov == 0 || N == 0) return CCMPC_OK;
  CCMPC_REQUIRE(pred && z && pos_out && z_out, "null pointer");
  CCMPC_REQUIRE(ov_stride >= N && ld_out >= (n_ov - 1) * ov_stride + N, "store too small");
  const int64_t chunks = (N + kLoadChunk - 1) / kLoadChunk;
  CCMPC_REQUIRE(chunks < (int64_t(1) << 31), "N too large");
  const size_t lds = static_cast<size_t>(kLoadChunk) * (2 * T + 1) * sizeof(float);
  hipLaunchKernelGGL(load_predictions_kernel,
                     dim3(static_cast<unsigned>(chunks), static_cast<unsigned>(n_ov)), dim3(256),
                     lds, as_stream(stream), pred, z, z_bytes, rows, N, static_cast<int>(T),
                     n_latent, pos_out, ld_out, ov_stride, z_out, z_bad);
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}
