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
//              write-through; the OV's last arriving block sums them in the canonical order
//              (bucket.hpp) -> centres
//   B2 keys    per block: key histogram (LDS int atomics, exact), published write-through; the
//              OV's last arriving block scans them -> per chunk of 16 blocks the bin starts,
//              4-aligned cell offsets
//   B3 scatter per block: stable rank inside the block (wave ballots, waves in order) -> copy
//              the particle's 2T coordinates to its bucket slot
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
  int32_t *ctr;             // [2][n_ov] arrival counters (zero between calls)
  double *part;             // [n_ov][nb][E1]: latent counts [L] (as doubles; E1 even)
  int E1;
  double *gpart;            // [n_ov][G][max_k][2]: per 64-particle group kept-mode sums
  int G;                    // groups per OV = ceil(N / 64)
  double *centre;           // [n_ov][max_k][2]
  int32_t *hist;            // [n_ov][nb][nbins]
  int64_t *chunk_off;       // [n_ov][ceil(nb / kChunkRows)][nbins]: each chunk's bin starts
  // outputs
  float *out;
  int64_t ld_out;
  int64_t *cell_off, *cell_cnt;
  double *cell_pmf, *init_center;
};

__device__ __forceinline__ double block_sum256(double v, double *red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane == 0) red[w] = v;
  __syncthreads();
  const double s = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return s;
}

__device__ __forceinline__ void final_world(const BucketArgs &a, int o, int64_t i, double &x,
                                            double &y) {
  const float *p = a.pos + o * a.S_in + i;
  x = static_cast<double>(p[(2 * (a.T - 1)) * a.ld_in]) + a.minpos[2 * o];
  y = static_cast<double>(p[(2 * (a.T - 1) + 1) * a.ld_in]) + a.minpos[2 * o + 1];
}

__global__ __launch_bounds__(kBucketBlock) void bucket_stats(BucketArgs a) {
  BKT_TS(0, 0);
  __shared__ int cnt[64];
  __shared__ double red[4];
  __shared__ int flag;
  __shared__ int keep_s[64];
  __shared__ int zv_s[kMaxKept];
  __shared__ double nk_s[kMaxKept];
  __shared__ double2 sup_s[kMaxKept][kCentreSuper];
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
  // latent counts, published write-through; the OV's last arriver combines them
  double *mine = a.part + (static_cast<int64_t>(o) * a.nb + blk) * a.E1;
  const __amdgpu_buffer_rsrc_t rm = slab_rsrc(mine);
  for (int e = 2 * threadIdx.x; e < a.L; e += 2 * blockDim.x)
    st2_sc1(rm, 8 * e, static_cast<double>(cnt[e]),
            e + 1 < a.L ? static_cast<double>(cnt[e + 1]) : 0.0);
  BKT_TS(0, 2);
  if (!arrive_last(a.ctr + o, a.nb, &flag)) return;
  BKT_TS(0, 3);
  for (int l = threadIdx.x; l < a.L; l += blockDim.x) {
    const int k = keep_s[l];
    if (k >= 0) zv_s[k] = l;
  }
  __syncthreads();
  // n_k: kept mode k's own particles (integer-exact in any order); every mode's loads together
  const __amdgpu_buffer_rsrc_t rp = slab_rsrc(a.part + static_cast<int64_t>(o) * a.nb * a.E1);
  constexpr int KB = 4;
  for (int k0 = 0; k0 < K; k0 += KB) {
    double n[KB];
#pragma unroll
    for (int j = 0; j < KB; ++j) n[j] = 0.0;
    for (int b = threadIdx.x; b < a.nb; b += blockDim.x) {
      double2 c[KB];
#pragma unroll
      for (int j = 0; j < KB; ++j) {
        const int k = k0 + j < K ? k0 + j : K - 1;  // clamped: always a valid address
        c[j] = ld2_sc1(rp, 8 * (b * a.E1 + (zv_s[k] & ~1)));
      }
#pragma unroll
      for (int j = 0; j < KB; ++j) n[j] += (zv_s[k0 + j < K ? k0 + j : K - 1] & 1) ? c[j].y : c[j].x;
    }
#pragma unroll
    for (int j = 0; j < KB; ++j) {
      const double s = block_sum256(n[j], red);
      if (k0 + j < K && threadIdx.x == 0) nk_s[k0 + j] = s;
    }
  }
  // the canonical centre sums (bucket.hpp): superblocks in parallel, then left to right
  const int J = (a.G + kCentreSuper - 1) / kCentreSuper;
  double2 tot = {0.0, 0.0};  // thread k's running sum of mode k
  for (int j0 = 0; j0 < J; j0 += kCentreSuper) {
    const int nj = min(kCentreSuper, J - j0);
    for (int u = threadIdx.x; u < K * nj; u += blockDim.x) {
      const int k = u / nj, j = j0 + u % nj;
      sup_s[k][j - j0] = superblock_sum(j, a.G, [&](int gg) {
        return ld2_sc1(rg, 16 * (gg * a.max_k + k));
      });
    }
    __syncthreads();
    if (threadIdx.x < K)
      for (int j = 0; j < nj; ++j) {
        tot.x += sup_s[threadIdx.x][j].x;
        tot.y += sup_s[threadIdx.x][j].y;
      }
    __syncthreads();
  }
  if (threadIdx.x < K) {
    const int k = threadIdx.x;
    const double cx = tot.x / nk_s[k], cy = tot.y / nk_s[k];
    a.centre[(o * a.max_k + k) * 2] = cx;
    a.centre[(o * a.max_k + k) * 2 + 1] = cy;
    const int cell = a.cell_base[o] + k;
    a.init_center[2 * cell] = cx;
    a.init_center[2 * cell + 1] = cy;
  }
  BKT_TS(0, 4);
}

__global__ __launch_bounds__(kBucketBlock) void bucket_hist(BucketArgs a) {
  BKT_TS(1, 0);
  __shared__ int h[kMaxBins];
  __shared__ int64_t start[kMaxBins];
  __shared__ int flag;
  __shared__ int keep_s[64];
  __shared__ double cen_s[kMaxKept][2];
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
  int32_t *hist0 = a.hist + static_cast<int64_t>(o) * a.nb * stride;
  const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(hist0, 0, 0x7fffffff,
                                                                       0x00020000);
  for (int b = threadIdx.x; b < nbins; b += blockDim.x)
    st1_sc1(rh, 4 * static_cast<int>(blk * stride + b), h[b]);
  BKT_TS(1, 2);
  if (!arrive_last(a.ctr + a.n_ov + o, a.nb, &flag)) return;
  BKT_TS(1, 3);
  // The OV's scan, as integer sums over the published block histograms (exact: the order of the
  // additions does not matter).  (1) per (chunk of kChunkRows blocks, bin) column sums -- every
  // load of a task in flight together, two tasks per round, all threads -- into chunk_off and
  // the bin totals (LDS int64 atomics); (2) bin starts and cell offsets; (3) per bin, each
  // chunk's start in place of its sum.  bucket_scatter adds the block's offset inside its chunk
  // (<= kChunkRows - 1 rows).  The old per-bin serial column walk over all nb blocks (twice) was
  // a dependent chain of ~nb / 8 round trips: 63 us at N = 100 000.
  const int nch = (a.nb + kChunkRows - 1) / kChunkRows;
  int64_t *coff = a.chunk_off + static_cast<int64_t>(o) * nch * stride;
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) start[b] = 0;
  __syncthreads();
  const int tasks = nch * nbins;
  auto chunk_sum = [&](int task) {
    const int c = task / nbins, b = task - c * nbins;
    const int r0 = c * kChunkRows, nr = min(kChunkRows, a.nb - r0);
    int32_t v[kChunkRows];
#pragma unroll
    for (int j = 0; j < kChunkRows; ++j)
      v[j] = ld1_sc1(rh, 4 * static_cast<int>((r0 + (j < nr ? j : nr - 1)) * stride + b));
    int64_t sum = 0;
#pragma unroll
    for (int j = 0; j < kChunkRows; ++j) sum += j < nr ? v[j] : 0;
    return sum;
  };
  for (int t0 = threadIdx.x; t0 < tasks; t0 += 2 * blockDim.x) {
    const int t1 = t0 + blockDim.x;
    const int64_t s0 = chunk_sum(t0);
    const int64_t s1 = t1 < tasks ? chunk_sum(t1) : 0;
    coff[(t0 / nbins) * stride + t0 % nbins] = s0;
    atomicAdd(reinterpret_cast<unsigned long long *>(&start[t0 % nbins]),
              static_cast<unsigned long long>(s0));
    if (t1 < tasks) {
      coff[(t1 / nbins) * stride + t1 % nbins] = s1;
      atomicAdd(reinterpret_cast<unsigned long long *>(&start[t1 % nbins]),
                static_cast<unsigned long long>(s1));
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's chunk sums, read below
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
  // each chunk's start in every bin: the bin's start + the sums of the chunks before it
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(coff, 0, 0x7fffffff,
                                                                       0x00020000);
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) {
    int64_t run = start[b];
    for (int c0 = 0; c0 < nch; c0 += 8) {
      int64_t v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {  // 8-byte sc1 loads: L2-served (no stale L1 line)
        const int c = c0 + j < nch ? c0 + j : nch - 1;
        const int off = 8 * static_cast<int>(c * stride + b);
        const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rc, off, 0, 16);
        const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rc, off + 4, 0, 16);
        v[j] = static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (c0 + j < nch) coff[(c0 + j) * stride + b] = run;
        run += c0 + j < nch ? v[j] : 0;
      }
    }
  }
  BKT_TS(1, 4);
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
  const int nch = (a.nb + kChunkRows - 1) / kChunkRows, ch = blk / kChunkRows;
  const int64_t *coff = a.chunk_off + (static_cast<int64_t>(o) * nch + ch) * stride;
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
  size_t ctr, part, gpart, centre, hist, chunk_off, total;
  int E1, G;
};

inline WsLayout bucket_ws(int64_t n_ov, int64_t N, int64_t L, int64_t max_k) {
  const int64_t nb = (N + kSpan - 1) / kSpan;
  WsLayout w;
  w.E1 = static_cast<int>((L + 1) & ~int64_t(1));
  w.G = static_cast<int>((N + kCentreGroup - 1) / kCentreGroup);
  size_t o = 0;
  w.ctr = o;  // arrival counters first: the zero-filled head of the workspace
  o += align256(sizeof(int32_t) * 2 * n_ov);
  w.part = o;
  o += align256(sizeof(double) * n_ov * nb * w.E1);
  w.gpart = o;
  o += align256(sizeof(double) * n_ov * w.G * max_k * 2);
  w.centre = o;
  o += align256(sizeof(double) * n_ov * max_k * 2);
  w.hist = o;
  o += align256(sizeof(int32_t) * n_ov * nb * max_k * (L + 1));
  w.chunk_off = o;
  o += align256(sizeof(int64_t) * n_ov * ((nb + kChunkRows - 1) / kChunkRows) * max_k * (L + 1));
  w.total = o;
  return w;
}

}  // namespace ccmpc

using namespace ccmpc;

#if defined(CCMPC_PROBE) && (CCMPC_PROBE & 4)
// which: 0 stats (slots 0 start, 1 loaded, 2 published, 3 last arriver, 4 done), 1 hist (same),
// 2 scatter (0 start, 1 loaded, 2 done)  (tools/probe_step.py)
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
  a.part = reinterpret_cast<double *>(ws + L.part);
  a.E1 = L.E1;
  a.gpart = reinterpret_cast<double *>(ws + L.gpart);
  a.G = L.G;
  a.centre = reinterpret_cast<double *>(ws + L.centre);
  a.hist = reinterpret_cast<int32_t *>(ws + L.hist);
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
