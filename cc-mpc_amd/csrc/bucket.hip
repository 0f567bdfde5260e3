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
// mode and 1 + z for a rare latent.  Five short kernels:
//   B1 stats   per block: latent counts (LDS int atomics, exact) and per-kept-mode sums of the
//              final positions (fixed-order block reductions)
//   B2 centres one block per OV: sums in block order -> centres
//   B3 keys    per block: key histogram (LDS int atomics, exact)
//   B4 scan    one block per OV: bin offsets (bin-major, block-minor), 4-aligned cell offsets
//   B5 scatter per block: stable rank inside the block (wave ballots, waves in order) -> copy
//              the particle's 2T coordinates to its bucket slot
// Everything is integer-exact except the centre sums, whose fixed order makes them
// deterministic; the bucketed store is bit-identical across runs.
#include "ccmpc_common.hpp"

namespace ccmpc {

constexpr int kBucketBlock = 256;
constexpr int kPerThread = 4;
constexpr int kSpan = kBucketBlock * kPerThread;  // particles per block, in sample order
constexpr int kMaxBins = 1024;
constexpr int kMaxKept = 16;

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
  int32_t *cnt_lat;         // [n_ov][nb][L]
  double *sum_xy;           // [n_ov][nb][max_k][2]
  double *centre;           // [n_ov][max_k][2]
  int32_t *hist;            // [n_ov][nb][nbins]
  int64_t *bin_off;         // [n_ov][nb][nbins]
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

// bucket key of particle i of OV o (needs centres for rare latents)
__device__ __forceinline__ int key_of(const BucketArgs &a, int o, int64_t i) {
  const int zv = a.z[o * a.N + i];
  const int k = a.keep_map[o * a.L + zv];
  if (k >= 0) return k * (a.L + 1);
  double x, y;
  final_world(a, o, i, x, y);
  const int K = a.n_kept[o];
  int best = 0;
  double bd = INFINITY;
  for (int j = 0; j < K; ++j) {
    const double dx = x - a.centre[(o * a.max_k + j) * 2], dy = y - a.centre[(o * a.max_k + j) * 2 + 1];
    const double d = sqrt(dx * dx + dy * dy);
    if (d < bd) {
      bd = d;
      best = j;
    }
  }
  return best * (a.L + 1) + 1 + zv;
}

__global__ __launch_bounds__(kBucketBlock) void bucket_stats(BucketArgs a) {
  __shared__ int cnt[64];
  __shared__ double red[4];
  const int o = blockIdx.y, blk = blockIdx.x;
  for (int l = threadIdx.x; l < a.L; l += blockDim.x) cnt[l] = 0;
  __syncthreads();
  const int64_t i0 = static_cast<int64_t>(blk) * kSpan;
  int zs[kPerThread];
  double xs[kPerThread], ys[kPerThread];
#pragma unroll
  for (int r = 0; r < kPerThread; ++r) {
    const int64_t i = i0 + r * kBucketBlock + threadIdx.x;
    zs[r] = -1;
    xs[r] = ys[r] = 0.0;
    if (i < a.N) {
      zs[r] = a.z[o * a.N + i];
      atomicAdd(&cnt[zs[r]], 1);
      final_world(a, o, i, xs[r], ys[r]);
    }
  }
  for (int k = 0; k < a.n_kept[o]; ++k) {
    double sx = 0.0, sy = 0.0;
#pragma unroll
    for (int r = 0; r < kPerThread; ++r) {
      const bool mine = zs[r] >= 0 && a.keep_map[o * a.L + zs[r]] == k;
      sx += mine ? xs[r] : 0.0;
      sy += mine ? ys[r] : 0.0;
    }
    sx = block_sum256(sx, red);
    sy = block_sum256(sy, red);
    if (threadIdx.x == 0) {
      double *d = a.sum_xy + ((static_cast<int64_t>(o) * a.nb + blk) * a.max_k + k) * 2;
      d[0] = sx;
      d[1] = sy;
    }
  }
  __syncthreads();
  for (int l = threadIdx.x; l < a.L; l += blockDim.x)
    a.cnt_lat[(static_cast<int64_t>(o) * a.nb + blk) * a.L + l] = cnt[l];
}

__global__ __launch_bounds__(64) void bucket_centres(BucketArgs a) {
  const int o = blockIdx.x;
  for (int k = threadIdx.x; k < a.n_kept[o]; k += blockDim.x) {
    int zv = 0;
    for (int l = 0; l < a.L; ++l)
      if (a.keep_map[o * a.L + l] == k) zv = l;
    int64_t n = 0;
    double sx = 0.0, sy = 0.0;
    for (int b = 0; b < a.nb; ++b) {
      n += a.cnt_lat[(static_cast<int64_t>(o) * a.nb + b) * a.L + zv];
      const double *s = a.sum_xy + ((static_cast<int64_t>(o) * a.nb + b) * a.max_k + k) * 2;
      sx += s[0];
      sy += s[1];
    }
    a.centre[(o * a.max_k + k) * 2] = sx / static_cast<double>(n);
    a.centre[(o * a.max_k + k) * 2 + 1] = sy / static_cast<double>(n);
    const int cell = a.cell_base[o] + k;
    a.init_center[2 * cell] = sx / static_cast<double>(n);
    a.init_center[2 * cell + 1] = sy / static_cast<double>(n);
  }
}

__global__ __launch_bounds__(kBucketBlock) void bucket_hist(BucketArgs a) {
  __shared__ int h[kMaxBins];
  const int o = blockIdx.y, blk = blockIdx.x;
  const int nbins = a.n_kept[o] * (a.L + 1);
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const int64_t i0 = static_cast<int64_t>(blk) * kSpan;
#pragma unroll
  for (int r = 0; r < kPerThread; ++r) {
    const int64_t i = i0 + r * kBucketBlock + threadIdx.x;
    if (i < a.N) atomicAdd(&h[key_of(a, o, i)], 1);
  }
  __syncthreads();
  const int64_t stride = static_cast<int64_t>(a.max_k) * (a.L + 1);
  for (int b = threadIdx.x; b < nbins; b += blockDim.x)
    a.hist[(static_cast<int64_t>(o) * a.nb + blk) * stride + b] = h[b];
}

__global__ __launch_bounds__(256) void bucket_scan(BucketArgs a) {
  __shared__ int64_t tot[kMaxBins];
  __shared__ int64_t start[kMaxBins];
  const int o = blockIdx.x;
  const int K = a.n_kept[o];
  const int G = a.L + 1;
  const int nbins = K * G;
  const int64_t stride = static_cast<int64_t>(a.max_k) * G;
  const int32_t *hist = a.hist + static_cast<int64_t>(o) * a.nb * stride;
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) {
    int64_t s = 0;
    for (int blk = 0; blk < a.nb; ++blk) s += hist[blk * stride + b];
    tot[b] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t cur = a.region[o];
    for (int k = 0; k < K; ++k) {
      int64_t n = 0;
      for (int gi = 0; gi < G; ++gi) {
        start[k * G + gi] = cur + n;
        n += tot[k * G + gi];
      }
      const int cell = a.cell_base[o] + k;
      a.cell_off[cell] = cur;
      a.cell_cnt[cell] = n;
      a.cell_pmf[cell] = static_cast<double>(n) / static_cast<double>(a.N);
      cur += (n + 3) & ~int64_t(3);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) {
    int64_t s = start[b];
    for (int blk = 0; blk < a.nb; ++blk) {
      a.bin_off[(static_cast<int64_t>(o) * a.nb + blk) * stride + b] = s;
      s += hist[blk * stride + b];
    }
  }
}

__global__ __launch_bounds__(kBucketBlock) void bucket_scatter(BucketArgs a) {
  __shared__ int run[kMaxBins];        // particles of each bin in earlier rounds of this block
  __shared__ int wcnt[4][kMaxBins];    // per wave counts of the current round
  const int o = blockIdx.y, blk = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nbins = a.n_kept[o] * (a.L + 1);
  const int64_t stride = static_cast<int64_t>(a.max_k) * (a.L + 1);
  const int64_t *boff = a.bin_off + (static_cast<int64_t>(o) * a.nb + blk) * stride;
  for (int b = threadIdx.x; b < nbins; b += blockDim.x) run[b] = 0;
  const int64_t i0 = static_cast<int64_t>(blk) * kSpan;
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int r = 0; r < kPerThread; ++r) {
    for (int b = threadIdx.x; b < 4 * nbins; b += blockDim.x) wcnt[b / nbins][b % nbins] = 0;
    __syncthreads();
    const int64_t i = i0 + r * kBucketBlock + threadIdx.x;  // sample order = (round, wave, lane)
    const bool valid = i < a.N;
    const int key = valid ? key_of(a, o, i) : -1;
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
      for (int v = 0; v < w; ++v) before += wcnt[v][key];
      const int64_t dst = boff[key] + before + rank;
      const float *src = a.pos + o * a.S_in + i;
      for (int row = 0; row < 2 * a.T; ++row) a.out[row * a.ld_out + dst] = src[row * a.ld_in];
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nbins; b += blockDim.x)
      run[b] += wcnt[0][b] + wcnt[1][b] + wcnt[2][b] + wcnt[3][b];
    __syncthreads();
  }
}

inline size_t align256(size_t b) { return (b + 255) / 256 * 256; }

struct WsLayout {
  size_t cnt_lat, sum_xy, centre, hist, bin_off, total;
};

inline WsLayout bucket_ws(int64_t n_ov, int64_t N, int64_t L, int64_t max_k) {
  const int64_t nb = (N + kSpan - 1) / kSpan;
  WsLayout w;
  size_t o = 0;
  w.cnt_lat = o;
  o += align256(sizeof(int32_t) * n_ov * nb * L);
  w.sum_xy = o;
  o += align256(sizeof(double) * n_ov * nb * max_k * 2);
  w.centre = o;
  o += align256(sizeof(double) * n_ov * max_k * 2);
  w.hist = o;
  o += align256(sizeof(int32_t) * n_ov * nb * max_k * (L + 1));
  w.bin_off = o;
  o += align256(sizeof(int64_t) * n_ov * nb * max_k * (L + 1));
  w.total = o;
  return w;
}

}  // namespace ccmpc

using namespace ccmpc;

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
  a.cnt_lat = reinterpret_cast<int32_t *>(ws + L.cnt_lat);
  a.sum_xy = reinterpret_cast<double *>(ws + L.sum_xy);
  a.centre = reinterpret_cast<double *>(ws + L.centre);
  a.hist = reinterpret_cast<int32_t *>(ws + L.hist);
  a.bin_off = reinterpret_cast<int64_t *>(ws + L.bin_off);
  a.out = pos_out;
  a.ld_out = ld_out;
  a.cell_off = cell_off;
  a.cell_cnt = cell_cnt;
  a.cell_pmf = cell_pmf;
  a.init_center = init_center;
  hipStream_t s = as_stream(stream);
  const dim3 grid(static_cast<unsigned>(a.nb), static_cast<unsigned>(n_ov));
  hipLaunchKernelGGL(bucket_stats, grid, dim3(kBucketBlock), 0, s, a);
  hipLaunchKernelGGL(bucket_centres, dim3(static_cast<unsigned>(n_ov)), dim3(64), 0, s, a);
  hipLaunchKernelGGL(bucket_hist, grid, dim3(kBucketBlock), 0, s, a);
  hipLaunchKernelGGL(bucket_scan, dim3(static_cast<unsigned>(n_ov)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(bucket_scatter, grid, dim3(kBucketBlock), 0, s, a);
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}
