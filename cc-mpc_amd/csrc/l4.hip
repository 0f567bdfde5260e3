// Per-particle headings, bounding-box vertices and the L4 outer approximation.
//
// Replaces, for every (cell, t):
//   yaws           ovehicle.py:72-76  atan2 of the step delta, step 0 measured from past[-1]
//   vertices       v8ideal/__init__.py:627-640 (utility.npu.vertices_of_bboxes, restated from
//                  midlevel/util.py:104-124): 4 corners of a lon x lat box at each particle
//   A_union/b_union v8ideal/__init__.py:694-736 -> midlevel/util.py:171-200: A = [I; -I] R(theta)
//                  with theta the mean heading, b = max over particles and corners of A v
//   t=0 yaw stats  v8ideal/__init__.py:872, :875 (mean and ddof=1 variance of yaw at t=0)
//
// One workgroup per (cell, t): pass 1 sums the headings (block reduction in a fixed order, so
// the mean is bitwise reproducible), pass 2 takes the max of the four projections over every
// corner, from registers for the particles pass 1 kept (re-reading the two steps beyond them).
// Max is order-independent, so b is exact whatever the reduction order.
#include "gram.hpp"

namespace ccmpc {

#ifndef CCMPC_PROBE
#define CCMPC_PROBE 0
#endif
// CCMPC_PROBE & 4 (diagnostic build only): per-workgroup phase timestamps (s_memrealtime,
// 100 MHz) read back by ccmpc_probe_l4_timestamps (tools/probe_l4.py).
#if CCMPC_PROBE & 4
constexpr int kL4ProbeSlots = 8, kL4ProbeMaxWG = 4096;
__device__ unsigned long long g_l4_ts[kL4ProbeMaxWG * kL4ProbeSlots];
#define L4_TS(k)                                                                               \
  do {                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < kL4ProbeMaxWG)                                        \
      g_l4_ts[blockIdx.x * kL4ProbeSlots + (k)] = __builtin_amdgcn_s_memrealtime();            \
  } while (0)
// the split kernels (pass = 0, 1): 0 start, 1 located, 2 particle loop done, 3 reduced and
// published, 4 last arriver, 5 done (tools/probe_step.py)
__device__ unsigned long long g_l4s_ts[2][kL4ProbeMaxWG * kL4ProbeSlots];
#define L4S_TS(pass, k)                                                                        \
  do {                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < kL4ProbeMaxWG)                                        \
      g_l4s_ts[pass][blockIdx.x * kL4ProbeSlots + (k)] = __builtin_amdgcn_s_memrealtime();     \
  } while (0)
#else
#define L4_TS(k) \
  do {           \
  } while (0)
#define L4S_TS(pass, k) \
  do {                  \
  } while (0)
#endif

template <typename P>
__device__ __forceinline__ double world(const P *pos, int64_t ld, int row, int64_t i, double o) {
  return static_cast<double>(pos[static_cast<int64_t>(row) * ld + i]) + o;
}

template <typename P>
__device__ __forceinline__ double heading(const P *pos, int64_t ld, int t, int64_t i, double o0,
                                          double o1, double px, double py) {
  const double x = world(pos, ld, 2 * t, i, o0), y = world(pos, ld, 2 * t + 1, i, o1);
  double xp, yp;
  if (t == 0) {
    xp = px;
    yp = py;
  } else {
    xp = world(pos, ld, 2 * t - 2, i, o0);
    yp = world(pos, ld, 2 * t - 1, i, o1);
  }
  return atan2(y - yp, x - xp);
}

__device__ __forceinline__ double block_sum(double v, double *red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  const int nw = blockDim.x >> 6;
  for (int k = 0; k < nw; ++k) s += red[k];
  __syncthreads();
  return s;
}

__device__ __forceinline__ double block_max(double v, double *red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = -INFINITY;
  const int nw = blockDim.x >> 6;
  for (int k = 0; k < nw; ++k) s = fmax(s, red[k]);
  __syncthreads();
  return s;
}

// A particle's heading and the (cos, sin) of it.  cos(atan2(dy, dx)) = dx / r and sin = dy / r
// with r = hypot(dx, dy): two divisions instead of a second transcendental (within 2 ulp of
// cos / sin of the rounded atan2, far below the 1e-13 vertex tolerance); a zero step keeps
// sincos of atan2, whose signed-zero cases the ratio cannot express.
__device__ __forceinline__ void heading_cs(double dx, double dy, double &yaw, double &S, double &C) {
#if CCMPC_L4_PROBE_NOATAN  // diagnostic build only: the transcendental's share of the kernel
  yaw = dy * dx;
#else
  yaw = atan2(dy, dx);
#endif
  const double r = sqrt(dx * dx + dy * dy);
  if (r > 0.0 && isfinite(r)) {
    C = dx / r;
    S = dy / r;
  } else {
    sincos(yaw, &S, &C);
  }
}

#ifndef CCMPC_L4_THREADS
#define CCMPC_L4_THREADS 512
#endif
constexpr int kL4Threads = CCMPC_L4_THREADS;  // 8 waves: 2 per SIMD, f64 chains overlap
constexpr int kL4Cache = 12;     // headings kept in registers between the passes (6144 particles)

template <typename P>
__global__ __launch_bounds__(kL4Threads) void l4_kernel(
    const P *__restrict__ pos, int64_t ld, int T, const double *__restrict__ origin,
    const int64_t *__restrict__ cell_off, const int64_t *__restrict__ cell_cnt,
    const double *__restrict__ past_last, const double *__restrict__ bbox,
    double *__restrict__ out_A, double *__restrict__ out_b, double *__restrict__ out_yaw_mean,
    double *__restrict__ out_yaw0_var, double *__restrict__ out_yaw,
    double *__restrict__ out_vertices) {
  __shared__ double red[16];
  L4_TS(0);
  const int cell = blockIdx.x / T, t = blockIdx.x % T;
  const int64_t off = cell_off[cell], n = cell_cnt[cell];
  const double o0 = origin ? origin[2 * cell] : 0.0, o1 = origin ? origin[2 * cell + 1] : 0.0;
  const double px = past_last[2 * cell], py = past_last[2 * cell + 1];
  const double lon = bbox[2 * cell], lat = bbox[2 * cell + 1];
  const P *base = pos + off;
  const int nth = blockDim.x;

  // the step delta of particle i (step 0 measured from past[-1], ovehicle.py:72-76)
  auto delta = [&](int64_t i, double &x, double &y, double &dx, double &dy) {
    x = world(base, ld, 2 * t, i, o0);
    y = world(base, ld, 2 * t + 1, i, o1);
    const double xp = t == 0 ? px : world(base, ld, 2 * t - 2, i, o0);
    const double yp = t == 0 ? py : world(base, ld, 2 * t - 1, i, o1);
    dx = x - xp;
    dy = y - yp;
  };

  // pass 1: headings, mean (and the t = 0 variance, shifted by the first particle's heading);
  // the first kL4Cache headings of each thread (and their cos / sin) stay in registers
  double s = 0.0, s1 = 0.0, s2 = 0.0;
  const double shift = (t == 0 && n > 0) ? heading(base, ld, 0, 0, o0, o1, px, py) : 0.0;
  double yc[kL4Cache], sc[kL4Cache], cc[kL4Cache], xc[kL4Cache], vc[kL4Cache];
  auto take = [&](int64_t i, double y) {
    s += y;
    if (t == 0) {
      const double d = y - shift;
      s1 += d;
      s2 += d * d;
    }
    if (out_yaw) out_yaw[static_cast<int64_t>(t) * ld + off + i] = y;
  };
#pragma unroll
  for (int j = 0; j < kL4Cache; ++j) {
    const int64_t i = threadIdx.x + static_cast<int64_t>(j) * nth;
    if (i < n) {
      double dx, dy;
      delta(i, xc[j], vc[j], dx, dy);
      heading_cs(dx, dy, yc[j], sc[j], cc[j]);
      take(i, yc[j]);
    }
  }
  for (int64_t i = threadIdx.x + static_cast<int64_t>(kL4Cache) * nth; i < n; i += nth) {
    double x, y, dx, dy;
    delta(i, x, y, dx, dy);
    take(i, atan2(dy, dx));
  }
  L4_TS(1);
  const double nn = static_cast<double>(n);
  const double theta = block_sum(s, red) / nn;
  L4_TS(2);
  if (t == 0) {
    const double a = block_sum(s1, red), b2 = block_sum(s2, red);
    if (threadIdx.x == 0) out_yaw0_var[cell] = (b2 - a * a / nn) / (nn - 1.0);
  }

  L4_TS(3);
  // pass 2: corners and the four support values of A = [I; -I] R(theta)
  const double ct = cos(theta), st = sin(theta);
  const double A[4][2] = {{ct, st}, {-st, ct}, {-ct, -st}, {st, -ct}};
  double mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  auto corners = [&](int64_t i, double x, double y, double S, double C) {
    // rows of Rot per corner (midlevel/util.py:109-118), disp = 0.5 * Rot @ [lon, lat]
    const double dx[4] = {0.5 * (C * lon + S * lat), 0.5 * (C * lon - S * lat),
                          0.5 * (-C * lon - S * lat), 0.5 * (-C * lon + S * lat)};
    const double dy[4] = {0.5 * (S * lon - C * lat), 0.5 * (S * lon + C * lat),
                          0.5 * (-S * lon + C * lat), 0.5 * (-S * lon - C * lat)};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const double vx = x + dx[c], vy = y + dy[c];
      if (out_vertices) {
        double *vp = out_vertices + (static_cast<int64_t>(t) * 8 + 2 * c) * ld + off + i;
        vp[0] = vx;
        vp[ld] = vy;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) mx[r] = fmax(mx[r], A[r][0] * vx + A[r][1] * vy);
    }
  };
#pragma unroll
  for (int j = 0; j < kL4Cache; ++j) {
    const int64_t i = threadIdx.x + static_cast<int64_t>(j) * nth;
    if (i < n) corners(i, xc[j], vc[j], sc[j], cc[j]);
  }
  for (int64_t i = threadIdx.x + static_cast<int64_t>(kL4Cache) * nth; i < n; i += nth) {
    double x, y, dx, dy, S, C;
    delta(i, x, y, dx, dy);
    const double r = sqrt(dx * dx + dy * dy);
    if (r > 0.0 && isfinite(r)) {  // cos / sin of the heading without the atan2 (heading_cs)
      C = dx / r;
      S = dy / r;
    } else {
      sincos(atan2(dy, dx), &S, &C);
    }
    corners(i, x, y, S, C);
  }
  L4_TS(4);
  double bm[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bm[r] = block_max(mx[r], red);
  L4_TS(5);
  if (threadIdx.x == 0) {
    const int64_t ct_idx = static_cast<int64_t>(cell) * T + t;
    for (int r = 0; r < 4; ++r) {
      out_A[ct_idx * 8 + 2 * r] = A[r][0];
      out_A[ct_idx * 8 + 2 * r + 1] = A[r][1];
      out_b[ct_idx * 4 + r] = bm[r];
    }
    out_yaw_mean[ct_idx] = theta;
  }
}

// ---- split over workgroups: every (cell, t) on S workgroups ------------------------------------
// One workgroup per (cell, t) is issue-bound on its f64 atan2 / division work for large clouds
// (a 5000-particle cell: 17 us on one CU; 100k particles would take ~0.3 ms), and uses one CU of
// 256.  The split form runs two launches of (cell, t, chunk) workgroups:
//   pass 1  headings of the chunk, partial sums (heading, shifted heading and its square for
//           t = 0) published write-through; the (cell, t)'s last arriver sums them in chunk order
//           -> theta, the yaw statistics, and theta for pass 2 in the workspace;
//   pass 2  the chunk's corners and the four support-value maxima, published the same way; the
//           last arriver takes the max over chunks (order-free) -> b.
// The hand-off is the moment reduction's (gram.hpp: sc1 stores, drain, agent-scope ticket, sc1
// loads); the counters at the head of the zero-filled workspace return to zero every call.
struct L4Split {
  int S;              // workgroups per (cell, t)
  int32_t *ctr;       // [2][n_cells T] arrival counters
  double *part1;      // [n_cells T][S][4]: sum yaw, sum (yaw - shift), sum (yaw - shift)^2, 0
  double *part2;      // [n_cells T][S][4]: the four maxima
  double *theta;      // [n_cells T]
};

inline size_t l4_split_bytes(int64_t T, int64_t n_cells, int S, size_t *o1, size_t *o2,
                             size_t *o3) {
  const int64_t ct = T * n_cells;
  size_t o = ((2 * ct * sizeof(int32_t) + 255) / 256) * 256;
  *o1 = o;
  o += ct * S * 4 * sizeof(double);
  *o2 = o;
  o += ct * S * 4 * sizeof(double);
  *o3 = o;
  o += ct * sizeof(double);
  return (o + 255) / 256 * 256;
}

// Average particles per cell up to which ccmpc_l4_split is ONE launch (pass 2 in the (cell, t)'s
// last arriver of pass 1).  Measured at the drop-in step's C2 shape (~2200 particles per cell):
// 139.6 us per step against 136.2 with the two launches (profiles/r02/v35_l4_one_launch.txt) --
// the last arriver's whole-cell pass costs more than the second launch saves.  Off (0).
#ifndef CCMPC_L4_TAIL2_MAX
#define CCMPC_L4_TAIL2_MAX 0
#endif
constexpr int64_t kL4Tail2Max = CCMPC_L4_TAIL2_MAX;

constexpr int kL4MaxSplit = 64;  // workgroups per (cell, t): one wave holds their partials

// Particles per workgroup on the average cell (build knob): 2048 halves the 784 workgroups of
// a 100k cloud at 1024, whose dispatch alone spread over 7-12 us (profiles/r03/l4_split:
// 100k drop-in graph 113 -> 104 us, C2 shape unchanged; 4096 costs the C2 shape 5 us).
#ifndef CCMPC_L4_SPLIT_CHUNK
#define CCMPC_L4_SPLIT_CHUNK 2048
#endif
#ifndef CCMPC_L4_SPLIT_THREADS  // threads per split workgroup (build knob)
#define CCMPC_L4_SPLIT_THREADS kL4Threads
#endif
constexpr int kL4SplitThreads = CCMPC_L4_SPLIT_THREADS;

inline int l4_split_factor(int64_t n_cells, int64_t n_bound) {
  const int64_t per = n_cells > 0 ? (n_bound + n_cells - 1) / n_cells : 0;
  const int64_t S = (per + CCMPC_L4_SPLIT_CHUNK - 1) / CCMPC_L4_SPLIT_CHUNK;
  return static_cast<int>(S < 1 ? 1 : (S > kL4MaxSplit ? kL4MaxSplit : S));
}

// Pass 2's per-particle work over [i0, i1) of one (cell, t): the bbox corners at the particle's
// own heading and the running maxima of the four support values of A (midlevel/util.py:109-124,
// :171-200).  fmax is exact and order-free, so any split of the particles gives the same b.
template <typename P>
__device__ __forceinline__ void corner_maxima(const P *base, int64_t ld, int t, int64_t i0,
                                              int64_t i1, int64_t off, double o0, double o1,
                                              double px, double py, double lon, double lat,
                                              const double (&A)[4][2], double (&mx)[4],
                                              double *__restrict__ out_vertices) {
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const double x = world(base, ld, 2 * t, i, o0), y = world(base, ld, 2 * t + 1, i, o1);
    const double xp = t == 0 ? px : world(base, ld, 2 * t - 2, i, o0);
    const double yp = t == 0 ? py : world(base, ld, 2 * t - 1, i, o1);
    const double dx = x - xp, dy = y - yp;
    double S, C;
    const double r = sqrt(dx * dx + dy * dy);
    if (r > 0.0 && isfinite(r)) {  // cos / sin of the heading without the atan2 (heading_cs)
      C = dx / r;
      S = dy / r;
    } else {
      sincos(atan2(dy, dx), &S, &C);
    }
    // rows of Rot per corner (midlevel/util.py:109-118), disp = 0.5 * Rot @ [lon, lat]
    const double ddx[4] = {0.5 * (C * lon + S * lat), 0.5 * (C * lon - S * lat),
                           0.5 * (-C * lon - S * lat), 0.5 * (-C * lon + S * lat)};
    const double ddy[4] = {0.5 * (S * lon - C * lat), 0.5 * (S * lon + C * lat),
                           0.5 * (-S * lon + C * lat), 0.5 * (-S * lon - C * lat)};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const double vx = x + ddx[c], vy = y + ddy[c];
      if (out_vertices) {
        double *vp = out_vertices + (static_cast<int64_t>(t) * 8 + 2 * c) * ld + off + i;
        vp[0] = vx;
        vp[ld] = vy;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) mx[q] = fmax(mx[q], A[q][0] * vx + A[q][1] * vy);
    }
  }
}

__device__ __forceinline__ void support_rows(double theta, double (&A)[4][2]) {
  const double ct_ = cos(theta), st_ = sin(theta);
  A[0][0] = ct_; A[0][1] = st_;
  A[1][0] = -st_; A[1][1] = ct_;
  A[2][0] = -ct_; A[2][1] = -st_;
  A[3][0] = st_; A[3][1] = -ct_;
}

template <typename P, bool TAIL2>
__global__ __launch_bounds__(kL4SplitThreads) void l4_pass1_kernel(
    const P *__restrict__ pos, int64_t ld, int T, const double *__restrict__ origin,
    const int64_t *__restrict__ cell_off, const int64_t *__restrict__ cell_cnt,
    const double *__restrict__ past_last, const double *__restrict__ bbox, L4Split sp,
    double *__restrict__ out_yaw_mean, double *__restrict__ out_yaw0_var,
    double *__restrict__ out_yaw, double *__restrict__ out_A, double *__restrict__ out_b) {
  __shared__ double red[16];
  __shared__ double theta_s;
  __shared__ int flag;
  L4S_TS(0, 0);
  const int ct = blockIdx.x / sp.S, part = blockIdx.x % sp.S;
  const int cell = ct / T, t = ct % T;
  const int64_t off = cell_off[cell], n = cell_cnt[cell];
  const double o0 = origin ? origin[2 * cell] : 0.0, o1 = origin ? origin[2 * cell + 1] : 0.0;
  const double px = past_last[2 * cell], py = past_last[2 * cell + 1];
  const P *base = pos + off;
  const int64_t chunk = (n + sp.S - 1) / sp.S;
  const int64_t i0 = part * chunk, i1 = min(n, i0 + chunk);
  const double shift = (t == 0 && n > 0) ? heading(base, ld, 0, 0, o0, o1, px, py) : 0.0;
  L4S_TS(0, 1);
  double s = 0.0, s1 = 0.0, s2 = 0.0;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const double y = heading(base, ld, t, i, o0, o1, px, py);
    s += y;
    if (t == 0) {
      const double d = y - shift;
      s1 += d;
      s2 += d * d;
    }
    if (out_yaw) out_yaw[static_cast<int64_t>(t) * ld + off + i] = y;
  }
  L4S_TS(0, 2);
  s = block_sum(s, red);
  if (t == 0) {
    s1 = block_sum(s1, red);
    s2 = block_sum(s2, red);
  }
  double *mine = sp.part1 + (static_cast<int64_t>(ct) * sp.S + part) * 4;
  const __amdgpu_buffer_rsrc_t rm = slab_rsrc(mine);
  if (threadIdx.x == 0) {
    st2_sc1(rm, 0, s, s1);
    st2_sc1(rm, 16, s2, 0.0);
  }
  L4S_TS(0, 3);
  if (!arrive_last(sp.ctr + ct, sp.S, &flag)) return;
  L4S_TS(0, 4);
  // every chunk's partials loaded at once (thread k: chunk k), then summed in chunk order by one
  // thread from LDS: deterministic, and one L2 round trip instead of S dependent ones
  const __amdgpu_buffer_rsrc_t rp = slab_rsrc(sp.part1 + static_cast<int64_t>(ct) * sp.S * 4);
  __shared__ double2 pu[kL4MaxSplit], pv[kL4MaxSplit];
  if (threadIdx.x < sp.S) {
    pu[threadIdx.x] = ld2_sc1(rp, 32 * threadIdx.x);
    pv[threadIdx.x] = ld2_sc1(rp, 32 * threadIdx.x + 16);
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // chunk order: deterministic
    double a = 0.0, b1 = 0.0, b2 = 0.0;
    for (int k = 0; k < sp.S; ++k) {
      a += pu[k].x;
      b1 += pu[k].y;
      b2 += pv[k].x;
    }
    const double nn = static_cast<double>(n);
    const double theta = a / nn;
    sp.theta[ct] = theta;
    theta_s = theta;
    out_yaw_mean[ct] = theta;
    if (t == 0) out_yaw0_var[cell] = (b2 - b1 * b1 / nn) / (nn - 1.0);
  }
  L4S_TS(0, 5);
  if (!TAIL2) return;
  // small cells: the (cell, t)'s last arriver runs pass 2 over the whole cell itself (no second
  // launch, no second hand-off; the maxima are order-free, so b is the two-pass b bit for bit)
  __syncthreads();
  double A[4][2];
  support_rows(theta_s, A);
  double mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  corner_maxima(base, ld, t, 0, n, off, o0, o1, px, py, bbox[2 * cell], bbox[2 * cell + 1], A, mx,
                static_cast<double *>(nullptr));
  double bm[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) bm[q] = block_max(mx[q], red);
  if (threadIdx.x == 0)
    for (int q = 0; q < 4; ++q) {
      out_A[static_cast<int64_t>(ct) * 8 + 2 * q] = A[q][0];
      out_A[static_cast<int64_t>(ct) * 8 + 2 * q + 1] = A[q][1];
      out_b[static_cast<int64_t>(ct) * 4 + q] = bm[q];
    }
}

template <typename P>
__global__ __launch_bounds__(kL4SplitThreads) void l4_pass2_kernel(
    const P *__restrict__ pos, int64_t ld, int T, const double *__restrict__ origin,
    const int64_t *__restrict__ cell_off, const int64_t *__restrict__ cell_cnt,
    const double *__restrict__ past_last, const double *__restrict__ bbox, L4Split sp,
    double *__restrict__ out_A, double *__restrict__ out_b, double *__restrict__ out_vertices) {
  __shared__ double red[16];
  __shared__ int flag;
  L4S_TS(1, 0);
  const int ct = blockIdx.x / sp.S, part = blockIdx.x % sp.S;
  const int cell = ct / T, t = ct % T;
  const int64_t off = cell_off[cell], n = cell_cnt[cell];
  const double o0 = origin ? origin[2 * cell] : 0.0, o1 = origin ? origin[2 * cell + 1] : 0.0;
  const double px = past_last[2 * cell], py = past_last[2 * cell + 1];
  const double lon = bbox[2 * cell], lat = bbox[2 * cell + 1];
  const P *base = pos + off;
  const int64_t chunk = (n + sp.S - 1) / sp.S;
  const int64_t i0 = part * chunk, i1 = min(n, i0 + chunk);
  const double theta = sp.theta[ct];  // written by pass 1 (an earlier launch)
  double A[4][2];
  support_rows(theta, A);
  L4S_TS(1, 1);
  double mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  corner_maxima(base, ld, t, i0, i1, off, o0, o1, px, py, lon, lat, A, mx, out_vertices);
  L4S_TS(1, 2);
  double bm[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) bm[q] = block_max(mx[q], red);
  double *mine = sp.part2 + (static_cast<int64_t>(ct) * sp.S + part) * 4;
  const __amdgpu_buffer_rsrc_t rm = slab_rsrc(mine);
  if (threadIdx.x == 0) {
    st2_sc1(rm, 0, bm[0], bm[1]);
    st2_sc1(rm, 16, bm[2], bm[3]);
  }
  L4S_TS(1, 3);
  const int nct = gridDim.x / sp.S;
  if (!arrive_last(sp.ctr + nct + ct, sp.S, &flag)) return;
  L4S_TS(1, 4);
  // the maxima over chunks (order-free): the first wave loads them all at once and reduces
  if (threadIdx.x < 64) {
    const __amdgpu_buffer_rsrc_t rp = slab_rsrc(sp.part2 + static_cast<int64_t>(ct) * sp.S * 4);
    double b[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    if (threadIdx.x < sp.S) {
      const double2 u = ld2_sc1(rp, 32 * threadIdx.x), v = ld2_sc1(rp, 32 * threadIdx.x + 16);
      b[0] = u.x;
      b[1] = u.y;
      b[2] = v.x;
      b[3] = v.y;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) b[q] = fmax(b[q], __shfl_xor(b[q], o, 64));
    if (threadIdx.x == 0)
      for (int q = 0; q < 4; ++q) {
        out_A[static_cast<int64_t>(ct) * 8 + 2 * q] = A[q][0];
        out_A[static_cast<int64_t>(ct) * 8 + 2 * q + 1] = A[q][1];
        out_b[static_cast<int64_t>(ct) * 4 + q] = b[q];
      }
  }
  L4S_TS(1, 5);
}

}  // namespace ccmpc

using namespace ccmpc;

#if CCMPC_PROBE & 4
extern "C" int ccmpc_probe_l4_timestamps(void *host, int reset) {
  const size_t bytes = sizeof(g_l4_ts);
  if (reset) {
    static unsigned long long zeros[kL4ProbeMaxWG * kL4ProbeSlots];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_l4_ts), zeros, bytes) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_l4_ts), bytes) == hipSuccess ? 0 : -1;
}
extern "C" int ccmpc_probe_l4_split_timestamps(void *host, int which, int reset) {
  if (which < 0 || which > 1) return -1;
  const size_t bytes = sizeof(g_l4s_ts[0]);
  if (reset) {
    static unsigned long long zeros[kL4ProbeMaxWG * kL4ProbeSlots];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_l4s_ts), zeros, bytes, which * bytes) == hipSuccess
               ? 0 : -1;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_l4s_ts), bytes, which * bytes) == hipSuccess
             ? 0 : -1;
}
#endif

extern "C" int ccmpc_l4(const void *positions, int dtype, int64_t ld, int64_t T,
                        const double *origin, const int64_t *cell_off, const int64_t *cell_cnt,
                        int64_t n_cells, const double *past_last, const double *bbox,
                        double *out_A, double *out_b, double *out_yaw_mean,
                        double *out_yaw0_var, double *out_yaw, double *out_vertices,
                        ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T >= 1 && T <= 40, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_cells >= 0 && n_cells * T < (int64_t(1) << 31), "bad n_cells");
  if (n_cells == 0) return CCMPC_OK;
  CCMPC_REQUIRE(positions && cell_off && cell_cnt && past_last && bbox && out_A && out_b &&
                    out_yaw_mean && out_yaw0_var,
                "null pointer");
  CCMPC_REQUIRE(dtype == CCMPC_F64 || dtype == CCMPC_F32, "bad dtype");
  const dim3 grid(static_cast<unsigned>(n_cells * T));
  if (dtype == CCMPC_F64)
    hipLaunchKernelGGL((l4_kernel<double>), grid, dim3(kL4Threads), 0, as_stream(stream),
                       static_cast<const double *>(positions), ld, static_cast<int>(T), origin,
                       cell_off, cell_cnt, past_last, bbox, out_A, out_b, out_yaw_mean,
                       out_yaw0_var, out_yaw, out_vertices);
  else
    hipLaunchKernelGGL((l4_kernel<float>), grid, dim3(kL4Threads), 0, as_stream(stream),
                       static_cast<const float *>(positions), ld, static_cast<int>(T), origin,
                       cell_off, cell_cnt, past_last, bbox, out_A, out_b, out_yaw_mean,
                       out_yaw0_var, out_yaw, out_vertices);
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}

extern "C" size_t ccmpc_l4_workspace_bytes(int64_t T, int64_t n_cells, int64_t n_particles_bound) {
  if (T < 1 || T > 40 || n_cells < 0 || n_particles_bound < 0) return 0;
  size_t o1, o2, o3;
  return l4_split_bytes(T, n_cells, l4_split_factor(n_cells, n_particles_bound), &o1, &o2, &o3);
}

extern "C" int ccmpc_l4_split(const void *positions, int dtype, int64_t ld, int64_t T,
                              const double *origin, const int64_t *cell_off,
                              const int64_t *cell_cnt, int64_t n_cells,
                              int64_t n_particles_bound, const double *past_last,
                              const double *bbox, void *workspace, size_t workspace_bytes,
                              double *out_A, double *out_b, double *out_yaw_mean,
                              double *out_yaw0_var, double *out_yaw, double *out_vertices,
                              ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T >= 1 && T <= 40, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_cells >= 0 && n_cells * T * 64 < (int64_t(1) << 31), "bad n_cells");
  if (n_cells == 0) return CCMPC_OK;
  CCMPC_REQUIRE(positions && cell_off && cell_cnt && past_last && bbox && out_A && out_b &&
                    out_yaw_mean && out_yaw0_var,
                "null pointer");
  CCMPC_REQUIRE(dtype == CCMPC_F64 || dtype == CCMPC_F32, "bad dtype");
  CCMPC_REQUIRE(workspace && aligned(workspace, 256), "workspace must be 256-byte aligned");
  const int S = l4_split_factor(n_cells, n_particles_bound);
  size_t o1, o2, o3;
  if (workspace_bytes < l4_split_bytes(T, n_cells, S, &o1, &o2, &o3)) {
    set_error("ccmpc_l4_split: workspace too small");
    return CCMPC_ERR_WORKSPACE;
  }
  char *w = static_cast<char *>(workspace);
  const L4Split sp{S, reinterpret_cast<int32_t *>(w), reinterpret_cast<double *>(w + o1),
                   reinterpret_cast<double *>(w + o2), reinterpret_cast<double *>(w + o3)};
  const dim3 grid(static_cast<unsigned>(n_cells * T * S));
  hipStream_t s = as_stream(stream);
  const int Ti = static_cast<int>(T);
  // small cells (<= kL4Tail2Max particles on average, no vertex output): one launch, pass 2 in
  // the (cell, t)'s last arriver of pass 1
  const bool tail2 = !out_vertices && n_particles_bound <= kL4Tail2Max * n_cells;
  auto run = [&](auto tag) {
    using P = decltype(tag);
    const P *p = static_cast<const P *>(positions);
    if (tail2) {
      hipLaunchKernelGGL((l4_pass1_kernel<P, true>), grid, dim3(kL4SplitThreads), 0, s, p, ld, Ti,
                         origin, cell_off, cell_cnt, past_last, bbox, sp, out_yaw_mean,
                         out_yaw0_var, out_yaw, out_A, out_b);
      return;
    }
    hipLaunchKernelGGL((l4_pass1_kernel<P, false>), grid, dim3(kL4SplitThreads), 0, s, p, ld, Ti,
                       origin, cell_off, cell_cnt, past_last, bbox, sp, out_yaw_mean,
                       out_yaw0_var, out_yaw, out_A, out_b);
    hipLaunchKernelGGL((l4_pass2_kernel<P>), grid, dim3(kL4SplitThreads), 0, s, p, ld, Ti, origin,
                       cell_off, cell_cnt, past_last, bbox, sp, out_A, out_b, out_vertices);
  };
  if (dtype == CCMPC_F64)
    run(double{});
  else
    run(float{});
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}
