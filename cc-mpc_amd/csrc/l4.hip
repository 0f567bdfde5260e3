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

#ifndef CCMPC_L4_THREADS
#define CCMPC_L4_THREADS 1024
#endif
// one workgroup per (cell, t): 16 waves, 4 per SIMD, so the f64 atan2 chains of a 5000-particle
// cell overlap (C2 step: 14.8 us against 16.2 at 512 threads, profiles/r06/probes/l4wg_*)
constexpr int kL4Threads = CCMPC_L4_THREADS;
constexpr int kL4Cache = 5120 / kL4Threads;  // particles per thread kept in registers between passes

// ---- split over workgroups: every (cell, t) on S workgroups ------------------------------------
// One workgroup per (cell, t) is issue-bound on its f64 atan2 / division work for large clouds
// (a 5000-particle cell: 17 us on one CU; 100k particles would take ~0.3 ms), and uses one CU of
// 256.  The split form spreads each (cell, t) over S chunk workgroups in two phases:
//   phase 1  headings of the chunk, partial sums (heading, shifted heading and its square for
//            t = 0) published write-through; the (cell, t)'s last arriver sums them in chunk
//            order -> theta, the yaw statistics, and theta for phase 2;
//   phase 2  the chunk's corners and the four support-value maxima, published the same way; the
//            last arriver takes the max over chunks (order-free) -> b.
// The hand-off is the moment reduction's (gram.hpp: sc1 stores, drain, agent-scope ticket, sc1
// loads); the counters at the head of the zero-filled workspace return to zero every call.
//
// Measured as ONE launch (start tickets; ticket j ran phase 1 of chunk j, then phase 2 of chunk
// j - S after its (cell, t)'s theta, deadlock-free in any residency): no faster (C2 step graph
// 75.6 vs 75.0 us, 100k 107.2 vs 106.8; the 100k phases are f64-issue bound and the overlap
// only shares the SIMDs), so two launches (profiles/r06/README.md).
struct L4Split {
  int S;              // workgroups per (cell, t)
  int32_t *ctr;       // [2][n_cells T] arrival counters
  double *part1;      // [n_cells T][S][4]: sum yaw, sum (yaw - shift), sum (yaw - shift)^2, 0
  double *part2;      // [n_cells T][S][4]: the four maxima
  double *theta;      // [n_cells T][2]: theta, 0 (16-byte slots for the sc1 hand-off)
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
  o += ct * 2 * sizeof(double);
  return (o + 255) / 256 * 256;
}

constexpr int kL4MaxSplit = 64;  // workgroups per (cell, t): one wave holds their partials

// Particles per workgroup on the average cell (build knob): 2048 halves the 784 workgroups of
// a 100k cloud at 1024, whose dispatch alone spread over 7-12 us (profiles/r03/l4_split:
// 100k drop-in graph 113 -> 104 us, C2 shape unchanged; 4096 costs the C2 shape 5 us).
#ifndef CCMPC_L4_SPLIT_CHUNK
#define CCMPC_L4_SPLIT_CHUNK 2048
#endif
#ifndef CCMPC_L4_SPLIT_THREADS  // threads per split workgroup (build knob)
#define CCMPC_L4_SPLIT_THREADS 512
#endif
constexpr int kL4SplitThreads = CCMPC_L4_SPLIT_THREADS;

inline int l4_split_factor(int64_t n_cells, int64_t n_bound) {
  const int64_t per = n_cells > 0 ? (n_bound + n_cells - 1) / n_cells : 0;
  const int64_t S = (per + CCMPC_L4_SPLIT_CHUNK - 1) / CCMPC_L4_SPLIT_CHUNK;
  return static_cast<int>(S < 1 ? 1 : (S > kL4MaxSplit ? kL4MaxSplit : S));
}

// Workgroup sums / maxima of several values at once: each value reduced exactly as block_sum /
// block_max reduce it (the xor butterfly, then the waves in order), one barrier pair for all.
template <int K>
__device__ __forceinline__ void block_sums(double (&v)[K], double *red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
    if (lane == 0) red[k * 16 + w] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double s = 0.0;
    for (int j = 0; j < nw; ++j) s += red[k * 16 + j];
    v[k] = s;
  }
  __syncthreads();
}
__device__ __forceinline__ void block_max4(double (&v)[4], double *red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] = fmax(v[k], __shfl_xor(v[k], o, 64));
    if (lane == 0) red[k * 16 + w] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    double s = -INFINITY;
    for (int j = 0; j < nw; ++j) s = fmax(s, red[k * 16 + j]);
    v[k] = s;
  }
  __syncthreads();
}

// One (cell, t)'s geometry, as the chunk workgroups read it
struct L4Cell {
  int ct, cell, t, part;
  int64_t off, n, i0, i1;
  double o0, o1, px, py;
};
__device__ __forceinline__ L4Cell l4_cell(const L4Split &sp, int T, int chunk_id,
                                          const double *__restrict__ origin,
                                          const int64_t *__restrict__ cell_off,
                                          const int64_t *__restrict__ cell_cnt,
                                          const double *__restrict__ past_last) {
  L4Cell c;
  c.ct = chunk_id / sp.S;
  c.part = chunk_id % sp.S;
  c.cell = c.ct / T;
  c.t = c.ct % T;
  c.off = cell_off[c.cell];
  c.n = cell_cnt[c.cell];
  c.o0 = origin ? origin[2 * c.cell] : 0.0;
  c.o1 = origin ? origin[2 * c.cell + 1] : 0.0;
  c.px = past_last[2 * c.cell];
  c.py = past_last[2 * c.cell + 1];
  const int64_t chunk = (c.n + sp.S - 1) / sp.S;
  c.i0 = c.part * chunk;
  c.i1 = min(c.n, c.i0 + chunk);
  return c;
}

// particles per thread whose loads are issued together, before their arithmetic: 4 covers a
// 2048-particle chunk at 512 threads
#ifndef CCMPC_L4_PRE
#define CCMPC_L4_PRE 4
#endif
constexpr int kL4Pre = CCMPC_L4_PRE;

// A particle's step delta (step 0 from past[-1], ovehicle.py:72-76) and its position
template <typename P>
__device__ __forceinline__ void step_delta(const P *base, int64_t ld, const L4Cell &c, int64_t i,
                                           double &dx, double &dy, double *x = nullptr,
                                           double *y = nullptr) {
  const double xx = world(base, ld, 2 * c.t, i, c.o0), yy = world(base, ld, 2 * c.t + 1, i, c.o1);
  const double xp = c.t == 0 ? c.px : world(base, ld, 2 * c.t - 2, i, c.o0);
  const double yp = c.t == 0 ? c.py : world(base, ld, 2 * c.t - 1, i, c.o1);
  dx = xx - xp;
  dy = yy - yp;
  if (x) {
    *x = xx;
    *y = yy;
  }
}

// Phase 1 of one chunk: the headings' partial sums, published; the (cell, t)'s last arriver sums
// the chunks in chunk order and writes theta (also to sp.theta, for phase 2) and the yaw
// statistics.  Returns true in the last arriver (every thread), with theta in *theta_s.
template <typename P>
__device__ __forceinline__ bool l4_phase1(const P *__restrict__ pos, int64_t ld, const L4Cell &c,
                                          const L4Split &sp, double *red, int *flag,
                                          double *theta_s, double *__restrict__ out_yaw_mean,
                                          double *__restrict__ out_yaw0_var,
                                          double *__restrict__ out_yaw) {
  const P *base = pos + c.off;
  const int t = c.t;
  const double shift = (t == 0 && c.n > 0) ? heading(base, ld, 0, 0, c.o0, c.o1, c.px, c.py) : 0.0;
  double v[3] = {0.0, 0.0, 0.0};
  auto take = [&](int64_t i, double y) {
    v[0] += y;
    if (t == 0) {
      const double d = y - shift;
      v[1] += d;
      v[2] += d * d;
    }
    if (out_yaw) out_yaw[static_cast<int64_t>(t) * ld + c.off + i] = y;
  };
  // the first kL4Pre particles' loads all in flight before their atan2s (one memory round trip,
  // not one per particle), then the rest one by one; summed in particle order either way
  double dx[kL4Pre], dy[kL4Pre];
#pragma unroll
  for (int k = 0; k < kL4Pre; ++k) {
    const int64_t i = c.i0 + threadIdx.x + static_cast<int64_t>(k) * blockDim.x;
    if (i < c.i1) step_delta(base, ld, c, i, dx[k], dy[k]);
  }
#pragma unroll
  for (int k = 0; k < kL4Pre; ++k) {
    const int64_t i = c.i0 + threadIdx.x + static_cast<int64_t>(k) * blockDim.x;
    if (i < c.i1) take(i, atan2(dy[k], dx[k]));
  }
  for (int64_t i = c.i0 + threadIdx.x + static_cast<int64_t>(kL4Pre) * blockDim.x; i < c.i1;
       i += blockDim.x) {
    double ddx, ddy;
    step_delta(base, ld, c, i, ddx, ddy);
    take(i, atan2(ddy, ddx));
  }
  L4S_TS(0, 1);
  if (t == 0)
    block_sums<3>(v, red);
  else
    block_sums<1>(reinterpret_cast<double(&)[1]>(v), red);
  double *mine = sp.part1 + (static_cast<int64_t>(c.ct) * sp.S + c.part) * 4;
  const __amdgpu_buffer_rsrc_t rm = slab_rsrc(mine);
  if (threadIdx.x == 0) {
    st2_sc1(rm, 0, v[0], v[1]);
    st2_sc1(rm, 16, v[2], 0.0);
  }
  L4S_TS(0, 2);
  if (!arrive_last(sp.ctr + c.ct, sp.S, flag)) return false;
  // every chunk's partials loaded at once (thread k: chunk k), then summed in chunk order by one
  // thread from LDS: deterministic, and one L2 round trip instead of S dependent ones
  const __amdgpu_buffer_rsrc_t rp = slab_rsrc(sp.part1 + static_cast<int64_t>(c.ct) * sp.S * 4);
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
    const double nn = static_cast<double>(c.n);
    const double theta = a / nn;
    st2_sc1(slab_rsrc(sp.theta + 2 * static_cast<int64_t>(c.ct)), 0, theta, 0.0);
    *theta_s = theta;
    out_yaw_mean[c.ct] = theta;
    if (t == 0) out_yaw0_var[c.cell] = (b2 - b1 * b1 / nn) / (nn - 1.0);
  }
  __syncthreads();
  return true;
}

__device__ __forceinline__ void support_rows(double theta, double (&A)[4][2]) {
  const double ct_ = cos(theta), st_ = sin(theta);
  A[0][0] = ct_; A[0][1] = st_;
  A[1][0] = -st_; A[1][1] = ct_;
  A[2][0] = -ct_; A[2][1] = -st_;
  A[3][0] = st_; A[3][1] = -ct_;
}

// A particle's step delta and the cos / sin of its heading without the atan2: (dx, dy) times
// 1 / |(dx, dy)| from the hardware rsqrt with one Newton step (within 2 ulp of cos / sin of the
// rounded atan2); a zero step keeps sincos of atan2, whose signed-zero cases the ratio cannot
// express
__device__ __forceinline__ void heading_cs_rsq(double dx, double dy, double &S, double &C) {
  const double n2 = dx * dx + dy * dy;
  if (n2 > 0.0 && n2 < INFINITY) {
    double r = __builtin_amdgcn_rsq(n2);
    r = r * fma(-0.5 * n2 * r, r, 1.5);
    C = dx * r;
    S = dy * r;
  } else {
    sincos(atan2(dy, dx), &S, &C);
  }
}

// One particle's bbox (midlevel/util.py:109-118: corners x + 0.5 Rot(phi) [+-lon, +-lat]) into
// the running maxima of the four support values of A (util.py:171-200), A = [a; b; -a; -b],
// a = (cos theta, sin theta), b = (-sin theta, cos theta).  Over the four corners,
// max_k a . v_k = a . p + 0.5 (lon |a . Rot e_x| + lat |a . Rot e_y|) -- the corners themselves
// are not formed (within a few ulp of max_k over the rounded corner projections).  fmax is
// exact and order-free, so any split of the particles gives the same b.
__device__ __forceinline__ void support_max(double x, double y, double S, double C, double lon,
                                            double lat, double ct, double st, double (&mx)[4]) {
  const double u = ct * C + st * S;  // a . Rot e_x  ( = b . Rot e_y)
  const double w = st * C - ct * S;  // a . Rot e_y  ( = -b . Rot e_x)
  const double ap = ct * x + st * y, bp = ct * y - st * x;
  const double h0 = 0.5 * (lon * fabs(u) + lat * fabs(w));
  const double h1 = 0.5 * (lon * fabs(w) + lat * fabs(u));
  mx[0] = fmax(mx[0], ap + h0);
  mx[1] = fmax(mx[1], bp + h1);
  mx[2] = fmax(mx[2], h0 - ap);
  mx[3] = fmax(mx[3], h1 - bp);
}

// The particle's four corners into out_vertices (rows 8 t + 2 k, 8 t + 2 k + 1 at vp)
__device__ __forceinline__ void write_corners(double x, double y, double S, double C, double lon,
                                              double lat, double *__restrict__ vp, int64_t ld) {
  const double ddx[4] = {0.5 * (C * lon + S * lat), 0.5 * (C * lon - S * lat),
                         0.5 * (-C * lon - S * lat), 0.5 * (-C * lon + S * lat)};
  const double ddy[4] = {0.5 * (S * lon - C * lat), 0.5 * (S * lon + C * lat),
                         0.5 * (-S * lon + C * lat), 0.5 * (-S * lon - C * lat)};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    vp[2 * k * ld] = x + ddx[k];
    vp[(2 * k + 1) * ld] = y + ddy[k];
  }
}

// One workgroup per (cell, t) (ccmpc_l4): pass 1's headings and pass 2's support maxima in one
// launch with no hand-off; the first kL4Cache particles of each thread keep their position and
// heading cos / sin in registers between the passes.  The split form's arithmetic (rsqrt cos /
// sin, the closed-form box support); the mean heading's sum runs over the workgroup's threads in
// one order (block_sums), so it differs from the split form's chunk order by rounding only.
template <typename P>
__global__ __launch_bounds__(kL4Threads) void l4_kernel(
    const P *__restrict__ pos, int64_t ld, int T, const double *__restrict__ origin,
    const int64_t *__restrict__ cell_off, const int64_t *__restrict__ cell_cnt,
    const double *__restrict__ past_last, const double *__restrict__ bbox,
    double *__restrict__ out_A, double *__restrict__ out_b, double *__restrict__ out_yaw_mean,
    double *__restrict__ out_yaw0_var, double *__restrict__ out_yaw,
    double *__restrict__ out_vertices) {
  __shared__ double red[64];
  L4_TS(0);
  L4Split one{};
  one.S = 1;
  const L4Cell c = l4_cell(one, T, blockIdx.x, origin, cell_off, cell_cnt, past_last);
  const int t = c.t;
  const int64_t n = c.n, off = c.off;
  const double lon = bbox[2 * c.cell], lat = bbox[2 * c.cell + 1];
  const P *base = pos + off;
  const int nth = blockDim.x;

  // pass 1: headings, mean (and the t = 0 variance, shifted by the first particle's heading)
  const double shift = (t == 0 && n > 0) ? heading(base, ld, 0, 0, c.o0, c.o1, c.px, c.py) : 0.0;
  double v[3] = {0.0, 0.0, 0.0};
  auto take = [&](int64_t i, double y) {
    v[0] += y;
    if (t == 0) {
      const double d = y - shift;
      v[1] += d;
      v[2] += d * d;
    }
    if (out_yaw) out_yaw[static_cast<int64_t>(t) * ld + off + i] = y;
  };
  double xc[kL4Cache], yc[kL4Cache], dxc[kL4Cache], dyc[kL4Cache];
#pragma unroll
  for (int j = 0; j < kL4Cache; ++j) {   // every cached particle's loads first
    const int64_t i = threadIdx.x + static_cast<int64_t>(j) * nth;
    if (i < n) step_delta(base, ld, c, i, dxc[j], dyc[j], &xc[j], &yc[j]);
  }
#pragma unroll
  for (int j = 0; j < kL4Cache; ++j) {
    const int64_t i = threadIdx.x + static_cast<int64_t>(j) * nth;
#if CCMPC_L4_PROBE_NOATAN  // diagnostic build only: the transcendental's share of the kernel
    if (i < n) take(i, dyc[j] * dxc[j]);
#else
    if (i < n) take(i, atan2(dyc[j], dxc[j]));
#endif
  }
  for (int64_t i = threadIdx.x + static_cast<int64_t>(kL4Cache) * nth; i < n; i += nth) {
    double dx, dy;
    step_delta(base, ld, c, i, dx, dy);
    take(i, atan2(dy, dx));
  }
  L4_TS(1);
  if (t == 0)
    block_sums<3>(v, red);
  else
    block_sums<1>(reinterpret_cast<double(&)[1]>(v), red);
  const double nn = static_cast<double>(n);
  const double theta = v[0] / nn;
  L4_TS(2);
  if (t == 0 && threadIdx.x == 0) out_yaw0_var[c.cell] = (v[2] - v[1] * v[1] / nn) / (nn - 1.0);
  L4_TS(3);
  // pass 2: the four support values of A = [I; -I] R(theta) over every particle's box
  double A[4][2];
  support_rows(theta, A);
  double mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  double *vbase = out_vertices ? out_vertices + static_cast<int64_t>(t) * 8 * ld + off : nullptr;
#pragma unroll
  for (int j = 0; j < kL4Cache; ++j) {
    const int64_t i = threadIdx.x + static_cast<int64_t>(j) * nth;
    if (i < n) {
      double S, C;
      heading_cs_rsq(dxc[j], dyc[j], S, C);
      support_max(xc[j], yc[j], S, C, lon, lat, A[0][0], A[0][1], mx);
      if (vbase) write_corners(xc[j], yc[j], S, C, lon, lat, vbase + i, ld);
    }
  }
  for (int64_t i = threadIdx.x + static_cast<int64_t>(kL4Cache) * nth; i < n; i += nth) {
    double x, y, dx, dy, S, C;
    step_delta(base, ld, c, i, dx, dy, &x, &y);
    heading_cs_rsq(dx, dy, S, C);
    support_max(x, y, S, C, lon, lat, A[0][0], A[0][1], mx);
    if (vbase) write_corners(x, y, S, C, lon, lat, vbase + i, ld);
  }
  L4_TS(4);
  block_max4(mx, red);
  L4_TS(5);
  if (threadIdx.x == 0) {
    const int64_t ct_idx = static_cast<int64_t>(c.cell) * T + t;
    for (int r = 0; r < 4; ++r) {
      out_A[ct_idx * 8 + 2 * r] = A[r][0];
      out_A[ct_idx * 8 + 2 * r + 1] = A[r][1];
      out_b[ct_idx * 4 + r] = mx[r];
    }
    out_yaw_mean[ct_idx] = theta;
  }
}

// Phase 2 of one chunk after theta: the maxima published; the (cell, t)'s last arriver takes the
// max over chunks and writes A and b.  Returns true in the last arriver.
__device__ __forceinline__ bool l4_phase2_finish(const L4Cell &c, const L4Split &sp, int nct,
                                                 const double (&A)[4][2], double (&mx)[4],
                                                 double *red, int *flag,
                                                 double *__restrict__ out_A,
                                                 double *__restrict__ out_b) {
  block_max4(mx, red);
  double *mine = sp.part2 + (static_cast<int64_t>(c.ct) * sp.S + c.part) * 4;
  const __amdgpu_buffer_rsrc_t rm = slab_rsrc(mine);
  if (threadIdx.x == 0) {
    st2_sc1(rm, 0, mx[0], mx[1]);
    st2_sc1(rm, 16, mx[2], mx[3]);
  }
  if (!arrive_last(sp.ctr + nct + c.ct, sp.S, flag)) return false;
  // the maxima over chunks (order-free): the first wave loads them all at once and reduces
  if (threadIdx.x < 64) {
    const __amdgpu_buffer_rsrc_t rp =
        slab_rsrc(sp.part2 + static_cast<int64_t>(c.ct) * sp.S * 4);
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
        out_A[static_cast<int64_t>(c.ct) * 8 + 2 * q] = A[q][0];
        out_A[static_cast<int64_t>(c.ct) * 8 + 2 * q + 1] = A[q][1];
        out_b[static_cast<int64_t>(c.ct) * 4 + q] = b[q];
      }
  }
  return true;
}

template <typename P>
__global__ __launch_bounds__(kL4SplitThreads) void l4_pass1_kernel(
    const P *__restrict__ pos, int64_t ld, int T, const double *__restrict__ origin,
    const int64_t *__restrict__ cell_off, const int64_t *__restrict__ cell_cnt,
    const double *__restrict__ past_last, L4Split sp, double *__restrict__ out_yaw_mean,
    double *__restrict__ out_yaw0_var, double *__restrict__ out_yaw) {
  __shared__ double red[64];
  __shared__ double theta_s;
  __shared__ int flag;
  L4S_TS(0, 0);
  const L4Cell c = l4_cell(sp, T, blockIdx.x, origin, cell_off, cell_cnt, past_last);
  l4_phase1(pos, ld, c, sp, red, &flag, &theta_s, out_yaw_mean, out_yaw0_var, out_yaw);
  L4S_TS(0, 3);
}

template <typename P>
__global__ __launch_bounds__(kL4SplitThreads) void l4_pass2_kernel(
    const P *__restrict__ pos, int64_t ld, int T, const double *__restrict__ origin,
    const int64_t *__restrict__ cell_off, const int64_t *__restrict__ cell_cnt,
    const double *__restrict__ past_last, const double *__restrict__ bbox, L4Split sp,
    double *__restrict__ out_A, double *__restrict__ out_b, double *__restrict__ out_vertices) {
  __shared__ double red[64];
  __shared__ int flag;
  L4S_TS(1, 0);
  const L4Cell c = l4_cell(sp, T, blockIdx.x, origin, cell_off, cell_cnt, past_last);
  const double lon = bbox[2 * c.cell], lat = bbox[2 * c.cell + 1];
  const P *base = pos + c.off;
  double A[4][2];
  support_rows(sp.theta[2 * c.ct], A);  // written by pass 1 (an earlier launch)
  L4S_TS(1, 1);
  double mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  double *vbase = out_vertices ? out_vertices + static_cast<int64_t>(c.t) * 8 * ld + c.off : nullptr;
  auto take = [&](int64_t i, double x, double y, double dx, double dy) {
    double S, C;
    heading_cs_rsq(dx, dy, S, C);
    support_max(x, y, S, C, lon, lat, A[0][0], A[0][1], mx);
    if (vbase) write_corners(x, y, S, C, lon, lat, vbase + i, ld);
  };
  double px[kL4Pre], py[kL4Pre], dx[kL4Pre], dy[kL4Pre];  // loads first, as in phase 1
#pragma unroll
  for (int k = 0; k < kL4Pre; ++k) {
    const int64_t i = c.i0 + threadIdx.x + static_cast<int64_t>(k) * blockDim.x;
    if (i < c.i1) step_delta(base, ld, c, i, dx[k], dy[k], &px[k], &py[k]);
  }
#pragma unroll
  for (int k = 0; k < kL4Pre; ++k) {
    const int64_t i = c.i0 + threadIdx.x + static_cast<int64_t>(k) * blockDim.x;
    if (i < c.i1) take(i, px[k], py[k], dx[k], dy[k]);
  }
  for (int64_t i = c.i0 + threadIdx.x + static_cast<int64_t>(kL4Pre) * blockDim.x; i < c.i1;
       i += blockDim.x) {
    double x, y, ddx, ddy;
    step_delta(base, ld, c, i, ddx, ddy, &x, &y);
    take(i, x, y, ddx, ddy);
  }
  L4S_TS(1, 2);
  l4_phase2_finish(c, sp, gridDim.x / sp.S, A, mx, red, &flag, out_A, out_b);
  L4S_TS(1, 3);
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
  const int64_t nct = n_cells * T;
  const L4Split sp{S, reinterpret_cast<int32_t *>(w), reinterpret_cast<double *>(w + o1),
                   reinterpret_cast<double *>(w + o2), reinterpret_cast<double *>(w + o3)};
  hipStream_t s = as_stream(stream);
  const int Ti = static_cast<int>(T);
  const dim3 grid(static_cast<unsigned>(nct * S));
  auto run = [&](auto tag) {
    using P = decltype(tag);
    const P *p = static_cast<const P *>(positions);
    hipLaunchKernelGGL((l4_pass1_kernel<P>), grid, dim3(kL4SplitThreads), 0, s, p, ld, Ti, origin,
                       cell_off, cell_cnt, past_last, sp, out_yaw_mean, out_yaw0_var, out_yaw);
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
