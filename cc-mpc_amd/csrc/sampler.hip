// GMM-latent particle sampler: the tail of Trajectron++'s predict path that the reference calls
// through collect/in_simulation/midlevel/prediction.py:81-86 (latent.sample_p, p_y_xz).
//
// Per particle (one lane each):
//   z ~ Categorical(p(z|x))          inverse CDF of a Philox uniform  (DiscreteLatent.sample_p)
//   for t < T:
//     a_t = mu_{z,t} + L_{z,t} eps_t, L = [[s0, 0], [s1 rho, s1 sqrt(1 - rho^2)]]  (GMM2D.rsample,
//                                                                       one component)
//     (x, y, phi, v) <- Unicycle.dynamic((x, y, phi, v), a_t)   exact integration at constant
//                                                               turn rate / acceleration
//   write (x_t, y_t) as float32, scene-relative (Trajectron++ works relative to minpos; the
//   reference adds minpos in float64 afterwards, v8ideal/__init__.py:486)
//
// The GMM parameters are per (OV, latent, step) -- the decoder's output; the learned encoder /
// GRU decoder that produce them are upstream of this boundary (absent submodule).
// Float32 arithmetic throughout, as torch runs it; the noise and the transcendentals are
// evaluated in float64 and rounded to float32.
#include "sampler.hpp"

#include <type_traits>

namespace ccmpc {

#if defined(CCMPC_PROBE) && (CCMPC_PROBE & 4)
__device__ unsigned long long g_samp_ts[kStepProbeWG * kStepProbeSlots];
#endif

// Where the draw's parameters and noise come from:
//  PP    per-particle GMM parameters gmm[o][t][5][N] (what p_y_xz emits: its GRU decoder is
//        autoregressive, so every sample carries its own parameters) instead of per (OV, latent,
//        step) parameters gmm[o][L][T][5] selected by z;
//  ZIN   latent ids injected (torch's one-hot z argmax, prediction.py:103) instead of the Philox
//        inverse CDF;
//  EPSIN noise injected eps[o][t][2][N] (torch's randn inside GMM2D.rsample) instead of Philox.
// Per-particle arrays are particle-minor, so a wave's reads of one (t, k) are one contiguous run.
//
// Two phases per block of kSampP particles: the per-step actions do not depend on the state
// (the noise and the parameters are fixed by (particle, t, z)), so kSlots waves draw the T
// actions of the block's particles in parallel into LDS (the Philox / Box-Muller / exp work),
// then one wave runs the Unicycle chain, one lane per particle -- the serial part is just the
// integration.
constexpr int kSampP = 64;       // particles per chain wave (one lane each)
constexpr int kSlots = 8;        // waves drawing actions
constexpr int kSampThreads = kSampP * kSlots;
// Chain waves per block: 1 for small clouds (many short blocks spread the serial chain phase);
// 4 for large ones (N > kSampWideN per OV): one block per 256 particles instead of 64, so a
// 100 000-particle cloud is 391 blocks of which four waves integrate, not 1563 blocks each
// running one chain wave while seven wait.  The per-particle arithmetic and Philox keys do not
// depend on the block shape: the same bits either way.
constexpr int kSampWideN = 8192;

template <bool PP, bool ZIN, bool EPSIN, int NCH>
__global__ __launch_bounds__(kSampThreads) void sample_unicycle_kernel(
    const double *__restrict__ init_state, const double *__restrict__ latent_cdf, int n_latent,
    const float *__restrict__ gmm, const int32_t *__restrict__ z_in,
    const float *__restrict__ eps_in, int64_t N, int T, float dt, uint64_t seed_arg,
    const uint64_t *__restrict__ seed_dev, uint32_t ov_base, int32_t *__restrict__ out_z,
    float *__restrict__ out_pos, int64_t ld) {
  constexpr int PB = kSampP * NCH;       // particles per block
  extern __shared__ float act[];          // (dphi, a) per (t, particle): [2][T][PB]
  __shared__ int zs[PB];
  __shared__ double cdf_s[64];           // this OV's latent CDF, one coalesced read
  __shared__ float gmm_s[PP ? 1 : 64 * 40 * 5 / 4];  // per-latent rows, staged when they fit
  CCMPC_STEP_TS(g_samp_ts, 0);
  const int ov = blockIdx.y;
  const int lane = threadIdx.x & (kSampP - 1), slot = threadIdx.x / kSampP;
  // a seed in device memory lets a captured graph draw fresh particles on every replay
  const uint64_t seed = seed_dev ? *seed_dev : seed_arg;
  const uint32_t key = ov_base + static_cast<uint32_t>(ov);  // global OV id keys the streams
  const int64_t blk0 = static_cast<int64_t>(blockIdx.x) * PB;
  if (!ZIN && threadIdx.x < n_latent)
    cdf_s[threadIdx.x] = latent_cdf[static_cast<int64_t>(ov) * n_latent + threadIdx.x];
  // the OV's per-latent parameter table (L x T x 5 floats) read once, in parallel with the CDF,
  // so the z-dependent parameter reads below are LDS reads, not a dependent global round trip
  const int gsz = n_latent * T * 5;
  const bool staged = !PP && gsz <= static_cast<int>(sizeof(gmm_s) / sizeof(float));
  if (staged)
    stage_gmm_coefs(gmm + static_cast<int64_t>(ov) * gsz, gsz / 5, gmm_s, threadIdx.x,
                    blockDim.x);
  __syncthreads();
  CCMPC_STEP_TS(g_samp_ts, 1);
  for (int q = threadIdx.x; q < PB; q += blockDim.x) {
    const int64_t i = blk0 + q;
    if (i >= N) continue;
    int z;
    if (ZIN) {
      z = z_in[static_cast<int64_t>(ov) * N + i];
      z = z < 0 ? 0 : (z >= n_latent ? n_latent - 1 : z);  // memory safety; the host validates
    } else {
      z = draw_latent(i, key, seed, cdf_s, n_latent);
    }
    zs[q] = z;
    out_z[static_cast<int64_t>(ov) * N + i] = z;
  }
  __syncthreads();
  CCMPC_STEP_TS(g_samp_ts, 2);
  // every (t, chain) pair's 64 actions: chain c = the block's particles 64 c .. 64 c + 63
  for (int u = slot; u < T * NCH; u += kSlots) {
    const int t = u / NCH, c = u - t * NCH;
    const int q = c * kSampP + lane;
    const int64_t i = blk0 + q;
    if (i < N)
      draw_action<PP, EPSIN>(t, i, zs[q], ov, T, n_latent, N, key, seed, gmm, gmm_s, staged,
                             eps_in, act[t * PB + q], act[(T + t) * PB + q]);
  }
  __syncthreads();
  CCMPC_STEP_TS(g_samp_ts, 3);
  if (slot >= NCH) return;
  const int q = slot * kSampP + lane;
  const int64_t i = blk0 + q;
  if (i >= N) return;
  const double *st = init_state + 4 * ov;
  float x = static_cast<float>(st[0]), y = static_cast<float>(st[1]);
  float phi = static_cast<float>(st[2]), v = static_cast<float>(st[3]);
  float s0, c0;
  sincos_rn(phi, s0, c0);
  float *o = out_pos + static_cast<int64_t>(ov) * ((N + 3) & ~int64_t(3)) + i;
  for (int t = 0; t < T; ++t) {
    unicycle_step(x, y, phi, v, s0, c0, act[t * PB + q], act[(T + t) * PB + q], dt);
    o[(2 * t) * ld] = x;
    o[(2 * t + 1) * ld] = y;
  }
  CCMPC_STEP_TS(g_samp_ts, 4);
}

template <bool PP, bool ZIN, bool EPSIN>
static hipError_t launch_sampler(int64_t n_ov, hipStream_t s, const double *init_state,
                                 const double *latent_cdf, int n_latent, const float *gmm,
                                 const int32_t *z_in, const float *eps_in, int64_t N, int T,
                                 float dt, uint64_t seed, const uint64_t *seed_dev,
                                 uint32_t ov_base, int32_t *out_z, float *out_pos, int64_t ld) {
  auto go = [&](auto nch) -> hipError_t {
    constexpr int NCH = decltype(nch)::value, PB = kSampP * NCH;
    const dim3 grid(static_cast<unsigned>((N + PB - 1) / PB), static_cast<unsigned>(n_ov));
    const size_t lds = sizeof(float) * 2 * T * PB;
    if (lds > 48 * 1024) {
      // long horizons on wide blocks: allow the larger dynamic LDS.  The attribute is per
      // device, and cheap to set, so it is set on every such launch (the current device may
      // change between calls) and a failure is reported here rather than as a launch error
      const hipError_t e = hipFuncSetAttribute(
          reinterpret_cast<const void *>(&sample_unicycle_kernel<PP, ZIN, EPSIN, NCH>),
          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((sample_unicycle_kernel<PP, ZIN, EPSIN, NCH>), grid, dim3(kSampThreads),
                       lds, s, init_state, latent_cdf, n_latent, gmm, z_in, eps_in, N, T, dt,
                       seed, seed_dev, ov_base, out_z, out_pos, ld);
    return hipSuccess;
  };
  if (N > kSampWideN) return go(std::integral_constant<int, 4>{});
  return go(std::integral_constant<int, 1>{});
}

}  // namespace ccmpc

using namespace ccmpc;

#if defined(CCMPC_PROBE) && (CCMPC_PROBE & 4)
// slots: 0 start, 1 tables staged, 2 z drawn, 3 actions drawn, 4 chain done (tools/probe_step.py)
extern "C" int ccmpc_probe_sampler_timestamps(void *host, int reset) {
  const size_t bytes = sizeof(g_samp_ts);
  if (reset) {
    static unsigned long long zeros[kStepProbeWG * kStepProbeSlots];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_samp_ts), zeros, bytes) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_samp_ts), bytes) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int ccmpc_sample_unicycle_ex(const double *init_state, const double *latent_cdf,
                                        int64_t n_latent, const float *gmm, int32_t gmm_layout,
                                        const int32_t *z_in, const float *eps_in, int64_t n_ov,
                                        int64_t N, int64_t T, double dt, uint64_t seed,
                                        const uint64_t *seed_dev, int64_t ov_base,
                                        int32_t *out_z, float *out_pos, int64_t ld,
                                        ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T >= 1 && T <= 40, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_latent >= 1 && n_latent <= 64, "n_latent must be in [1, 64]");
  CCMPC_REQUIRE(n_ov >= 0 && n_ov < 65536, "bad n_ov");
  CCMPC_REQUIRE(N >= 1 && N < (int64_t(1) << 32), "bad N");
  CCMPC_REQUIRE(ov_base >= 0 && ov_base + n_ov <= (int64_t(1) << 32), "bad ov_base");
  CCMPC_REQUIRE(gmm_layout == CCMPC_GMM_PER_LATENT || gmm_layout == CCMPC_GMM_PER_PARTICLE,
                "bad gmm_layout");
  const bool pp = gmm_layout == CCMPC_GMM_PER_PARTICLE;
  // per-particle parameters come from a decoder conditioned on each sample's z: z is an input
  CCMPC_REQUIRE(!pp || z_in, "per-particle GMM parameters need the injected z_in");
  CCMPC_REQUIRE(pp || n_ov * n_latent * T * 5 < (int64_t(1) << 40), "gmm too large");
  CCMPC_REQUIRE(!pp || n_ov * T * 5 * N < (int64_t(1) << 40), "gmm too large");
  if (n_ov == 0) return CCMPC_OK;
  CCMPC_REQUIRE(init_state && gmm && out_z && out_pos, "null pointer");
  CCMPC_REQUIRE(z_in || latent_cdf, "latent_cdf is needed when z is drawn here");
  CCMPC_REQUIRE(ld >= n_ov * ((N + 3) & ~int64_t(3)), "ld too small");
  hipStream_t s = as_stream(stream);
  const int L = static_cast<int>(n_latent), Ti = static_cast<int>(T);
  const float fdt = static_cast<float>(dt);
  const uint32_t base = static_cast<uint32_t>(ov_base);
  hipError_t attr = hipSuccess;
#define CCMPC_SAMPLER(PP, ZIN, EPSIN)                                                        \
  attr = launch_sampler<PP, ZIN, EPSIN>(n_ov, s, init_state, latent_cdf, L, gmm, z_in, eps_in, \
                                        N, Ti, fdt, seed, seed_dev, base, out_z, out_pos, ld)
  const int mode = (pp ? 4 : 0) | (z_in ? 2 : 0) | (eps_in ? 1 : 0);
  switch (mode) {
    case 0: CCMPC_SAMPLER(false, false, false); break;
    case 1: CCMPC_SAMPLER(false, false, true); break;
    case 2: CCMPC_SAMPLER(false, true, false); break;
    case 3: CCMPC_SAMPLER(false, true, true); break;
    case 6: CCMPC_SAMPLER(true, true, false); break;
    default: CCMPC_SAMPLER(true, true, true); break;
  }
#undef CCMPC_SAMPLER
  if (attr != hipSuccess) {
    set_error(std::string(__func__) + ": hipFuncSetAttribute(MaxDynamicSharedMemorySize) "
              "failed: " + hipGetErrorString(attr));
    return CCMPC_ERR_LAUNCH;
  }
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}

extern "C" int ccmpc_sample_unicycle(const double *init_state, const double *latent_cdf,
                                     int64_t n_latent, const float *gmm, int64_t n_ov, int64_t N,
                                     int64_t T, double dt, uint64_t seed, int64_t ov_base,
                                     int32_t *out_z, float *out_pos, int64_t ld,
                                     ccmpc_stream_t stream) {
  CCMPC_REQUIRE(latent_cdf, "null pointer");
  return ccmpc_sample_unicycle_ex(init_state, latent_cdf, n_latent, gmm, CCMPC_GMM_PER_LATENT,
                                  nullptr, nullptr, n_ov, N, T, dt, seed, nullptr, ov_base, out_z,
                                  out_pos, ld, stream);
}
