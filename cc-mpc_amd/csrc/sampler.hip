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
#include "ccmpc_common.hpp"

namespace ccmpc {

// float32 sin/cos/exp evaluated in float64 and rounded once: correctly rounded in practice, so
// the result does not depend on which libm computes it (the oracle does the same), and the
// (sin(phi + w dt) - sin(phi)) / w cancellation cannot amplify a 1-ulp libm difference.
__device__ __forceinline__ void sincos_rn(float a, float &s, float &c) {
  double sd, cd;
  sincos(static_cast<double>(a), &sd, &cd);
  s = static_cast<float>(sd);
  c = static_cast<float>(cd);
}

__device__ __forceinline__ float exp_rn(float a) {
  return static_cast<float>(exp(static_cast<double>(a)));
}

__device__ __forceinline__ void unicycle_step(float &x, float &y, float &phi, float &v, float dphi,
                                              float a, float dt) {
  const bool straight = fabsf(dphi) <= 1e-2f;
  const float w = straight ? 1.0f : dphi;
  const float phi1 = phi + w * dt;
  float s0, c0, s1, c1;
  sincos_rn(phi, s0, c0);
  sincos_rn(phi1, s1, c1);
  if (straight) {
    x = x + v * c0 * dt + (a / 2.0f) * c0 * dt * dt;
    y = y + v * s0 * dt + (a / 2.0f) * s0 * dt * dt;
  } else {
    const float dsin = (s1 - s0) / w, dcos = (c1 - c0) / w;
    const float aw = a / w;
    x = x + aw * dcos + v * dsin + aw * s1 * dt;
    y = y - v * dcos + aw * dsin - aw * c1 * dt;
    phi = phi1;
  }
  v = v + a * dt;
}

__global__ __launch_bounds__(256) void sample_unicycle_kernel(
    const double *__restrict__ init_state, const double *__restrict__ latent_cdf, int n_latent,
    const float *__restrict__ gmm, int64_t N, int T, float dt, uint64_t seed, uint32_t ov_base,
    int32_t *__restrict__ out_z, float *__restrict__ out_pos, int64_t ld) {
  const int ov = blockIdx.y;
  const uint32_t key = ov_base + static_cast<uint32_t>(ov);  // global OV id keys the streams
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const double *cdf = latent_cdf + static_cast<int64_t>(ov) * n_latent;
  const u32x4 w = philox4x32(static_cast<uint32_t>(i), 0u, key, STREAM_SAMPLER_Z, seed);
  const double u = uniform53(w.x, w.y);
  int z = n_latent - 1;
  for (int k = 0; k < n_latent; ++k) {
    if (cdf[k] > u) {  // numpy searchsorted(cdf, u, side='right')
      z = k;
      break;
    }
  }
  out_z[static_cast<int64_t>(ov) * N + i] = z;
  const double *st = init_state + 4 * ov;
  float x = static_cast<float>(st[0]), y = static_cast<float>(st[1]);
  float phi = static_cast<float>(st[2]), v = static_cast<float>(st[3]);
  const float *g = gmm + (static_cast<int64_t>(ov) * n_latent + z) * T * 5;
  float *o = out_pos + static_cast<int64_t>(ov) * ((N + 3) & ~int64_t(3)) + i;
  for (int t = 0; t < T; ++t) {
    double e0d, e1d;
    normal_pair(static_cast<uint32_t>(i), static_cast<uint32_t>(t), key, STREAM_SAMPLER_EPS, seed,
                e0d, e1d);
    const float e0 = static_cast<float>(e0d), e1 = static_cast<float>(e1d);
    const float mu0 = g[5 * t], mu1 = g[5 * t + 1];
    const float s0 = exp_rn(g[5 * t + 2]), s1 = exp_rn(g[5 * t + 3]), rho = g[5 * t + 4];
    const float dphi = mu0 + s0 * e0;
    const float acc = (mu1 + (s1 * rho) * e0) + (s1 * sqrtf(1.0f - rho * rho)) * e1;
    unicycle_step(x, y, phi, v, dphi, acc, dt);
    o[(2 * t) * ld] = x;
    o[(2 * t + 1) * ld] = y;
  }
}

}  // namespace ccmpc

using namespace ccmpc;

extern "C" int ccmpc_sample_unicycle(const double *init_state, const double *latent_cdf,
                                     int64_t n_latent, const float *gmm, int64_t n_ov, int64_t N,
                                     int64_t T, double dt, uint64_t seed, int64_t ov_base,
                                     int32_t *out_z, float *out_pos, int64_t ld,
                                     ccmpc_stream_t stream) {
  CCMPC_REQUIRE(T >= 1 && T <= 40, "T must be in [1, 40]");
  CCMPC_REQUIRE(n_latent >= 1 && n_latent <= 64, "n_latent must be in [1, 64]");
  CCMPC_REQUIRE(n_ov >= 0 && n_ov < 65536, "bad n_ov");
  CCMPC_REQUIRE(N >= 1 && N < (int64_t(1) << 32), "bad N");
  CCMPC_REQUIRE(ov_base >= 0 && ov_base + n_ov <= (int64_t(1) << 32), "bad ov_base");
  if (n_ov == 0) return CCMPC_OK;
  CCMPC_REQUIRE(init_state && latent_cdf && gmm && out_z && out_pos, "null pointer");
  CCMPC_REQUIRE(ld >= n_ov * ((N + 3) & ~int64_t(3)), "ld too small");
  const dim3 grid(static_cast<unsigned>((N + 255) / 256), static_cast<unsigned>(n_ov));
  hipLaunchKernelGGL(sample_unicycle_kernel, grid, dim3(256), 0, as_stream(stream), init_state,
                     latent_cdf, static_cast<int>(n_latent), gmm, N, static_cast<int>(T),
                     static_cast<float>(dt), seed, static_cast<uint32_t>(ov_base), out_z, out_pos,
                     ld);
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}
