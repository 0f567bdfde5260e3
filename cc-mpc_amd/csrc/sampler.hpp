// Sampler device helpers shared by the sampler (sampler.hip) and the fused sampler + bucketing
// kernel (sample_bucket.hip): Trajectron++'s GMM2D draw and Unicycle.dynamic step, float32 as
// torch runs them.
#pragma once
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

// One Unicycle.dynamic step.  (s0, c0) = sin / cos of the current heading, carried from the
// previous step: the heading after a turning step IS that step's phi + w dt, whose sin / cos
// it already evaluated, and a straight step keeps phi -- so each step evaluates one sincos
// (none when straight) with exactly the values of a fresh sincos_rn(phi).
__device__ __forceinline__ void unicycle_step(float &x, float &y, float &phi, float &v, float &s0,
                                              float &c0, float dphi, float a, float dt) {
  const bool straight = fabsf(dphi) <= 1e-2f;
  if (straight) {
    x = x + v * c0 * dt + (a / 2.0f) * c0 * dt * dt;
    y = y + v * s0 * dt + (a / 2.0f) * s0 * dt * dt;
  } else {
    const float w = dphi;
    const float phi1 = phi + w * dt;
    float s1, c1;
    sincos_rn(phi1, s1, c1);
    const float dsin = (s1 - s0) / w, dcos = (c1 - c0) / w;
    const float aw = a / w;
    x = x + aw * dcos + v * dsin + aw * s1 * dt;
    y = y - v * dcos + aw * dsin - aw * c1 * dt;
    phi = phi1;
    s0 = s1;
    c0 = c1;
  }
  v = v + a * dt;
}

// One GMM2D component's reparametrised draw (Trajectron++ GMM2D.rsample with one component):
// a = mu + L eps, L = [[s0, 0], [s1 rho, s1 sqrt(clamp(1 - rho^2, 1e-5, 1))]], s = exp(log s);
// the matmul row is summed before mu is added, as `mus + squeeze(L @ eps)` does.
__device__ __forceinline__ void gmm2d_action(float mu0, float mu1, float ls0, float ls1, float rho,
                                             float e0, float e1, float &dphi, float &acc) {
  const float s0 = exp_rn(ls0), s1 = exp_rn(ls1);
  const float omr2 = fminf(fmaxf(1.0f - rho * rho, 1e-5f), 1.0f);
  dphi = mu0 + s0 * e0;  // + 0 * e1: adds a signed zero, never changes s0 e0 unless it is 0
  acc = mu1 + ((s1 * rho) * e0 + (s1 * sqrtf(omr2)) * e1);
}

// Latent id of particle i by inverse CDF of its Philox uniform (DiscreteLatent.sample_p:
// numpy searchsorted(cdf, u, side='right'), clamped to the last latent); cdf in LDS.  The cdf is
// a cumulative sum (non-decreasing), so the first k with cdf[k] > u is the number of entries
// <= u: a count over independent LDS reads, not a search whose every step waits on the last
// read (the early-exit loop was a chain of up to L dependent LDS round trips per draw).
__device__ __forceinline__ int draw_latent(int64_t i, uint32_t key, uint64_t seed,
                                           const double *cdf, int n_latent) {
  const u32x4 w = philox4x32(static_cast<uint32_t>(i), 0u, key, STREAM_SAMPLER_Z, seed);
  const double u = uniform53(w.x, w.y);
  int z = 0;
#pragma unroll 8
  for (int k = 0; k < n_latent - 1; ++k) z += cdf[k] <= u ? 1 : 0;
  return z;
}

// Particle i's action at step t (GMM2D.rsample of its component): per-particle parameters at
// gmm[ov][5t + k][N] or the per-latent row of z (from the LDS copy gmm_s when staged); noise
// injected at eps_in[ov][2t + c][N] or drawn from Philox.
template <bool PP, bool EPSIN>
__device__ __forceinline__ void draw_action(int t, int64_t i, int z, int ov, int T, int n_latent,
                                            int64_t N, uint32_t key, uint64_t seed,
                                            const float *__restrict__ gmm,
                                            const float *gmm_s, bool staged,
                                            const float *__restrict__ eps_in, float &dphi,
                                            float &acc) {
  float e0, e1;
  if (EPSIN) {
    const float *ep = eps_in + static_cast<int64_t>(ov) * T * 2 * N + i;
    e0 = ep[(2 * t) * N];
    e1 = ep[(2 * t + 1) * N];
  } else {
    double e0d, e1d;
    normal_pair(static_cast<uint32_t>(i), static_cast<uint32_t>(t), key, STREAM_SAMPLER_EPS, seed,
                e0d, e1d);
    e0 = static_cast<float>(e0d);
    e1 = static_cast<float>(e1d);
  }
  const float *g = PP ? gmm + static_cast<int64_t>(ov) * T * 5 * N + i
                      : gmm + (static_cast<int64_t>(ov) * n_latent + z) * T * 5;
  float p[5];
#pragma unroll
  for (int k = 0; k < 5; ++k)
    p[k] = PP ? g[(5 * t + k) * N] : (staged ? gmm_s[(z * T + t) * 5 + k] : g[5 * t + k]);
  gmm2d_action(p[0], p[1], p[2], p[3], p[4], e0, e1, dphi, acc);
}

}  // namespace ccmpc
