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
// the matmul row is summed before mu is added, as `mus + squeeze(L @ eps)` does.  Split in two:
// the coefficients {mu0, mu1, s0, s1 rho, s1 sqrt(.)} depend only on the parameters (per (OV,
// latent, step) in the per-latent mode: computed once per table entry when the table is staged,
// not per particle -- two float64 exp's per action fewer), then the draw; the float32 products
// are the same roundings either way.
__device__ __forceinline__ void gmm2d_coefs(float mu0, float mu1, float ls0, float ls1, float rho,
                                            float c[5]) {
  const float s0 = exp_rn(ls0), s1 = exp_rn(ls1);
  const float omr2 = fminf(fmaxf(1.0f - rho * rho, 1e-5f), 1.0f);
  c[0] = mu0;
  c[1] = mu1;
  c[2] = s0;
  c[3] = s1 * rho;
  c[4] = s1 * sqrtf(omr2);
}

__device__ __forceinline__ void gmm2d_draw(const float c[5], float e0, float e1, float &dphi,
                                           float &acc) {
  dphi = c[0] + c[2] * e0;  // + 0 * e1: adds a signed zero, never changes s0 e0 unless it is 0
  acc = c[1] + (c[3] * e0 + c[4] * e1);
}

// The per-latent parameter table gmm[L][T][5] of one OV as coefficient rows in LDS (threads
// tid, tid + nth, ... of the block).
__device__ __forceinline__ void stage_gmm_coefs(const float *__restrict__ g, int entries,
                                                float *gmm_s, int tid, int nth) {
  for (int e = tid; e < entries; e += nth) {
    float c[5];
    gmm2d_coefs(g[5 * e], g[5 * e + 1], g[5 * e + 2], g[5 * e + 3], g[5 * e + 4], c);
#pragma unroll
    for (int k = 0; k < 5; ++k) gmm_s[5 * e + k] = c[k];
  }
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

// Particle i's action at step t from its standard-normal pair (e0, e1): GMM2D.rsample of its
// component, per-particle parameters at gmm[ov][5t + k][N] or the per-latent row of z (its
// coefficient row in LDS, gmm_s, when staged by stage_gmm_coefs).
template <bool PP>
__device__ __forceinline__ void action_from_noise(int t, int64_t i, int z, int ov, int T,
                                                  int n_latent, int64_t N,
                                                  const float *__restrict__ gmm,
                                                  const float *gmm_s, bool staged, float e0,
                                                  float e1, float &dphi, float &acc) {
  const float *g = PP ? gmm + static_cast<int64_t>(ov) * T * 5 * N + i
                      : gmm + (static_cast<int64_t>(ov) * n_latent + z) * T * 5;
  float c[5];
  if (!PP && staged) {
#pragma unroll
    for (int k = 0; k < 5; ++k) c[k] = gmm_s[(z * T + t) * 5 + k];
  } else {
    float p[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) p[k] = PP ? g[(5 * t + k) * N] : g[5 * t + k];
    gmm2d_coefs(p[0], p[1], p[2], p[3], p[4], c);
  }
  gmm2d_draw(c, e0, e1, dphi, acc);
}

// Particle i's action at step t: noise injected at eps_in[ov][2t + c][N] or drawn from Philox
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
  action_from_noise<PP>(t, i, z, ov, T, n_latent, N, gmm, gmm_s, staged, e0, e1, dphi, acc);
}

}  // namespace ccmpc
