// Throughput of the sampler's float64 pieces on the chip (GPU box):
//   hipcc -O3 --offload-arch=gfx950 -I../cc-mpc_amd/csrc -I../include tools/f64_rate.hip -o /tmp/f64_rate
// One thread per (particle, step) pair, 800 000 pairs (C1's 100 000 particles x 8 steps), each
// piece timed alone over 20 launches: the Philox draw, the Box-Muller pair (Philox + log + sqrt +
// sincos in f64), sincos_rn, exp_rn, and the full per-latent action.
#include "../cc-mpc_amd/csrc/sampler.hpp"

#include <cstdio>

using namespace ccmpc;

template <int WHAT>
__global__ __launch_bounds__(256) void piece(float *out, uint64_t seed, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float r = 0.0f;
  if (WHAT == 0) {
    const u32x4 w = philox4x32(static_cast<uint32_t>(i), 3u, 7u, STREAM_SAMPLER_EPS, seed);
    r = static_cast<float>(w.x ^ w.y ^ w.z ^ w.w);
  } else if (WHAT == 1) {
    double a, b;
    normal_pair(static_cast<uint32_t>(i), 3u, 7u, STREAM_SAMPLER_EPS, seed, a, b);
    r = static_cast<float>(a) + static_cast<float>(b);
  } else if (WHAT == 2) {
    float s, c;
    sincos_rn(static_cast<float>(i) * 1e-5f, s, c);
    r = s + c;
  } else if (WHAT == 3) {
    r = exp_rn(static_cast<float>(i) * -1e-6f);
  } else if (WHAT == 4) {
    double u = uniform53(static_cast<uint32_t>(i) * 2654435761u, 12345u);
    r = static_cast<float>(log(1.0 - u));
  } else if (WHAT == 5) {
    double u = uniform53(static_cast<uint32_t>(i) * 2654435761u, 12345u);
    double s, c;
    sincos(2.0 * M_PI * u, &s, &c);
    r = static_cast<float>(s + c);
  }
  out[i] = r;
}

template <int WHAT>
static float time_piece(float *out, int n) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int blocks = (n + 255) / 256;
  hipLaunchKernelGGL(piece<WHAT>, dim3(blocks), dim3(256), 0, 0, out, 1ull, n);
  hipEventRecord(a, 0);
  for (int r = 0; r < 20; ++r)
    hipLaunchKernelGGL(piece<WHAT>, dim3(blocks), dim3(256), 0, 0, out, 1ull + r, n);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0.0f;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / 20.0f;
}

int main() {
  const int n = 800000;
  float *out;
  if (hipMalloc(&out, n * sizeof(float)) != hipSuccess) return 1;
  printf("us per launch of %d threads (empty-ish launch floor included)\n", n);
  printf("philox       %.2f\n", time_piece<0>(out, n));
  printf("normal_pair  %.2f\n", time_piece<1>(out, n));
  printf("log f64      %.2f\n", time_piece<4>(out, n));
  printf("sincos f64   %.2f\n", time_piece<5>(out, n));
  printf("sincos_rn    %.2f\n", time_piece<2>(out, n));
  printf("exp_rn       %.2f\n", time_piece<3>(out, n));
  hipFree(out);
  return 0;
}
