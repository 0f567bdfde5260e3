// Microbenchmark: sustained v_mfma_f64_16x16x4_f64 and v_fma_f64 rates on gfx950 (the guide
// tables have no f64 row).  One launch of 256*k workgroups x 4 waves; each wave runs ITERS
// iterations over 8 independent accumulators.  Prints cycles/MFMA/SIMD and TFLOP/s.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void mfma_loop(double *out, double a0) {
  d4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = a0 + threadIdx.x, b = a0 - threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void mfma4_loop(double *out, double a0) {
  double acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = 0;
  double a = a0 + threadIdx.x, b = a0 - threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void fma_loop(double *out, double a0) {
  double acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = i;
  double a = a0 + threadIdx.x, b = a0 - threadIdx.x;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = __builtin_fma(a, acc[i], b);
  }
  double s = 0;
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double *out;
  const int max_blocks = 256 * 8;
  hipMalloc(&out, sizeof(double) * max_blocks * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int wps : {1, 2}) {  // waves per SIMD
    const int blocks = 256 * wps;
    mfma_loop<<<blocks, 256>>>(out, 1.0);
    hipEventRecord(e0);
    mfma_loop<<<blocks, 256>>>(out, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double n_mfma = double(blocks) * 4 * ITERS * 8;
    const double flops = n_mfma * 16 * 16 * 4 * 2;
    printf("mfma_f64_16x16x4 waves/SIMD=%d: %.3f ms  %.1f TFLOP/s  %.1f cycles/MFMA/SIMD @2.4GHz\n",
           wps, ms, flops / ms / 1e9, (ms * 1e-3 * 2.4e9) / (n_mfma / 1024));
    mfma4_loop<<<blocks, 256>>>(out, 1.0);
    hipEventRecord(e0);
    mfma4_loop<<<blocks, 256>>>(out, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    {
      const double n4 = double(blocks) * 4 * ITERS * 8;
      printf("mfma_f64_4x4x4_4b waves/SIMD=%d: %.3f ms  %.1f TFLOP/s  %.1f cycles/MFMA/SIMD @2.4GHz\n",
             wps, ms, n4 * 4 * 4 * 4 * 4 * 2 / ms / 1e9, (ms * 1e-3 * 2.4e9) / (n4 / 1024));
    }
    fma_loop<<<blocks, 256>>>(out, 1.0);
    hipEventRecord(e0);
    fma_loop<<<blocks, 256>>>(out, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    const double fl = double(blocks) * 256 * ITERS * 16 * 2;
    printf("v_fma_f64 waves/SIMD=%d: %.3f ms  %.1f TFLOP/s\n", wps, ms, fl / ms / 1e9);
  }
  return 0;
}
