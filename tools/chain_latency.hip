// One wave's dependent-chain latencies on the chip (GPU box): the regime of the planning QP's
// active-set kernel (one wave per scene).  Per chain: ns per dependent op on the wall clock
// (s_memrealtime, 100 MHz) and shader-clock ticks per op (clock64), whose ratio is the shader
// clock the lone wave ran at.
//   hipcc -O3 --offload-arch=gfx950 tools/chain_latency.hip -o /tmp/chain_latency
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kN = 200000;

template <int WHAT>
__global__ __launch_bounds__(64) void chain(double *out, double seed, unsigned long long *t) {
  __shared__ double lds[64];
  __shared__ int idx[64];
  lds[threadIdx.x] = seed + threadIdx.x;
  idx[threadIdx.x] = (threadIdx.x * 5 + 1) & 63;
  __syncthreads();
  double v = seed + threadIdx.x;
  int k = threadIdx.x;
  const unsigned long long w0 = wall_clock64(), c0 = clock64();
  for (int i = 0; i < kN; ++i) {
    if (WHAT == 0) {
      v = fma(v, 0.999999, 1e-7);                       // dependent f64 FMA
    } else if (WHAT == 1) {
      k = idx[k];                                       // dependent LDS load
    } else if (WHAT == 2) {
      v = __builtin_amdgcn_rsq(v * v + 1.0);            // rsq + mul + add chain
    } else {
      const unsigned lo = __builtin_amdgcn_readlane(__double2loint(v), i & 63);
      const unsigned hi = __builtin_amdgcn_readlane(__double2hiint(v), i & 63);
      v = fma(__hiloint2double(hi, lo), 0.5, 1.0);      // broadcast + FMA chain
    }
  }
  const unsigned long long w1 = wall_clock64(), c1 = clock64();
  out[threadIdx.x] = v + k;
  if (threadIdx.x == 0) {
    t[0] = w1 - w0;
    t[1] = c1 - c0;
  }
}

template <int WHAT>
static void run(const char *name, double *out, unsigned long long *t) {
  hipLaunchKernelGGL(chain<WHAT>, dim3(1), dim3(64), 0, 0, out, 1.0, t);
  hipLaunchKernelGGL(chain<WHAT>, dim3(1), dim3(64), 0, 0, out, 1.0, t);
  hipDeviceSynchronize();
  unsigned long long h[2];
  hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
  const double ns = h[0] * 10.0 / kN, ticks = double(h[1]) / kN;
  printf("%-22s %7.2f ns/op  %7.2f clock64 ticks/op  -> %6.0f MHz\n", name, ns, ticks,
         ticks / ns * 1e3);
}

int main() {
  double *out;
  unsigned long long *t;
  if (hipMalloc(&out, 64 * sizeof(double)) != hipSuccess) return 1;
  if (hipMalloc(&t, 2 * sizeof(unsigned long long)) != hipSuccess) return 1;
  run<0>("f64 fma", out, t);
  run<1>("lds load", out, t);
  run<2>("f64 mul+add+rsq", out, t);
  run<3>("readlane x2 + fma", out, t);
  hipFree(out);
  hipFree(t);
  return 0;
}
