// Workgroup dispatch spread on gfx950: start timestamps (s_memrealtime, 100 MHz) of every
// workgroup of one launch, for the C2 grid (86 x 256 threads) at several LDS footprints.
// Build: hipcc -O3 --offload-arch=gfx950 dispatch_bench.hip -o dispatch_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

template <int LDS_DOUBLES>
__global__ __launch_bounds__(256) void start_kernel(unsigned long long *ts, double *sink) {
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  __shared__ double lds[LDS_DOUBLES];
  lds[threadIdx.x % LDS_DOUBLES] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) {
    ts[blockIdx.x] = t;
    if (lds[1] == 12345.0) sink[0] = 1.0;
  }
}

template <int LDS>
void run(int blocks, unsigned long long *d_ts, double *d_sink, const char *name) {
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(start_kernel<LDS>, dim3(blocks), dim3(256), 0, 0, d_ts, d_sink);
    (void)hipDeviceSynchronize();
  }
  std::vector<unsigned long long> ts(blocks);
  (void)hipMemcpy(ts.data(), d_ts, blocks * 8, hipMemcpyDeviceToHost);
  const unsigned long long t0 = *std::min_element(ts.begin(), ts.end());
  std::vector<double> rel(blocks);
  for (int i = 0; i < blocks; ++i) rel[i] = (ts[i] - t0) / 100.0;
  std::vector<double> sorted = rel;
  std::sort(sorted.begin(), sorted.end());
  printf("%-10s blocks=%4d  start spread: median %.2f us, p90 %.2f us, max %.2f us; "
         "last block %.2f us\n",
         name, blocks, sorted[blocks / 2], sorted[blocks * 9 / 10], sorted[blocks - 1],
         rel[blocks - 1]);
}

int main() {
  unsigned long long *d_ts;
  double *d_sink;
  (void)hipMalloc(&d_ts, 8192 * 8);
  (void)hipMalloc(&d_sink, 8);
  for (int blocks : {86, 256, 700}) {
    run<64>(blocks, d_ts, d_sink, "lds 0.5K");
    run<2125>(blocks, d_ts, d_sink, "lds 17K");
  }
  return 0;
}
