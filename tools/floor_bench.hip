// Latency floor of a one-launch cycle on gfx950: back-to-back launch time (hipGraph of 50
// launches between HIP events) of minimal kernels at the C2 grid (86 x 256 threads):
//   empty            -- dispatch + retire only
//   chainN           -- N dependent global loads (pointer chase in a small read-only table, so
//                       L2/MALL hits after the first replay), one lane per workgroup
//   arrive           -- one 16-byte sc1 store per lane, vmcnt(0), barrier, agent atomic ticket,
//                       last arriver reads every slab back with sc1 loads (the combine hand-off)
//   chain1+arrive    -- a locate-like load, then the hand-off
// Build: hipcc -O3 --offload-arch=gfx950 floor_bench.hip -o floor_bench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned int b128_t __attribute__((__vector_size__(16)));

__global__ __launch_bounds__(256) void k_empty(int *sink) {
  if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) sink[0] = 1;
}

template <int N>
__global__ __launch_bounds__(256) void k_chain(const int *__restrict__ tab, int *sink) {
  int i = threadIdx.x & 7;
#pragma unroll
  for (int k = 0; k < N; ++k) i = tab[i];
  if (i == 12345) sink[0] = i;
}

template <bool LOCATE>
__global__ __launch_bounds__(256) void k_arrive(const int *__restrict__ tab, double *slabs,
                                               int *counter, double *out, int *sink) {
  __shared__ int flag;
  int i = 0;
  if (LOCATE) i = tab[threadIdx.x & 7];  // the item's cell table
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(slabs, 0, 0x7fffffff, 0x00020000);
  const double2 v = {static_cast<double>(blockIdx.x + i), 1.0};
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(b128_t, v), r,
                                         (blockIdx.x * 256 + threadIdx.x) * 16, 0, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = t == static_cast<int>(gridDim.x) - 1;
    if (last) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag = last;
  }
  __syncthreads();
  if (!flag) return;
  double s = 0.0;
  for (int b = 0; b < static_cast<int>(gridDim.x); b += 16) {
    double2 acc = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int bb = b + j < static_cast<int>(gridDim.x) ? b + j : b;
      const double2 x = __builtin_bit_cast(
          double2, __builtin_amdgcn_raw_buffer_load_b128(r, (bb * 256 + threadIdx.x) * 16, 0, 16));
      acc.x += x.x;
      acc.y += x.y;
    }
    s += acc.x + acc.y;
  }
  out[threadIdx.x] = s;
  (void)sink;
}

template <typename F>
static double time_us(F launch, int blocks) {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipGraph_t g;
  hipGraphExec_t ge;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 50; ++i) launch(s, blocks);
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 8; ++rep) {
    (void)hipEventRecord(a, s);
    (void)hipGraphLaunch(ge, s);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    if (rep > 0 && ms < best) best = ms;
  }
  (void)hipGraphExecDestroy(ge);
  (void)hipGraphDestroy(g);
  (void)hipStreamDestroy(s);
  return best * 1000.0 / 50.0;
}

int main() {
  int *tab, *sink, *counter;
  double *slabs, *out;
  (void)hipMalloc(&tab, 64 * sizeof(int));
  (void)hipMalloc(&sink, 64);
  (void)hipMalloc(&counter, 256);
  (void)hipMalloc(&slabs, 1024 * 256 * 16);
  (void)hipMalloc(&out, 256 * 8);
  int h[64];
  for (int i = 0; i < 64; ++i) h[i] = (i + 1) & 7;
  (void)hipMemcpy(tab, h, sizeof(h), hipMemcpyHostToDevice);
  (void)hipMemset(counter, 0, 256);
  for (int blocks : {86, 256, 700}) {
    printf("blocks %4d: empty %6.2f  chain1 %6.2f  chain2 %6.2f  chain4 %6.2f  chain8 %6.2f  "
           "arrive %6.2f  chain1+arrive %6.2f us\n",
           blocks,
           time_us([&](hipStream_t s, int n) { k_empty<<<n, 256, 0, s>>>(sink); }, blocks),
           time_us([&](hipStream_t s, int n) { k_chain<1><<<n, 256, 0, s>>>(tab, sink); }, blocks),
           time_us([&](hipStream_t s, int n) { k_chain<2><<<n, 256, 0, s>>>(tab, sink); }, blocks),
           time_us([&](hipStream_t s, int n) { k_chain<4><<<n, 256, 0, s>>>(tab, sink); }, blocks),
           time_us([&](hipStream_t s, int n) { k_chain<8><<<n, 256, 0, s>>>(tab, sink); }, blocks),
           time_us([&](hipStream_t s, int n) {
             k_arrive<false><<<n, 256, 0, s>>>(tab, slabs, counter, out, sink);
           }, blocks),
           time_us([&](hipStream_t s, int n) {
             k_arrive<true><<<n, 256, 0, s>>>(tab, slabs, counter, out, sink);
           }, blocks));
  }
  return 0;
}
