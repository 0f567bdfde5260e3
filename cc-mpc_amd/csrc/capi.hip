// Error plumbing and version entry points of the C ABI (include/ccmpc.h).
#include <string>

#include "ccmpc_common.hpp"

namespace ccmpc {
static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }
}  // namespace ccmpc

extern "C" int ccmpc_abi_version(void) { return CCMPC_ABI_VERSION; }

extern "C" const char *ccmpc_last_error(void) { return ccmpc::g_last_error.c_str(); }

extern "C" const char *ccmpc_status_string(int status) {
  switch (status) {
    case CCMPC_OK: return "ok";
    case CCMPC_ERR_ARG: return "invalid argument";
    case CCMPC_ERR_LAUNCH: return "kernel launch failed";
    case CCMPC_ERR_WORKSPACE: return "workspace too small";
    case CCMPC_ERR_UNSUPPORTED: return "unsupported configuration";
    case CCMPC_REC_SINGULAR: return "singular matrix (LinAlgError in the reference)";
    case CCMPC_REC_NO_TANGENT: return "no real tangent (n^T Sigma n <= 0)";
    case CCMPC_REC_NONFINITE: return "non-finite slope or moment";
    case CCMPC_REC_NOT_PD: return "conditional covariance not positive definite";
    case CCMPC_REC_NOT_PSD: return "covariance not positive semi-definite (complex sqrtm)";
    default: return "unknown status";
  }
}

// Stream-ordered byte copy between host and device buffers (any direction; the runtime infers
// it from the pointers).  Lets a captured planning-step graph carry its packed H2D input copy
// and D2H output copy as graph nodes (ccmpc/step.py).
extern "C" int ccmpc_copy_async(void *dst, const void *src, size_t bytes, ccmpc_stream_t stream) {
  CCMPC_REQUIRE(dst && src, "null pointer");
  if (bytes == 0) return CCMPC_OK;
  const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, ccmpc::as_stream(stream));
  if (e != hipSuccess) {
    ccmpc::set_error(std::string("ccmpc_copy_async: ") + hipGetErrorString(e));
    return CCMPC_ERR_LAUNCH;
  }
  return CCMPC_OK;
}

// The same copy as a kernel of 16-byte lanes that reads / writes the pinned host side directly
// (host allocations are device-accessible by their host address on this platform): a graph
// kernel node instead of a memcpy node (ccmpc/step.py measures both).  bytes % 16 == 0 and
// 16-byte aligned pointers.
__global__ __launch_bounds__(256) void copy16_kernel(uint4 *__restrict__ dst,
                                                     const uint4 *__restrict__ src, size_t n) {
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x)
    dst[i] = src[i];
}

extern "C" int ccmpc_copy_kernel_async(void *dst, const void *src, size_t bytes,
                                       ccmpc_stream_t stream) {
  CCMPC_REQUIRE(dst && src, "null pointer");
  CCMPC_REQUIRE(bytes % 16 == 0 && ccmpc::aligned(dst, 16) && ccmpc::aligned(src, 16),
                "bytes and pointers must be 16-byte aligned");
  if (bytes == 0) return CCMPC_OK;
  const size_t n = bytes / 16;
  const unsigned blocks = static_cast<unsigned>(n < 64 * 256 ? (n + 255) / 256 : 64);
  hipLaunchKernelGGL(copy16_kernel, dim3(blocks), dim3(256), 0, ccmpc::as_stream(stream),
                     static_cast<uint4 *>(dst), static_cast<const uint4 *>(src), n);
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}

// One 8-byte value from device memory to a pinned host word, made visible to the host after
// everything this stream wrote before it: a system-scope release (which writes back the L2, so
// an earlier kernel's writes to host memory land first), then a system-scope store.  The host
// polls the word instead of synchronising the stream (ccmpc/step.py: a step's records are on
// the host as soon as their copy-out is, while the L4 branch of the same graph still runs).
__global__ __launch_bounds__(64) void signal_host_kernel(int64_t *dst, const int64_t *src) {
  if (threadIdx.x != 0) return;
  const int64_t v = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __atomic_thread_fence(__ATOMIC_RELEASE);  // system scope (the default)
  __hip_atomic_store(dst, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Copy-out and signal in one single-workgroup kernel: every wave copies its share, waits for
// its stores (vmcnt(0)), the workgroup meets at a barrier, then one thread makes everything the
// CU wrote visible at system scope (the release writes back this XCD's L2, where all of this
// kernel's stores went) and stores the value.  One launch less on a planning step's critical
// path than ccmpc_copy_kernel_async followed by ccmpc_signal_host.
__global__ __launch_bounds__(1024) void copy16_signal_kernel(uint4 *__restrict__ dst,
                                                             const uint4 *__restrict__ src,
                                                             size_t n, int64_t *host_word,
                                                             const int64_t *value) {
  constexpr int U = 4;  // 4 loads in flight per thread before the stores (64 KB in one pass)
  for (size_t base = 0; base < n; base += U * blockDim.x) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * blockDim.x + threadIdx.x;
      if (i < n) v[u] = src[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + u * blockDim.x + threadIdx.x;
      if (i < n) dst[i] = v[u];
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's stores have landed in L2
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t v = __hip_atomic_load(value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_thread_fence(__ATOMIC_RELEASE);  // system scope
    __hip_atomic_store(host_word, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

extern "C" int ccmpc_copy_signal_async(void *dst, const void *src, size_t bytes,
                                       int64_t *host_word, const int64_t *value,
                                       ccmpc_stream_t stream) {
  CCMPC_REQUIRE(dst && src && host_word && value, "null pointer");
  CCMPC_REQUIRE(bytes % 16 == 0 && ccmpc::aligned(dst, 16) && ccmpc::aligned(src, 16) &&
                    ccmpc::aligned(host_word, 8) && ccmpc::aligned(value, 8),
                "bytes and pointers must be 16-byte (words 8-byte) aligned");
  hipLaunchKernelGGL(copy16_signal_kernel, dim3(1), dim3(1024), 0, ccmpc::as_stream(stream),
                     static_cast<uint4 *>(dst), static_cast<const uint4 *>(src), bytes / 16,
                     host_word, value);
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}

extern "C" int ccmpc_signal_host(int64_t *host_word, const int64_t *value, ccmpc_stream_t stream) {
  CCMPC_REQUIRE(host_word && value, "null pointer");
  CCMPC_REQUIRE(ccmpc::aligned(host_word, 8) && ccmpc::aligned(value, 8),
                "pointers must be 8-byte aligned");
  hipLaunchKernelGGL(signal_host_kernel, dim3(1), dim3(64), 0, ccmpc::as_stream(stream),
                     host_word, value);
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}

// Stream capture into an executable graph, replay and release (ccmpc/step.py's planning-step
// graphs capture only this library's calls and event record / wait pairs, so they need no
// framework graph object).  Relaxed capture mode: calls of other threads are not affected.
extern "C" int ccmpc_graph_capture_begin(ccmpc_stream_t stream) {
  const hipError_t e = hipStreamBeginCapture(ccmpc::as_stream(stream), hipStreamCaptureModeRelaxed);
  if (e != hipSuccess) {
    ccmpc::set_error(std::string("ccmpc_graph_capture_begin: ") + hipGetErrorString(e));
    return CCMPC_ERR_LAUNCH;
  }
  return CCMPC_OK;
}

extern "C" int ccmpc_graph_capture_end(ccmpc_stream_t stream, void **out_exec) {
  CCMPC_REQUIRE(out_exec, "null pointer");
  *out_exec = nullptr;
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(ccmpc::as_stream(stream), &g);
  if (e == hipSuccess) {
    hipGraphExec_t x = nullptr;
    e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e == hipSuccess) *out_exec = x;
  }
  if (e != hipSuccess) {
    ccmpc::set_error(std::string("ccmpc_graph_capture_end: ") + hipGetErrorString(e));
    return CCMPC_ERR_LAUNCH;
  }
  return CCMPC_OK;
}

extern "C" int ccmpc_graph_launch(void *exec, ccmpc_stream_t stream) {
  CCMPC_REQUIRE(exec, "null graph");
  const hipError_t e = hipGraphLaunch(static_cast<hipGraphExec_t>(exec), ccmpc::as_stream(stream));
  if (e != hipSuccess) {
    ccmpc::set_error(std::string("ccmpc_graph_launch: ") + hipGetErrorString(e));
    return CCMPC_ERR_LAUNCH;
  }
  return CCMPC_OK;
}

extern "C" int ccmpc_graph_destroy(void *exec) {
  if (!exec) return CCMPC_OK;
  const hipError_t e = hipGraphExecDestroy(static_cast<hipGraphExec_t>(exec));
  if (e != hipSuccess) {
    ccmpc::set_error(std::string("ccmpc_graph_destroy: ") + hipGetErrorString(e));
    return CCMPC_ERR_LAUNCH;
  }
  return CCMPC_OK;
}

// ---- compact records for the multi-GPU exchange ---------------------------------------------
// One thread per record: the five fields the QP reads (n, rhs, side, status, t_tau) out of the
// 128-byte record into a 32-byte ccmpc_gather_rec, as two 16-byte stores.
__global__ __launch_bounds__(256) void compact_records_kernel(const unsigned char *__restrict__ rec,
                                                              int affine, int64_t n,
                                                              double4 *__restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned char *r = rec + i * 128;
  const double2 nn = *reinterpret_cast<const double2 *>(r);
  const double rhs = *reinterpret_cast<const double *>(r + (affine ? 32 : 16));
  const int4 tail = *reinterpret_cast<const int4 *>(r + 112);  // which, side, status, t_tau
  const uint32_t ss = (static_cast<uint32_t>(static_cast<uint16_t>(tail.y))) |
                      (static_cast<uint32_t>(static_cast<uint16_t>(tail.z)) << 16);
  double4 v;
  v.x = nn.x;
  v.y = nn.y;
  v.z = rhs;
  v.w = __builtin_bit_cast(double, (static_cast<uint64_t>(static_cast<uint32_t>(tail.w)) << 32) |
                                       ss);
  out[i] = v;
}

extern "C" int ccmpc_compact_records(const void *rec, int rec_kind, int64_t n_rec,
                                     ccmpc_gather_rec *out, ccmpc_stream_t stream) {
  CCMPC_REQUIRE(rec_kind == CCMPC_REC_KIND_HALFSPACE || rec_kind == CCMPC_REC_KIND_AFFINE,
                "rec_kind must be CCMPC_REC_KIND_HALFSPACE or _AFFINE");
  CCMPC_REQUIRE(n_rec >= 0, "bad n_rec");
  if (n_rec == 0) return CCMPC_OK;
  CCMPC_REQUIRE(rec && out, "null pointer");
  CCMPC_REQUIRE(ccmpc::aligned(rec, 16) && ccmpc::aligned(out, 32), "misaligned records");
  const int64_t blocks = (n_rec + 255) / 256;
  CCMPC_REQUIRE(blocks < (int64_t(1) << 31), "too many records");
  hipLaunchKernelGGL(compact_records_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                     ccmpc::as_stream(stream), static_cast<const unsigned char *>(rec),
                     rec_kind == CCMPC_REC_KIND_AFFINE ? 1 : 0, n_rec,
                     reinterpret_cast<double4 *>(out));
  CCMPC_LAUNCH_CHECK();
  return CCMPC_OK;
}
