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
