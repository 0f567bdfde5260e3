// Shared device helpers for libccmpc (gfx950 / CDNA4).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <string>

#include "ccmpc.h"

namespace ccmpc {

// ---- host-side error plumbing --------------------------------------------------------------
void set_error(const std::string &msg);

#define CCMPC_REQUIRE(cond, msg)                                                              \
  do {                                                                                         \
    if (!(cond)) {                                                                             \
      ::ccmpc::set_error(std::string(__func__) + ": " + (msg));                                \
      return CCMPC_ERR_ARG;                                                                    \
    }                                                                                          \
  } while (0)

#define CCMPC_LAUNCH_CHECK()                                                                   \
  do {                                                                                         \
    hipError_t e_ = hipGetLastError();                                                         \
    if (e_ != hipSuccess) {                                                                    \
      ::ccmpc::set_error(std::string(__func__) + ": launch failed: " + hipGetErrorString(e_)); \
      return CCMPC_ERR_LAUNCH;                                                                 \
    }                                                                                          \
  } while (0)

inline hipStream_t as_stream(ccmpc_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline bool aligned(const void *p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

constexpr int kWave = 64;  // CDNA wavefront

// ---- Philox4x32-10 (mirrors oracle/philox.py) ----------------------------------------------
#ifndef CCMPC_PHILOX_MAD
#define CCMPC_PHILOX_MAD 1
#endif
constexpr uint32_t STREAM_IDEAL_Z = 0x1DEA0001u;
constexpr uint32_t STREAM_IDEAL_X0 = 0x1DEA0002u;
constexpr uint32_t STREAM_SAMPLER_EPS = 0x5A4D0001u;
constexpr uint32_t STREAM_SAMPLER_Z = 0x5A4D0002u;

struct u32x4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint64_t seed) {
  uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
#if CCMPC_PHILOX_MAD
    // one 32x32->64 product per multiplier (v_mad_u64_u32) instead of separate lo / hi
    // multiplies: both are quarter-rate, so this halves the integer multiply issue
    const uint64_t p0 = static_cast<uint64_t>(0xD2511F53u) * c0;
    const uint64_t p1 = static_cast<uint64_t>(0xCD9E8D57u) * c2;
    const uint32_t n0 = static_cast<uint32_t>(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = static_cast<uint32_t>(p0 >> 32) ^ c3 ^ k1;
    c0 = n0;
    c1 = static_cast<uint32_t>(p1);
    c2 = n2;
    c3 = static_cast<uint32_t>(p0);
#else
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
#endif
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}

__device__ __forceinline__ double uniform53(uint32_t a, uint32_t b) {
  return (static_cast<double>(a >> 5) * 67108864.0 + static_cast<double>(b >> 6)) *
         (1.0 / 9007199254740992.0);
}

// Box-Muller pair, float64 (oracle/philox.py normal_pair), in two halves a caller may run in
// separate passes: the radius sqrt(-2 log u1) and the angle's uniform, then the sin / cos.  A
// loop of whole pairs keeps both halves' polynomial coefficients in registers (the compiler
// hoists them out of the loop); two passes keep only one set live at a time.
__device__ __forceinline__ void normal_radius(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint64_t seed, double &r, double &u2) {
  const u32x4 w = philox4x32(c0, c1, c2, c3, seed);
  const double u1 = 1.0 - uniform53(w.x, w.y);
  u2 = uniform53(w.z, w.w);
  r = sqrt(-2.0 * log(u1));
}
__device__ __forceinline__ void normal_angle(double r, double u2, double &z0, double &z1) {
  double s, c;
  sincos(2.0 * M_PI * u2, &s, &c);
  z0 = r * c;
  z1 = r * s;
}
__device__ __forceinline__ void normal_pair(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint64_t seed, double &z0, double &z1) {
  double r, u2;
  normal_radius(c0, c1, c2, c3, seed, r, u2);
  normal_angle(r, u2, z0, z1);
}

// ---- diagnostic timestamps (PROBE=4 builds only) -------------------------------------------
// CCMPC_STEP_TS(table, k): workgroup (blockIdx.y * gridDim.x + blockIdx.x)'s slot k of a
// [4096][8] table gets s_memrealtime (100 MHz, one clock for every kernel of a step, so the
// gaps between kernels show).  Each file defines its own table and reader.
constexpr int kStepProbeWG = 4096, kStepProbeSlots = 8;
#if defined(CCMPC_PROBE) && (CCMPC_PROBE & 4)
#define CCMPC_STEP_TS(tab, k)                                                                 \
  do {                                                                                        \
    const unsigned wg_ = blockIdx.y * gridDim.x + blockIdx.x;                                 \
    if (threadIdx.x == 0 && wg_ < ::ccmpc::kStepProbeWG)                                      \
      (tab)[wg_ * ::ccmpc::kStepProbeSlots + (k)] = __builtin_amdgcn_s_memrealtime();         \
  } while (0)
#else
#define CCMPC_STEP_TS(tab, k) \
  do {                        \
  } while (0)
#endif

// ---- 2x2 symmetric helpers -----------------------------------------------------------------
struct Sym2 {
  double a, b, c;  // [[a, b], [b, c]]
};

}  // namespace ccmpc
