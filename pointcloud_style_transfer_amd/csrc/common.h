// Shared helpers for the pcst HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "pcst.h"

namespace pcst {

// Thread-local last-error string (the only mutable global state of the library).
void set_error(const char* fmt, ...);

#define PCST_CHECK_ARG(cond, ...)                       \
  do {                                                  \
    if (!(cond)) {                                      \
      ::pcst::set_error(__VA_ARGS__);                   \
      return PCST_EINVAL;                               \
    }                                                   \
  } while (0)

#define PCST_LAUNCH_CHECK(name)                                         \
  do {                                                                  \
    hipError_t e_ = hipGetLastError();                                  \
    if (e_ != hipSuccess) {                                             \
      ::pcst::set_error("%s: launch failed: %s", name, hipGetErrorString(e_)); \
      return (int)e_;                                                   \
    }                                                                   \
  } while (0)

#define PCST_HIP(call, name)                                            \
  do {                                                                  \
    hipError_t e_ = (call);                                             \
    if (e_ != hipSuccess) {                                             \
      ::pcst::set_error("%s: %s", name, hipGetErrorString(e_));         \
      return (int)e_;                                                   \
    }                                                                   \
  } while (0)

constexpr int kWave = 64;

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Workspace carving: 256-byte aligned sub-buffers of one caller-owned allocation.
// Default poll bound of the device-side cross-stream waits (pcst_signal_wait and the kernels that
// wait for a flag themselves): ~10 s.
constexpr int kSignalPolls = 1 << 26;

struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(void* b) : base(static_cast<char*>(b)) {}
  template <typename T>
  T* take(size_t count) {
    off = (off + 255) & ~size_t(255);
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += count * sizeof(T);
    return p;
  }
  size_t bytes() const { return (off + 255) & ~size_t(255); }
};

// Exact (non-contracted) fp32 primitives for reproducing the reference's CPU rounding.
__device__ __forceinline__ float fmul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float fadd(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fsub(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ float ffma(float a, float b, float c) { return __fmaf_rn(a, b, c); }
__device__ __forceinline__ double dmul(double a, double b) { return __dmul_rn(a, b); }
__device__ __forceinline__ double dadd(double a, double b) { return __dadd_rn(a, b); }

// One element of the fused CFG + DDIM update (sampler.hip: diffusion_model.py:248-260):
//   eps = eps_u + s*(eps_c - eps_u) (eps_u given), x0 = (x - c1*eps)/c2, x0 += 0.1*(src - x0)
//   (src given), x0 = tanh(x0/1.8)*1.8, x' = c3*x0 + c4*eps.  Shared by cfg_ddim_kernel and the
//   fused kNN finish (knn.hip), so both give the same bits.
__device__ __forceinline__ float cfg_ddim_value(float x, float eps, const float* eps_u,
                                                const float* src, float scale, float c1, float c2,
                                                float c3, float c4) {
  if (eps_u) {
    const float u = *eps_u;
    eps = __fadd_rn(u, __fmul_rn(scale, __fsub_rn(eps, u)));
  }
  float x0 = __fdiv_rn(__fsub_rn(x, __fmul_rn(c1, eps)), c2);
  if (src) x0 = __fadd_rn(x0, __fmul_rn(0.1f, __fsub_rn(*src, x0)));
  x0 = __fmul_rn(tanhf(__fdiv_rn(x0, 1.8f)), 1.8f);
  return __fadd_rn(__fmul_rn(c3, x0), __fmul_rn(c4, eps));
}
__device__ __forceinline__ double dsub(double a, double b) { return __dsub_rn(a, b); }

// Unfused squared norm ((x^2 + y^2) + z^2)   (SURVEY Q2).
__device__ __forceinline__ float sqnorm3(float x, float y, float z) {
  return fadd(fadd(fmul(x, x), fmul(y, y)), fmul(z, z));
}
// K=3 sgemm dot: fma(a2,b2,fma(a1,b1,a0*b0))   (SURVEY Q1).
__device__ __forceinline__ float dot3(float a0, float a1, float a2, float b0, float b1, float b2) {
  return ffma(a2, b2, ffma(a1, b1, fmul(a0, b0)));
}

__device__ __forceinline__ unsigned long long lanemask_lt() {
  const unsigned lane = threadIdx.x & 63;
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Ordered-int encoding of float for atomic min/max (monotone for all non-NaN floats).
__device__ __forceinline__ int32_t f2ord(float f) {
  int32_t i = __float_as_int(f);
  return i >= 0 ? i : (i ^ 0x7fffffff);
}
__device__ __forceinline__ float ord2f(int32_t i) {
  return __int_as_float(i >= 0 ? i : (i ^ 0x7fffffff));
}

}  // namespace pcst
