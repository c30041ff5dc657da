// Small per-cloud reductions shared by several kernels.
#pragma once
#include "common.h"

namespace pcst {
namespace {  // internal linkage: included by several translation units

// mm[b][0..2] = ordered-int min xyz, mm[b][3..5] = max xyz.
__global__ void cloud_mm_init_kernel(int32_t* mm, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B * 6) mm[i] = (i % 6) < 3 ? INT32_MAX : INT32_MIN;
}

__global__ __launch_bounds__(256) void cloud_minmax_kernel(const float* __restrict__ pts, int N,
                                                           int32_t* __restrict__ mm) {
  const int b = blockIdx.y;
  const float* P = pts + (int64_t)b * N * 3;
  float mn0 = 3.4e38f, mn1 = 3.4e38f, mn2 = 3.4e38f, mx0 = -3.4e38f, mx1 = -3.4e38f, mx2 = -3.4e38f;
  for (int n = blockIdx.x * 256 + threadIdx.x; n < N; n += gridDim.x * 256) {
    const float x = P[n * 3], y = P[n * 3 + 1], z = P[n * 3 + 2];
    mn0 = fminf(mn0, x); mn1 = fminf(mn1, y); mn2 = fminf(mn2, z);
    mx0 = fmaxf(mx0, x); mx1 = fmaxf(mx1, y); mx2 = fmaxf(mx2, z);
  }
  for (int off = 32; off >= 1; off >>= 1) {
    mn0 = fminf(mn0, __shfl_xor(mn0, off)); mn1 = fminf(mn1, __shfl_xor(mn1, off));
    mn2 = fminf(mn2, __shfl_xor(mn2, off)); mx0 = fmaxf(mx0, __shfl_xor(mx0, off));
    mx1 = fmaxf(mx1, __shfl_xor(mx1, off)); mx2 = fmaxf(mx2, __shfl_xor(mx2, off));
  }
  if ((threadIdx.x & 63) == 0) {
    int32_t* M = mm + b * 6;
    atomicMin(&M[0], f2ord(mn0)); atomicMin(&M[1], f2ord(mn1)); atomicMin(&M[2], f2ord(mn2));
    atomicMax(&M[3], f2ord(mx0)); atomicMax(&M[4], f2ord(mx1)); atomicMax(&M[5], f2ord(mx2));
  }
}

inline void launch_cloud_minmax(const float* pts, int B, int N, int32_t* mm, hipStream_t s) {
  hipLaunchKernelGGL(cloud_mm_init_kernel, dim3((unsigned)cdiv(B * 6, 256)), dim3(256), 0, s, mm, B);
  const int gx = (int)std::min<int64_t>(cdiv(N, 256), 64);
  hipLaunchKernelGGL(cloud_minmax_kernel, dim3(gx, B), dim3(256), 0, s, pts, N, mm);
}

}  // namespace
}  // namespace pcst
