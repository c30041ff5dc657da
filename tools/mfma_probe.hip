// MFMA issue-rate probe (perf experiment, not product code): how many cycles does one
// v_mfma_f32_32x32x16_bf16 take on MI355X in the patterns the noise MLP uses?
//   mode 0: one accumulator chain, A/B in registers
//   mode 1: four independent accumulators
//   mode 2: one chain, A fragment read from LDS per MFMA (ds_read_b128, 4 reads in flight)
//   mode 3: like 2, plus a 16-value fp32 -> bf16 epilogue every 16 MFMAs
//   mode 4: one LDS A read feeds 2 MFMAs (two column blocks, two chains)
//   mode 5: one LDS A read feeds 4 MFMAs
//   mode 6: like 2 with the reads software-pipelined 8 fragments ahead
// Grid: 256 workgroups x (64 * waves_per_simd * 4) threads; prints ns and cycles per MFMA
// per SIMD using the measured time and s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

template <int MODE>
__global__ void probe(int iters, float* out, long long* cyc) {
  __shared__ __attribute__((aligned(16))) char lds[32768];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 32768 / 4; i += blockDim.x) reinterpret_cast<float*>(lds)[i] = 0.001f * (i & 127);
  __syncthreads();
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(0.01f * (lane + j)); b[j] = (__bf16)(0.02f * (lane - j)); }
  f32x16 c0 = f32x16{}, c1 = f32x16{}, c2 = f32x16{}, c3 = f32x16{};
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {
#pragma unroll
      for (int k = 0; k < 16; ++k) c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    } else if (MODE == 1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
      }
    } else if (MODE == 4 || MODE == 5) {
      const bf16x8* F = reinterpret_cast<const bf16x8*>(lds) + lane;
#pragma unroll
      for (int k = 0; k < (MODE == 4 ? 8 : 4); ++k) {
        const bf16x8 fa = F[((it * 16 + k) & 31) * 64];
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, a, c1, 0, 0, 0);
        if (MODE == 5) {
          c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, b, c2, 0, 0, 0);
          c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, a, c3, 0, 0, 0);
        }
      }
    } else if (MODE == 6) {
      const bf16x8* F = reinterpret_cast<const bf16x8*>(lds) + lane;
      bf16x8 q[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) q[k] = F[((it * 16 + k) & 31) * 64];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const bf16x8 fa = q[k & 7];
        if (k + 8 < 16) q[k & 7] = F[((it * 16 + k + 8) & 31) * 64];
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, b, c0, 0, 0, 0);
      }
    } else {
      const bf16x8* F = reinterpret_cast<const bf16x8*>(lds) + lane;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const bf16x8 fa = F[((it * 16 + k) & 31) * 64];
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, b, c0, 0, 0, 0);
      }
      if (MODE == 3) {
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = (__bf16)fmaxf(c0[j] * 1e-3f, 0.0f);
      }
    }
  }
  long long t1 = clock64();
  float s = 0.f;
  for (int j = 0; j < 16; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
  if (s == 12345.f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main(int argc, char** argv) {
  const int wps = argc > 1 ? atoi(argv[1]) : 1;   // waves per SIMD
  const int iters = 2000;
  float* out;
  long long* cyc;
  hipMalloc(&out, 256 * 1024 * 4);
  hipMalloc(&cyc, 8);
  auto run = [&](auto kern, const char* name) {
    hipLaunchKernelGGL(kern, dim3(256), dim3(256 * wps), 0, 0, 10, out, cyc);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(256), dim3(256 * wps), 0, 0, iters, out, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double mf = (double)iters * 16 * wps;  // MFMAs per SIMD
    printf("%-28s waves/SIMD %d: %.3f ms  %.2f ns/MFMA/SIMD  %.1f clock64 ticks/MFMA/SIMD  %.0f TFLOP/s\n",
           name, wps, ms, ms * 1e6 / mf, (double)c / (iters * 16) , 256.0 * 4 * mf * 32768 / (ms * 1e-3) / 1e12);
  };
  run(probe<0>, "one chain, regs");
  run(probe<1>, "four chains, regs");
  run(probe<2>, "one chain, LDS A");
  run(probe<3>, "LDS A + epilogue/16");
  run(probe<4>, "LDS A per 2 MFMA");
  run(probe<5>, "LDS A per 4 MFMA");
  run(probe<6>, "LDS A, 8 ahead");
  return 0;
}
