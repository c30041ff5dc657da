// Microbenchmark (experiments only): the noise-MLP solo kernel's inner pattern in isolation.
// 256 work-groups (one per CU) of W waves loop over NSP superparts of 64 fragments held in LDS;
// per fragment a wave reads the fragment (KD ahead, counted waits) and issues 2
// v_mfma_f32_16x16x32_bf16 (one per column block).  Variants (argv): W = 4 (1 wave/SIMD) or 8 (2),
// bar = s_barrier every superpart (0/1), lds = fragment reads from LDS (0: from registers),
// acc = accumulator pattern (0: two chains like a W1 chunk, 1: 32 accumulators like W2).
// Prints ns per superpart per SIMD and the MFMA-bound figure (16 cycles per MFMA).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <int I, int N, class F>
__device__ __forceinline__ void sfor(F& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}
__device__ __forceinline__ bf16x8 rd(uint32_t addr, int off) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
  return v;
}
template <int N>
__device__ __forceinline__ void wt(bf16x8& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "n"(N));
}

template <int KD, bool BAR, bool LDS, int ACC, int NCB = 2, int DMA = 0>
__global__ __launch_bounds__(512) void probe(float* out, int nsp, long long* cyc, const char* src) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 65536 / 4; i += blockDim.x)
    reinterpret_cast<float*>(smem)[i] = (float)((i * 2654435761u) >> 20) * 1e-6f;
  __syncthreads();
  const uint32_t a = (uint32_t)(uintptr_t)smem + lane * 16;
  bf16x8 b0, b1;
  for (int j = 0; j < 8; ++j) {
    b0[j] = (__bf16)(0.01f * (lane + j));
    b1[j] = (__bf16)(0.02f * (lane - j));
  }
  f32x4 acc[32];
  for (int i = 0; i < 32; ++i) acc[i] = f32x4{0, 0, 0, 0};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < nsp; ++s) {
    bf16x8 w[KD + 1];
    auto pro = [&](auto fc) {
      constexpr int f = decltype(fc)::value;
      w[f] = rd(a, f * 1024);
    };
    if (LDS) sfor<0, KD>(pro);
    else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      for (int i = 0; i <= KD; ++i) w[i] = b0 + (bf16x8)(__bf16)(float)i;
    }
    auto it = [&](auto fc) {
      constexpr int f = decltype(fc)::value;
      if constexpr (LDS) {
        if constexpr (f + KD < 64) w[(f + KD) % (KD + 1)] = rd(a, (f + KD) * 1024);
        constexpr int after = (63 - f) < KD ? (63 - f) : KD;
        wt<after>(w[f % (KD + 1)]);
      }
      if constexpr (DMA && f % 4 == 1 && f < 32) {  // 8 pieces per wave into the other 64 KiB
        const int wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
        const int off = (wid * 8 + f / 4) * 1024 * 8 / nw;
        __builtin_amdgcn_global_load_lds((const void*)(src + (int64_t)(s % 55) * 65536 + off + lane * 16),
                                         (__attribute__((address_space(3))) void*)(smem + 65536 + off), 16, 0, 0);
      }
      if constexpr (NCB == 4) {
        constexpr int c = (f / 8) % 2;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          acc[c * 4 + cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[f % (KD + 1)], cb & 1 ? b1 : b0, acc[c * 4 + cb], 0, 0, 0);
      } else if constexpr (ACC == 0) {
        constexpr int c = (f / 8) % 2;
        acc[c * 2 + 0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[f % (KD + 1)], b0, acc[c * 2 + 0], 0, 0, 0);
        acc[c * 2 + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[f % (KD + 1)], b1, acc[c * 2 + 1], 0, 0, 0);
      } else {
        constexpr int r = f % 16;
        acc[r * 2 + 0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[f % (KD + 1)], b0, acc[r * 2 + 0], 0, 0, 0);
        acc[r * 2 + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[f % (KD + 1)], b1, acc[r * 2 + 1], 0, 0, 0);
      }
    };
    sfor<0, 64>(it);
    if (BAR) {
      if (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  f32x4 sum = acc[0];
  for (int i = 1; i < 32; ++i) sum += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = sum[0] + sum[1] + sum[2] + sum[3];
  if (lane == 0) cyc[blockIdx.x * 8 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int KD, bool BAR, bool LDS, int ACC, int NCB = 2, int DMA = 0>
static void run(int W, int nsp) {
  static char* src = nullptr;
  if (!src) {
    hipMalloc(&src, 55 * 65536);
    hipMemset(src, 0, 55 * 65536);
  }
  float* out;
  long long* cyc;
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&cyc, 256 * 8 * 8);
  hipMemset(cyc, 0, 256 * 8 * 8);
  auto k = probe<KD, BAR, LDS, ACC, NCB, DMA>;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(256), dim3(W * 64), 131072, 0, out, nsp, cyc, src);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, dim3(256), dim3(W * 64), 131072, 0, out, nsp, cyc, src);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long h[256 * 8];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double c = 0;
  int n = 0;
  for (int i = 0; i < 256 * 8; ++i)
    if (h[i]) c += h[i], ++n;
  c /= n;
  const double mfma_per_simd_sp = 64.0 * NCB * W / 4;   // NCB MFMAs x 64 fragments per wave
  const double ns_sp = ms * 1e6 / 10 / nsp;
  printf("W=%d ncb=%d kd=%d bar=%d lds=%d acc=%d dma=%d: %.1f ns/superpart, %.0f cycles/superpart/wave (MFMA-bound %.0f), "
         "%.1f TFLOP/s chip\n", W, NCB, KD, BAR, LDS, ACC, DMA, ns_sp, c / nsp, 16.0 * mfma_per_simd_sp,
         256.0 * 4 * mfma_per_simd_sp * 16384.0 / (ns_sp * 1e-9) / 1e12);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  const int nsp = 200;
  run<3, true, false, 0, 2>(8, nsp);  // warm-up line (first config runs slow)
  for (int rep = 0; rep < 2; ++rep) {
    run<3, true, true, 0, 2, 0>(8, nsp);
    run<3, true, true, 0, 2, 1>(8, nsp);
    run<6, true, true, 0, 2, 1>(8, nsp);
    run<3, true, true, 1, 2, 1>(8, nsp);
    run<3, true, true, 0, 4, 0>(4, nsp);
    run<3, true, true, 0, 4, 1>(4, nsp);
    run<6, true, true, 0, 4, 1>(4, nsp);
    run<3, true, false, 0, 2, 0>(8, nsp);
    run<3, true, false, 0, 4, 0>(4, nsp);
  }
  return 0;
}
