// bf16-MFMA GEMMs of the training path under autocast (trainer.py:81-106 runs the model inside
// torch.autocast; the reference's CUDA autocast computes its Linear layers in half precision
// with fp32 accumulation).  Operands arrive as fp32 tensors and are rounded to bf16 while they
// are staged into LDS; accumulation, bias, ReLU and outputs stay fp32.
//
//   gemm_nt:  C[m, o] = act(scale[o] * sum_k A[m, k] B[o, k] + shift[o])    forward / dX
//   wgrad:    C[o, i] = sum_m dZ[m, o] X[m, i]  (+ db[o] = sum_m dZ[m, o])  weight gradient
//
// Tile 128 x 128 per 256-thread workgroup: 2 x 2 waves, each 64 x 64 = 2 x 2 blocks of
// v_mfma_f32_32x32x16_bf16 (or _f16: the file is compiled twice, see train_mlp.hip).  K is staged 32 deep; an LDS row holds the 32 k-values of one
// output row or column as bf16 (64 B) padded to 80 B, so the 16-byte fragment reads of
// consecutive rows fall on distinct banks.  The weight gradient splits its reduction over the
// M rows into chunks (as csrc/sa_mlp.hip's exact-f32 wgrad) and combines them in order.
#include "common.h"

#include "train_h16.h"

#ifndef PCST_H16_F16
#define PCST_H16_F16 0
#endif

namespace pcst {
namespace PCST_H16_NS {

#if PCST_H16_F16
typedef _Float16 h16;
#else
typedef __bf16 h16;
#endif

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) h16 h16x8;
__device__ __forceinline__ auto mfma32_h16(h16x8 a, h16x8 b, __attribute__((ext_vector_type(16))) float c) {
#if PCST_H16_F16
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
#endif
}
typedef __attribute__((ext_vector_type(4))) h16 h16x4;

constexpr int kGT = 128, kGK = 32, kGLd = 40;  // tile, k slice, LDS row (bf16 elements)

__device__ __forceinline__ int grow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// one 32-deep k slice: 2 x 2 blocks x 2 k-steps of 32x32x16
__device__ __forceinline__ void mma_slice(const h16 (*As)[kGLd], const h16 (*Bs)[kGLd],
                                          int wr, int wc, int l32, int h, f32x16 (&acc)[2][2]) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    h16x8 a[2], b[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      a[t] = *reinterpret_cast<const h16x8*>(&As[wr * 64 + t * 32 + l32][ks * 16 + h * 8]);
      b[t] = *reinterpret_cast<const h16x8*>(&Bs[wc * 64 + t * 32 + l32][ks * 16 + h * 8]);
    }
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int bn = 0; bn < 2; ++bn)
        acc[bm][bn] = mfma32_h16(a[bm], b[bn], acc[bm][bn]);
  }
}

// stage rows [r0, r0+128) x k [k0, k0+32) of a row-major [R, K] fp32 matrix as bf16
template <bool VEC>
__device__ __forceinline__ void stage_rows(const float* __restrict__ S, int64_t R, int K,
                                           int64_t r0, int k0, h16 (*D)[kGLd], int tid) {
  if (VEC) {  // K % 4 == 0: float4 loads, 4 per thread
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int f = tid + 256 * it;
      const int r = f >> 3, kc = (f & 7) * 4;
      const int64_t row = r0 + r;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < R && k0 + kc < K) v = *reinterpret_cast<const float4*>(S + row * K + k0 + kc);
      h16x4 o;
      o[0] = (h16)v.x;
      o[1] = (h16)v.y;
      o[2] = (h16)v.z;
      o[3] = (h16)v.w;
      *reinterpret_cast<h16x4*>(&D[r][kc]) = o;
    }
  } else {
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int e = tid + 256 * it;
      const int r = e >> 5, k = e & 31;
      const int64_t row = r0 + r;
      const float v = (row < R && k0 + k < K) ? S[row * K + k0 + k] : 0.0f;
      D[r][k] = (h16)v;
    }
  }
}

// software-pipelined staging (K % 4 == 0): the next slice's float4s are loaded into registers
// while the MFMAs of the current slice run, then rounded and stored after the barrier
struct RowRegs {
  float4 v[4];
};

__device__ __forceinline__ void load_rows(const float* __restrict__ S, int64_t R, int K, int64_t r0,
                                          int k0, int tid, RowRegs& g) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int f = tid + 256 * it;
    const int r = f >> 3, kc = (f & 7) * 4;
    const int64_t row = r0 + r;
    g.v[it] = (row < R && k0 + kc < K) ? *reinterpret_cast<const float4*>(S + row * K + k0 + kc)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

__device__ __forceinline__ void store_rows(const RowRegs& g, h16 (*D)[kGLd], int tid) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int f = tid + 256 * it;
    const int r = f >> 3, kc = (f & 7) * 4;
    h16x4 o;
    o[0] = (h16)g.v[it].x;
    o[1] = (h16)g.v[it].y;
    o[2] = (h16)g.v[it].z;
    o[3] = (h16)g.v[it].w;
    *reinterpret_cast<h16x4*>(&D[r][kc]) = o;
  }
}

template <bool VEC>
__global__ __launch_bounds__(256) void gemm_nt_bf16_kernel(const float* __restrict__ A, int64_t M,
                                                           int K, const float* __restrict__ B,
                                                           int O, const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           int relu, float* __restrict__ C) {
  __shared__ __attribute__((aligned(16))) h16 As[kGT][kGLd];
  __shared__ __attribute__((aligned(16))) h16 Bs[kGT][kGLd];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, h = lane >> 5, l32 = lane & 31;
  const int64_t m0 = (int64_t)blockIdx.x * kGT;
  const int o0 = blockIdx.y * kGT;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  if (VEC) {
    RowRegs ga, gb;
    load_rows(A, M, K, m0, 0, tid, ga);
    load_rows(B, O, K, o0, 0, tid, gb);
    for (int k0 = 0; k0 < K; k0 += kGK) {
      store_rows(ga, As, tid);
      store_rows(gb, Bs, tid);
      __syncthreads();
      if (k0 + kGK < K) {
        load_rows(A, M, K, m0, k0 + kGK, tid, ga);
        load_rows(B, O, K, o0, k0 + kGK, tid, gb);
      }
      mma_slice(As, Bs, wr, wc, l32, h, acc);
      __syncthreads();
    }
  } else {
    for (int k0 = 0; k0 < K; k0 += kGK) {
      stage_rows<false>(A, M, K, m0, k0, As, tid);
      stage_rows<false>(B, O, K, o0, k0, Bs, tid);
      __syncthreads();
      mma_slice(As, Bs, wr, wc, l32, h, acc);
      __syncthreads();
    }
  }
#pragma unroll
  for (int bn = 0; bn < 2; ++bn) {
    const int o = o0 + wc * 64 + bn * 32 + l32;
    if (o >= O) continue;
    const float sc = scale ? scale[o] : 1.0f;
    const float sh = shift ? shift[o] : 0.0f;
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wr * 64 + bm * 32 + grow(r, h);
        float v = fmaf(acc[bm][bn][r], sc, sh);
        if (relu) v = fmaxf(v, 0.0f);
        if (m < M) C[m * O + o] = v;
      }
  }
}

struct ColRegs {
  float v[16];
};

__device__ __forceinline__ void load_cols(const float* __restrict__ S, int64_t Mend, int Cn,
                                          int64_t m0, int c0, int tid, ColRegs& g) {
  const int c = tid & 127, half = tid >> 7;
  const bool cv = c0 + c < Cn;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int64_t m = m0 + half * 16 + j;
    g.v[j] = (cv && m < Mend) ? S[m * Cn + c0 + c] : 0.0f;
  }
}

__device__ __forceinline__ void store_cols(const ColRegs& g, h16 (*D)[kGLd], int tid,
                                           float* colsum) {
  const int c = tid & 127, half = tid >> 7;
  h16x8 f[2];
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    s += g.v[j];
    f[j >> 3][j & 7] = (h16)g.v[j];
  }
  *reinterpret_cast<h16x8*>(&D[c][half * 16]) = f[0];
  *reinterpret_cast<h16x8*>(&D[c][half * 16 + 8]) = f[1];
  if (colsum) *colsum += s;
}

__global__ __launch_bounds__(256) void wgrad_bf16_kernel(const float* __restrict__ dZ,
                                                         const float* __restrict__ X, int64_t M,
                                                         int I, int O, int64_t rows_per_chunk,
                                                         int tiles_i, float* __restrict__ partW,
                                                         float* __restrict__ partB) {
  __shared__ __attribute__((aligned(16))) h16 As[kGT][kGLd];  // dZ^T: [o][m]
  __shared__ __attribute__((aligned(16))) h16 Bs[kGT][kGLd];  // X^T:  [i][m]
  __shared__ float bred[kGT];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, h = lane >> 5, l32 = lane & 31;
  const int o0 = (blockIdx.x / tiles_i) * kGT, i0 = (blockIdx.x % tiles_i) * kGT;
  const int chunk = blockIdx.y;
  const int64_t mb = (int64_t)chunk * rows_per_chunk;
  const int64_t me = mb + rows_per_chunk < M ? mb + rows_per_chunk : M;
  const bool bias = partB != nullptr && i0 == 0;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  float bsum = 0.0f;
  ColRegs ga, gb;
  load_cols(dZ, me, O, mb, o0, tid, ga);
  load_cols(X, me, I, mb, i0, tid, gb);
  for (int64_t k0 = mb; k0 < me; k0 += kGK) {
    store_cols(ga, As, tid, bias ? &bsum : nullptr);
    store_cols(gb, Bs, tid, nullptr);
    __syncthreads();
    if (k0 + kGK < me) {  // next slice in flight during this slice's MFMAs
      load_cols(dZ, me, O, k0 + kGK, o0, tid, ga);
      load_cols(X, me, I, k0 + kGK, i0, tid, gb);
    }
    mma_slice(As, Bs, wr, wc, l32, h, acc);
    __syncthreads();
  }
#pragma unroll
  for (int bn = 0; bn < 2; ++bn) {
    const int i = i0 + wc * 64 + bn * 32 + l32;
    if (i >= I) continue;
    float* pw = partW + (int64_t)chunk * O * I;
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + wr * 64 + bm * 32 + grow(r, h);
        if (o < O) pw[(int64_t)o * I + i] = acc[bm][bn][r];
      }
  }
  if (bias) {  // fp32 column sums of the chunk (unrounded dZ), two halves per column
    if (tid >= 128) bred[tid - 128] = bsum;
    __syncthreads();
    if (tid < 128 && o0 + tid < O) partB[(int64_t)chunk * O + o0 + tid] = bsum + bred[tid];
  }
}

// Chunk partials -> dW and db in one launch: a 256-thread block covers 64 outputs (of dW, then
// of db); wave w folds its quarter of the chunks in order into float64 with its loads in flight
// together, and the four quarters meet in LDS in order -- a fixed reduction tree (deterministic).
constexpr int kCombLoads = 32;
__global__ __launch_bounds__(256) void wgrad_bf16_combine_kernel(
    const float* __restrict__ partW, int64_t nW, const float* __restrict__ partB, int64_t nB,
    int chunks, float* __restrict__ outW, float* __restrict__ outB) {
  __shared__ double red[3][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t q = (int64_t)blockIdx.x * 64 + lane;
  const bool isW = q < nW;
  const bool valid = q < nW + nB;
  const float* part = isW ? partW : partB;
  const int64_t n = isW ? nW : nB;
  const int64_t e = isW ? q : q - nW;
  const int lo = (w * chunks) / 4, hi = ((w + 1) * chunks) / 4;
  double s = 0.0;
  if (valid) {
    for (int c0 = lo; c0 < hi; c0 += kCombLoads) {
      float v[kCombLoads];
#pragma unroll
      for (int u = 0; u < kCombLoads; ++u)
        if (c0 + u < hi) v[u] = part[(int64_t)(c0 + u) * n + e];
#pragma unroll
      for (int u = 0; u < kCombLoads; ++u)
        if (c0 + u < hi) s += (double)v[u];
    }
  }
  if (w) red[w - 1][lane] = s;
  __syncthreads();
  if (w == 0 && valid) {
#pragma unroll
    for (int k = 0; k < 3; ++k) s += red[k][lane];
    if (isW) outW[e] = (float)s; else outB[e] = (float)s;
  }
}

struct Bf16WgradPlan {
  int tiles_i, tiles_o, chunks;
  int64_t rows_per_chunk;
};

static Bf16WgradPlan bf16_wgrad_plan(int64_t M, int64_t I, int64_t O) {
  Bf16WgradPlan p;
  p.tiles_i = (int)cdiv(I, kGT);
  p.tiles_o = (int)cdiv(O, kGT);
  const int64_t tiles = (int64_t)p.tiles_i * p.tiles_o;
  int64_t chunks = cdiv(512, tiles);  // ~2 workgroups per CU; fewer partials to combine
  chunks = std::max<int64_t>(1, std::min<int64_t>(chunks, cdiv(M, 512)));
  p.rows_per_chunk = cdiv(cdiv(M, chunks), kGK) * kGK;
  p.chunks = (int)cdiv(M, p.rows_per_chunk);
  return p;
}

int gemm_nt_impl(const float* A, int64_t M, int64_t K, const float* B, int64_t O,
                 const float* scale, const float* shift, int relu, float* C, void* stream) {
  PCST_CHECK_ARG(M >= 0 && K > 0 && O > 0 && K < (1 << 20) && O < (1 << 20),
                 "gemm_nt_bf16: bad shape");
  if (M == 0) return PCST_OK;
  PCST_CHECK_ARG(A && B && C, "gemm_nt_bf16: null pointer");
  dim3 grid((unsigned)cdiv(M, kGT), (unsigned)cdiv(O, kGT));
  const bool vec = (K % 4 == 0) && ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0);
  if (vec)
    hipLaunchKernelGGL(gemm_nt_bf16_kernel<true>, grid, dim3(256), 0, as_stream(stream), A, M,
                       (int)K, B, (int)O, scale, shift, relu, C);
  else
    hipLaunchKernelGGL(gemm_nt_bf16_kernel<false>, grid, dim3(256), 0, as_stream(stream), A, M,
                       (int)K, B, (int)O, scale, shift, relu, C);
  PCST_LAUNCH_CHECK("gemm_nt_bf16");
  return PCST_OK;
}

int wgrad16_workspace_impl(int64_t M, int64_t I, int64_t O, size_t* bytes) {
  PCST_CHECK_ARG(M >= 0 && I > 0 && O > 0 && bytes, "linear_wgrad_bf16_workspace_size: bad args");
  const Bf16WgradPlan p = bf16_wgrad_plan(std::max<int64_t>(M, 1), I, O);
  *bytes = sizeof(float) * (size_t)p.chunks * (size_t)(O * I + O);
  return PCST_OK;
}

int wgrad16_impl(const float* dZ, const float* X, int64_t M, int64_t I, int64_t O, float* dW,
                 float* db, void* workspace, void* stream) {
  PCST_CHECK_ARG(M >= 0 && I > 0 && O > 0 && I < (1 << 20) && O < (1 << 20),
                 "linear_wgrad_bf16: bad shape");
  PCST_CHECK_ARG(dW && workspace && (M == 0 || (dZ && X)), "linear_wgrad_bf16: null pointer");
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    PCST_HIP(hipMemsetAsync(dW, 0, sizeof(float) * O * I, s), "memset");
    if (db) PCST_HIP(hipMemsetAsync(db, 0, sizeof(float) * O, s), "memset");
    return PCST_OK;
  }
  const Bf16WgradPlan p = bf16_wgrad_plan(M, I, O);
  float* partW = static_cast<float*>(workspace);
  float* partB = db ? partW + (int64_t)p.chunks * O * I : nullptr;
  hipLaunchKernelGGL(wgrad_bf16_kernel, dim3((unsigned)(p.tiles_i * p.tiles_o), (unsigned)p.chunks),
                     dim3(256), 0, s, dZ, X, M, (int)I, (int)O, p.rows_per_chunk, p.tiles_i, partW,
                     partB);
  const int64_t nW = O * I, nB = db ? O : 0;
  hipLaunchKernelGGL(wgrad_bf16_combine_kernel, dim3((unsigned)cdiv(nW + nB, 64)), dim3(256), 0, s,
                     partW, nW, partB, nB, p.chunks, dW, db);
  PCST_LAUNCH_CHECK("linear_wgrad_bf16");
  return PCST_OK;
}

}  // namespace PCST_H16_NS
}  // namespace pcst

#if !PCST_H16_F16
// C entry points (include/pcst.h): `f16` picks the operand format the fp32 inputs are rounded
// to -- 0 bf16, 1 fp16 (the reference trainer's autocast dtype).
extern "C" int pcst_gemm_nt_bf16(const float* A, int64_t M, int64_t K, const float* B, int64_t O,
                                 const float* scale, const float* shift, int relu, float* C,
                                 int f16, void* stream) {
  return f16 ? pcst::f16m::gemm_nt_impl(A, M, K, B, O, scale, shift, relu, C, stream)
             : pcst::bf16m::gemm_nt_impl(A, M, K, B, O, scale, shift, relu, C, stream);
}

extern "C" int pcst_linear_wgrad_bf16_workspace_size(int64_t M, int64_t I, int64_t O,
                                                     size_t* bytes) {
  return pcst::bf16m::wgrad16_workspace_impl(M, I, O, bytes);
}

extern "C" int pcst_linear_wgrad_bf16(const float* dZ, const float* X, int64_t M, int64_t I,
                                      int64_t O, float* dW, float* db, void* workspace, int f16,
                                      void* stream) {
  return f16 ? pcst::f16m::wgrad16_impl(dZ, X, M, I, O, dW, db, workspace, stream)
             : pcst::bf16m::wgrad16_impl(dZ, X, M, I, O, dW, db, workspace, stream);
}
#endif
