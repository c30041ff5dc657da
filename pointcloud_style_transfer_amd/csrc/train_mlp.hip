// Training-path GEMMs with bf16 activation storage and fused epilogues (the NoisePredictor's
// residual blocks, reference models/diffusion_model.py:48-52,57-58, trained under autocast by
// training/trainer.py:81-106).  Every product runs on v_mfma_f32_32x32x16_bf16 with fp32
// accumulation; operands are bf16 either in HBM (activations written by a previous epilogue)
// or rounded from fp32 while staged, so storing an activation as bf16 changes no product.
//
//   gemm_ex:   C[m, o] = epilogue(sum_k A[m, k] B[o, k])          forward and dX
//     EP_F32         act(acc + bias)                     -> fp32
//     EP_BF16        act(acc + bias)                     -> bf16
//     EP_RESID_DROP  resid + keep(m, o) * (acc + bias) * s -> fp32  (x + Dropout(Linear2(h)))
//     EP_RELU_MASK   acc * [h > 0]                       -> bf16  (ReLU backward of Linear1)
//     EP_ADD         acc + add                           -> fp32  (residual gradient sum)
//     EP_RESID_DROP16, EP_ADD16: the same with a 16-bit residual operand and output (the residual
//                    stream in autocast's 16-bit format, as the reference's autocast keeps it)
//   EP_BF16 / EP_ADD16 with C2: also C2 = 16-bit(C * keep(e) / (1 - p)), the next Dropout
//   backward's dD from the stored 16-bit C (the dropout_grad kernel's result, fused)
//   wgrad_ex:  dW[o, i] = sum_m dZ[m, o] X[m, i],  db[o] = sum_m dZ[m, o]
//   dropout_grad: dD = bf16(g * keep * s)  (Dropout backward, the mask regenerated)
//
// Dropout keeps element e = m * O + o iff hash(seed, e) >= p * 2^32: the mask is a pure function
// of (seed, e), so the backward regenerates it instead of storing it.
//
// gemm_ex tiles 128 x 128 per 256-thread workgroup (2 x 2 waves of 64 x 64, K staged 32 deep,
// software-pipelined through registers), maps tiles to workgroups so that the O-tiles of one
// M-tile run on one XCD back to back (the A rows are read from HBM once, then hit that XCD's
// L2), and writes the tile through LDS so the epilogue reads/writes rows with 16-byte accesses.
// wgrad_ex stages dZ and X row-major (coalesced) and feeds both MFMA operands with
// ds_read_b64_tr_b16 transposed reads; the M reduction is split into chunks whose partials are
// combined in chunk order (deterministic), as csrc/train_gemm.hip does.
//
// 16-bit operand format: this file is compiled twice (Makefile), as itself for bf16 and through
// train_mlp_f16.hip (PCST_H16_F16 = 1) for fp16 -- the autocast dtype of the reference's CUDA
// trainer (training/trainer.py:50,78; v_mfma_f32_32x32x16_f16 runs at the bf16 rate).  The
// kernels live in pcst::bf16m / pcst::f16m; the C entry points (bf16 build) dispatch on `f16`.
#include "common.h"
#include "train_h16.h"

#ifndef PCST_H16_F16
#define PCST_H16_F16 0
#endif

namespace pcst {
namespace PCST_H16_NS {

typedef __attribute__((ext_vector_type(16))) float f32x16;
#if PCST_H16_F16
typedef _Float16 h16;
#else
typedef __bf16 h16;
#endif
typedef __attribute__((ext_vector_type(8))) h16 h16x8;
typedef __attribute__((ext_vector_type(4))) h16 h16x4;
typedef __attribute__((ext_vector_type(2))) h16 h16x2;
typedef short v4i16 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma32_h16(h16x8 a, h16x8 b, f32x16 c) {
#if PCST_H16_F16
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
#endif
}
// 16-bit storage bits -> float
__device__ __forceinline__ float h16_to_f32(uint32_t bits16) {
#if PCST_H16_F16
  return (float)__builtin_bit_cast(_Float16, (uint16_t)bits16);
#else
  return __uint_as_float(bits16 << 16);
#endif
}

enum {
  EP_F32 = 0, EP_BF16 = 1, EP_RESID_DROP = 2, EP_RELU_MASK = 3, EP_ADD = 4, EP_COND = 5,
  EP_RESID_DROP16 = 6, EP_ADD16 = 7
};
// 16-bit output / 16-bit aux operand / the C2 dropout copy of a 16-bit output
__host__ __device__ constexpr bool ep_out16(int ep) {
  return ep == EP_BF16 || ep == EP_RELU_MASK || ep == EP_RESID_DROP16 || ep == EP_ADD16;
}
__host__ __device__ constexpr bool ep_aux16(int ep) {
  return ep == EP_RELU_MASK || ep == EP_RESID_DROP16 || ep == EP_ADD16;
}
__host__ __device__ constexpr bool ep_drop_copy(int ep) { return ep == EP_BF16 || ep == EP_ADD16; }
__host__ __device__ constexpr bool ep_dropout(int ep) { return ep == EP_RESID_DROP || ep == EP_RESID_DROP16; }
__host__ __device__ constexpr bool ep_no_bias(int ep) {
  return ep == EP_RELU_MASK || ep == EP_ADD || ep == EP_ADD16;
}

constexpr int kXT = 128, kXK = 32, kXLd = 40;  // tile, k slice, LDS row (bf16 elements, 80 B)
constexpr int kCLd = 132;                      // epilogue LDS row (floats)

__device__ __forceinline__ int xrow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// dropout draw of element e under a 64-bit seed
__device__ __forceinline__ uint32_t drop_hash(uint32_t slo, uint32_t shi, uint64_t e) {
  return mix32((uint32_t)e ^ slo ^ mix32((uint32_t)(e >> 32) + shi));
}

// ---- operand staging: rows [r0, r0+128) x k [k0, k0+32) of a row-major [R, K] matrix -> bf16 LDS
template <typename T>
struct XStage;

template <>
struct XStage<float> {  // K % 4 == 0
  float4 v[4];
  __device__ __forceinline__ void load(const float* __restrict__ S, int64_t R, int K, int64_t r0,
                                       int k0, int tid) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int f = tid + 256 * it;
      const int r = f >> 3, kc = (f & 7) * 4;
      const int64_t row = r0 + r;
      v[it] = (row < R && k0 + kc < K) ? *reinterpret_cast<const float4*>(S + row * K + k0 + kc)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __device__ __forceinline__ void store(h16 (*D)[kXLd], int tid) const {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int f = tid + 256 * it;
      const int r = f >> 3, kc = (f & 7) * 4;
      h16x4 o;
      o[0] = (h16)v[it].x;
      o[1] = (h16)v[it].y;
      o[2] = (h16)v[it].z;
      o[3] = (h16)v[it].w;
      *reinterpret_cast<h16x4*>(&D[r][kc]) = o;
    }
  }
};

template <>
struct XStage<uint16_t> {  // bf16 storage, K % 8 == 0
  uint4 v[2];
  __device__ __forceinline__ void load(const uint16_t* __restrict__ S, int64_t R, int K,
                                       int64_t r0, int k0, int tid) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int f = tid + 256 * it;
      const int r = f >> 2, kc = (f & 3) * 8;
      const int64_t row = r0 + r;
      v[it] = (row < R && k0 + kc < K) ? *reinterpret_cast<const uint4*>(S + row * K + k0 + kc)
                                       : make_uint4(0u, 0u, 0u, 0u);
    }
  }
  __device__ __forceinline__ void store(h16 (*D)[kXLd], int tid) const {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int f = tid + 256 * it;
      const int r = f >> 2, kc = (f & 3) * 8;
      *reinterpret_cast<uint4*>(&D[r][kc]) = v[it];
    }
  }
};

// one 32-deep k slice: 2 x 2 blocks x 2 k-steps of 32x32x16
__device__ __forceinline__ void xmma_slice(const h16 (*As)[kXLd], const h16 (*Bs)[kXLd],
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

struct GemmExArgs {
  const float* bias;
  int relu;
  const void* aux;  // EP_RESID_DROP: resid fp32 [M,O]; EP_RELU_MASK: h bf16 [M,O]; EP_ADD: fp32;
                    // EP_COND: [G, 2, O] fp32 (two per-group row vectors added in turn);
                    // EP_RESID_DROP16 / EP_ADD16: 16-bit [M,O]
  uint32_t seed_lo, seed_hi, thr;
  float scale;
  void* C;
  uint16_t* C2;     // optional bf16 copy of an fp32 output (EP_F32, EP_RESID_DROP, EP_COND; C may
                    // then be null for EP_COND), or the dropout copy (EP_BF16, EP_ADD16)
  int64_t group_rows;  // EP_COND: rows per group
};

__device__ __forceinline__ void store4_bf16(uint16_t* p, float a, float b, float c, float d) {
  h16x4 o;
  o[0] = (h16)a;
  o[1] = (h16)b;
  o[2] = (h16)c;
  o[3] = (h16)d;
  *reinterpret_cast<h16x4*>(p) = o;
}

// epilogue: two passes of 64 rows through LDS; thread -> (column quad tid % 32, rows
// tid / 32 + 8j), 16-byte row accesses for the output and the aux operand
template <int EP>
__device__ __forceinline__ void gemm_epilogue(const f32x16 (&acc)[2][2], float (*Cs)[kCLd],
                                              int64_t M, int O, int64_t m0, int o0,
                                              const GemmExArgs& args) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, h = lane >> 5, l32 = lane & 31;
  const int cq = (tid & 31) * 4, rl = tid >> 5;
  const int o = o0 + cq;
  const int nv = O - o < 4 ? (O - o > 0 ? O - o : 0) : 4;  // valid columns of the quad
  const bool vec = nv == 4 && (O & 3) == 0;
  float bias4[4] = {0.f, 0.f, 0.f, 0.f};
  if (args.bias)
    for (int u = 0; u < nv; ++u) bias4[u] = args.bias[o + u];
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (pass) __syncthreads();
    if (wr == pass) {
#pragma unroll
      for (int bm = 0; bm < 2; ++bm)
#pragma unroll
        for (int bn = 0; bn < 2; ++bn)
#pragma unroll
          for (int r = 0; r < 16; ++r) Cs[bm * 32 + xrow(r, h)][wc * 64 + bn * 32 + l32] = acc[bm][bn][r];
    }
    __syncthreads();
#pragma unroll 2
    for (int j = 0; j < 8; ++j) {
      const int rr = rl + 8 * j;
      const int64_t m = m0 + pass * 64 + rr;
      if (m >= M || nv == 0) continue;
      const float4 c = *reinterpret_cast<const float4*>(&Cs[rr][cq]);
      const int64_t e = m * O + o;
      float v[4] = {c.x + bias4[0], c.y + bias4[1], c.z + bias4[2], c.w + bias4[3]};
      if (ep_no_bias(EP)) {  // no bias on the gradient products
        v[0] = c.x;
        v[1] = c.y;
        v[2] = c.z;
        v[3] = c.w;
      }
      if ((EP == EP_F32 || EP == EP_BF16) && args.relu) {
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = fmaxf(v[u], 0.0f);
      }
      float y[4];
      if (ep_dropout(EP)) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool keep = drop_hash(args.seed_lo, args.seed_hi, (uint64_t)(e + u)) >= args.thr;
          y[u] = keep ? v[u] * args.scale : 0.0f;
        }
      } else if (EP == EP_COND) {  // ((acc + b) + cond0[g]) + cond1[g], the reference's order
        const float* cg = static_cast<const float*>(args.aux) + (m / args.group_rows) * 2 * O + o;
#pragma unroll
        for (int u = 0; u < 4; ++u) y[u] = u < nv ? (v[u] + cg[u]) + cg[O + u] : 0.0f;
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) y[u] = v[u];
      }
      if (EP == EP_RESID_DROP16 || EP == EP_ADD16) {  // 16-bit residual operand
        const uint16_t* a16 = static_cast<const uint16_t*>(args.aux) + e;
        for (int u = 0; u < nv; ++u) y[u] += h16_to_f32(a16[u]);
      }
      if (EP == EP_RESID_DROP || EP == EP_ADD || EP == EP_RELU_MASK) {
        if (vec) {
          if (EP == EP_RELU_MASK) {
            const uint2 hb = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(args.aux) + e);
            const int16_t hs[4] = {(int16_t)(hb.x & 0xffff), (int16_t)(hb.x >> 16),
                                   (int16_t)(hb.y & 0xffff), (int16_t)(hb.y >> 16)};
#pragma unroll
            for (int u = 0; u < 4; ++u) y[u] = hs[u] > 0 ? y[u] : 0.0f;
          } else {
            const float4 a = *reinterpret_cast<const float4*>(static_cast<const float*>(args.aux) + e);
            y[0] += a.x;
            y[1] += a.y;
            y[2] += a.z;
            y[3] += a.w;
          }
        } else {
          for (int u = 0; u < nv; ++u) {
            if (EP == EP_RELU_MASK)
              y[u] = (int16_t)static_cast<const uint16_t*>(args.aux)[e + u] > 0 ? y[u] : 0.0f;
            else
              y[u] += static_cast<const float*>(args.aux)[e + u];
          }
        }
      }
      if (ep_out16(EP)) {
        uint16_t* out = static_cast<uint16_t*>(args.C) + e;
        if (vec) {
          store4_bf16(out, y[0], y[1], y[2], y[3]);
        } else {
          for (int u = 0; u < nv; ++u) {
            const h16 b = (h16)y[u];
            out[u] = __builtin_bit_cast(uint16_t, b);
          }
        }
        if (ep_drop_copy(EP) && args.C2) {  // dD = 16-bit(C16 * keep / (1 - p))
          for (int u = 0; u < nv; ++u) {
            const bool keep = drop_hash(args.seed_lo, args.seed_hi, (uint64_t)(e + u)) >= args.thr;
            const float yr = (float)(h16)y[u];
            args.C2[e + u] = __builtin_bit_cast(uint16_t, (h16)(keep ? yr * args.scale : 0.0f));
          }
        }
      } else {
        float* out = static_cast<float*>(args.C) + e;
        if (vec) {
          if (EP != EP_COND || args.C) *reinterpret_cast<float4*>(out) = make_float4(y[0], y[1], y[2], y[3]);
          if (args.C2) store4_bf16(args.C2 + e, y[0], y[1], y[2], y[3]);
        } else {
          for (int u = 0; u < nv; ++u) {
            if (EP != EP_COND || args.C) out[u] = y[u];
            if (args.C2) args.C2[e + u] = __builtin_bit_cast(uint16_t, (h16)y[u]);
          }
        }
      }
    }
  }
}

template <typename TA, typename TB, int EP>
__global__ __launch_bounds__(256) void gemm_ex_kernel(const TA* __restrict__ A, int64_t M, int K,
                                                      const TB* __restrict__ B, int O,
                                                      int tiles_o, int ntiles, int per_xcd,
                                                      GemmExArgs args) {
  constexpr int kStageBytes = 2 * kXT * kXLd * 2;  // As + Bs
  constexpr int kEpiBytes = 64 * kCLd * 4;         // half the C tile, fp32
  __shared__ __attribute__((aligned(16))) char smem[kStageBytes > kEpiBytes ? kStageBytes : kEpiBytes];
  h16 (*As)[kXLd] = reinterpret_cast<h16 (*)[kXLd]>(smem);
  h16 (*Bs)[kXLd] = reinterpret_cast<h16 (*)[kXLd]>(smem + kXT * kXLd * 2);
  float (*Cs)[kCLd] = reinterpret_cast<float (*)[kCLd]>(smem);

  // XCD-aware tile order: workgroup L runs on XCD L % 8; tile t = xcd * per_xcd + L / 8, so the
  // consecutive tiles of one XCD are the O-tiles of one M-tile
  const int L = blockIdx.x;
  const int t = (L & 7) * per_xcd + (L >> 3);
  if (t >= ntiles) return;
  const int64_t m0 = (int64_t)(t / tiles_o) * kXT;
  const int o0 = (t % tiles_o) * kXT;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, h = lane >> 5, l32 = lane & 31;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  XStage<TA> ga;
  XStage<TB> gb;
  ga.load(A, M, K, m0, 0, tid);
  gb.load(B, O, K, o0, 0, tid);
  for (int k0 = 0; k0 < K; k0 += kXK) {
    ga.store(As, tid);
    gb.store(Bs, tid);
    __syncthreads();
    if (k0 + kXK < K) {  // next slice in flight during this slice's MFMAs
      ga.load(A, M, K, m0, k0 + kXK, tid);
      gb.load(B, O, K, o0, k0 + kXK, tid);
    }
    xmma_slice(As, Bs, wr, wc, l32, h, acc);
    __syncthreads();
  }

  gemm_epilogue<EP>(acc, Cs, M, O, m0, o0, args);
}

// ---- bf16 x bf16 GEMM, K staged kBK deep through registers (the next slice's buffer loads in
// flight during this slice's MFMAs) into a double-buffered LDS image: one barrier per slice.
constexpr int kBK = 32;             // k slice
constexpr int kBLd = kBK + 8;       // LDS row, bf16 elements (+16 B pad: conflict-free row reads)
constexpr int kCPR = kBK / 8;       // 16-byte chunks per row slice
constexpr int kBIt = kCPR / 2;      // loads per thread per operand per slice

struct BfRegs {
  uint4 a[kBIt], b[kBIt];
};

typedef __amdgpu_buffer_rsrc_t rsrc_t;
// raw buffer over [p, p + bytes): loads past the end return 0, stores past it are dropped
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
typedef int v4i32 __attribute__((ext_vector_type(4)));
typedef int v2i32 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 bload16(rsrc_t r, uint32_t voff, uint32_t soff) {
  const v4i32 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0);
  return make_uint4((uint32_t)v.x, (uint32_t)v.y, (uint32_t)v.z, (uint32_t)v.w);
}

// slice k0 of the A rows / B rows: byte offsets per thread fixed for the tile, the slice offset
// is scalar; rows past M (or O) read 0 from the buffer bound, so the loads are branch-free
__device__ __forceinline__ void bf_load(rsrc_t ra, rsrc_t rb, const uint32_t (&va)[kBIt],
                                        const uint32_t (&vb)[kBIt], uint32_t soff, BfRegs& g) {
#pragma unroll
  for (int it = 0; it < kBIt; ++it) {
    g.a[it] = bload16(ra, va[it], soff);
    g.b[it] = bload16(rb, vb[it], soff);
  }
}

__device__ __forceinline__ void bf_store(const BfRegs& g, h16 (*As)[kBLd], h16 (*Bs)[kBLd],
                                         int tid) {
#pragma unroll
  for (int it = 0; it < kBIt; ++it) {
    const int r = tid / kCPR + (256 / kCPR) * it, kc = (tid % kCPR) * 8;
    *reinterpret_cast<uint4*>(&As[r][kc]) = g.a[it];
    *reinterpret_cast<uint4*>(&Bs[r][kc]) = g.b[it];
  }
}

// this wave's LDS writes done, then the workgroup barrier; the global loads in flight stay
// in flight (no vmcnt wait), and the memory clobber keeps LDS accesses on their side
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ void bf_mma(const h16 (*As)[kBLd], const h16 (*Bs)[kBLd], int wr,
                                       int wc, int l32, int h, f32x16 (&acc)[2][2]) {
#pragma unroll
  for (int ks = 0; ks < kBK / 16; ++ks) {
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

__device__ __forceinline__ uint2 pack4_bf16(float a, float b, float c, float d) {
  h16x4 o;
  o[0] = (h16)a;
  o[1] = (h16)b;
  o[2] = (h16)c;
  o[3] = (h16)d;
  return *reinterpret_cast<const uint2*>(&o);
}

// epilogue for O % 128 == 0 (every column quad valid) and buffers < 4 GiB: the LDS round trip
// of gemm_epilogue with 32-bit buffer offsets (rows past M are dropped by the buffer bound)
template <int EP, int PASSES = 2>
__device__ __forceinline__ void gemm_epilogue_fast(const f32x16 (&acc)[2][2], float (*Cs)[kCLd],
                                                   int64_t M, int O, int64_t m0, int o0,
                                                   const GemmExArgs& args) {
  constexpr int RP = kXT / PASSES;  // rows per pass (64 or 32)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, h = lane >> 5, l32 = lane & 31;
  const int cq = (tid & 31) * 4, rl = tid >> 5;
  constexpr bool kOutBf16 = ep_out16(EP);
  const uint32_t nel = (uint32_t)(M * O);
  const rsrc_t rc = make_rsrc(args.C, nel * (kOutBf16 ? 2u : 4u));
  const rsrc_t rc2 = make_rsrc(args.C2, args.C2 ? nel * 2u : 0u);
  const rsrc_t rx = make_rsrc(args.aux, args.aux ? nel * (ep_aux16(EP) ? 2u : 4u) : 0u);
  float bias4[4] = {0.f, 0.f, 0.f, 0.f};
  if (args.bias && !ep_no_bias(EP)) {
    const float4 b = *reinterpret_cast<const float4*>(args.bias + o0 + cq);
    bias4[0] = b.x;
    bias4[1] = b.y;
    bias4[2] = b.z;
    bias4[3] = b.w;
  }
#pragma unroll
  for (int pass = 0; pass < PASSES; ++pass) {
    if (pass) __syncthreads();
#pragma unroll
    for (int bm = 0; bm < 2; ++bm) {
      const int rb = wr * 64 + bm * 32;  // this block's first row in the tile
      if (rb / RP != pass) continue;
#pragma unroll
      for (int bn = 0; bn < 2; ++bn)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          Cs[rb % RP + xrow(r, h)][wc * 64 + bn * 32 + l32] = acc[bm][bn][r];
    }
    __syncthreads();
    const uint32_t e0 = (uint32_t)((m0 + pass * RP + rl) * O + o0 + cq);
#pragma unroll 4
    for (int j = 0; j < RP / 8; ++j) {
      const uint32_t e = e0 + (uint32_t)(8 * j * O);
      const float4 c = *reinterpret_cast<const float4*>(&Cs[rl + 8 * j][cq]);
      float y[4] = {c.x + bias4[0], c.y + bias4[1], c.z + bias4[2], c.w + bias4[3]};
      if ((EP == EP_F32 || EP == EP_BF16) && args.relu) {
#pragma unroll
        for (int u = 0; u < 4; ++u) y[u] = fmaxf(y[u], 0.0f);
      }
      if (ep_dropout(EP)) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool keep = drop_hash(args.seed_lo, args.seed_hi, (uint64_t)(e + u)) >= args.thr;
          y[u] = keep ? y[u] * args.scale : 0.0f;
        }
      }
      if (EP == EP_RESID_DROP16 || EP == EP_ADD16) {
        const v2i32 hb = __builtin_amdgcn_raw_buffer_load_b64(rx, (int)(e * 2u), 0, 0);
        y[0] += h16_to_f32((uint32_t)hb.x & 0xffffu);
        y[1] += h16_to_f32((uint32_t)hb.x >> 16);
        y[2] += h16_to_f32((uint32_t)hb.y & 0xffffu);
        y[3] += h16_to_f32((uint32_t)hb.y >> 16);
      }
      if (EP == EP_RESID_DROP || EP == EP_ADD) {
        const v4i32 a = __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(e * 4u), 0, 0);
#pragma unroll
        for (int u = 0; u < 4; ++u) y[u] += __int_as_float(a[u]);
      }
      if (EP == EP_RELU_MASK) {
        const v2i32 hb = __builtin_amdgcn_raw_buffer_load_b64(rx, (int)(e * 2u), 0, 0);
        const int16_t hs[4] = {(int16_t)(hb.x & 0xffff), (int16_t)((uint32_t)hb.x >> 16),
                               (int16_t)(hb.y & 0xffff), (int16_t)((uint32_t)hb.y >> 16)};
#pragma unroll
        for (int u = 0; u < 4; ++u) y[u] = hs[u] > 0 ? y[u] : 0.0f;
      }
      if (kOutBf16) {
        const uint2 pk = pack4_bf16(y[0], y[1], y[2], y[3]);
        __builtin_amdgcn_raw_buffer_store_b64(v2i32{(int)pk.x, (int)pk.y}, rc, (int)(e * 2u), 0, 0);
        if (ep_drop_copy(EP) && args.C2) {  // dD = 16-bit(C16 * keep / (1 - p))
          const uint32_t w[2] = {pk.x, pk.y};
          float d[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const bool keep = drop_hash(args.seed_lo, args.seed_hi, (uint64_t)(e + u)) >= args.thr;
            const float yr = h16_to_f32((w[u >> 1] >> (16 * (u & 1))) & 0xffffu);
            d[u] = keep ? yr * args.scale : 0.0f;
          }
          const uint2 pd = pack4_bf16(d[0], d[1], d[2], d[3]);
          __builtin_amdgcn_raw_buffer_store_b64(v2i32{(int)pd.x, (int)pd.y}, rc2, (int)(e * 2u), 0, 0);
        }
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(
            v4i32{__float_as_int(y[0]), __float_as_int(y[1]), __float_as_int(y[2]), __float_as_int(y[3])},
            rc, (int)(e * 4u), 0, 0);
        if (args.C2) {
          const uint2 pk = pack4_bf16(y[0], y[1], y[2], y[3]);
          __builtin_amdgcn_raw_buffer_store_b64(v2i32{(int)pk.x, (int)pk.y}, rc2, (int)(e * 2u), 0, 0);
        }
      }
    }
  }
}

template <int EP, bool FAST>
__global__ __launch_bounds__(256) void gemm_bf_kernel(const uint16_t* __restrict__ A, int64_t M,
                                                      int K, const uint16_t* __restrict__ B, int O,
                                                      int tiles_o, int ntiles, int per_xcd,
                                                      GemmExArgs args) {
  constexpr int kBuf = kXT * kBLd * 2;  // one operand image, bytes
  constexpr int kStage = 4 * kBuf;      // A, B x two buffers
  constexpr int kEpi = 64 * kCLd * 4;
  __shared__ __attribute__((aligned(16))) char smem[kStage > kEpi ? kStage : kEpi];
  typedef h16 Row[kBLd];
  Row* As0 = reinterpret_cast<Row*>(smem);
  Row* Bs0 = reinterpret_cast<Row*>(smem + kBuf);
  Row* As1 = reinterpret_cast<Row*>(smem + 2 * kBuf);
  Row* Bs1 = reinterpret_cast<Row*>(smem + 3 * kBuf);

  const int L = blockIdx.x;
  const int t = (L & 7) * per_xcd + (L >> 3);
  if (t >= ntiles) return;
  const int64_t m0 = (int64_t)(t / tiles_o) * kXT;
  const int o0 = (t % tiles_o) * kXT;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, h = lane >> 5, l32 = lane & 31;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  // K % 64 == 0 and M*K*2, O*K*2 < 2^31 (host-checked)
  const rsrc_t ra = make_rsrc(A, (uint32_t)(M * K * 2));
  const rsrc_t rb = make_rsrc(B, (uint32_t)((int64_t)O * K * 2));
  uint32_t va[kBIt], vb[kBIt];
#pragma unroll
  for (int it = 0; it < kBIt; ++it) {
    const int r = tid / kCPR + (256 / kCPR) * it, kc = (tid % kCPR) * 8;
    va[it] = (uint32_t)(((m0 + r) * K + kc) * 2);
    vb[it] = (uint32_t)((((int64_t)o0 + r) * K + kc) * 2);
  }
  const int nk = K / kBK;
  BfRegs g;
  bf_load(ra, rb, va, vb, 0, g);
  for (int k = 0; k < nk; ++k) {
    Row* As = (k & 1) ? As1 : As0;
    Row* Bs = (k & 1) ? Bs1 : Bs0;
    bf_store(g, As, Bs, tid);
    lds_barrier();  // one barrier per slice: the other buffer's readers finished a slice ago
    if (k + 1 < nk) bf_load(ra, rb, va, vb, (uint32_t)((k + 1) * kBK * 2), g);
    bf_mma(As, Bs, wr, wc, l32, h, acc);
  }
  __syncthreads();  // every wave's MFMA reads done before the epilogue reuses the LDS
  if (FAST)
    gemm_epilogue_fast<EP>(acc, reinterpret_cast<float (*)[kCLd]>(smem), M, O, m0, o0, args);
  else
    gemm_epilogue<EP>(acc, reinterpret_cast<float (*)[kCLd]>(smem), M, O, m0, o0, args);
}

// A 16-bit fragment read in inline asm (the residual-block kernels): invisible to the compiler's
// LDS-DMA tracking, which would otherwise drain vmcnt(0) (every weight slice in flight) at the
// loop head.  Each read's wait is a counted lgkmcnt tied to the registers it guards (as
// csrc/noise_mlp.hip does), so no MFMA is scheduled above it.
template <int OFF>
__device__ __forceinline__ h16x8 dma_read(uint32_t addr) {
  h16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}

// ---- Dropout backward: dD = bf16(g * keep * s), 4 elements per thread (n % 4 == 0)
__global__ void dropout_grad_kernel(const float4* __restrict__ g, int64_t n4, uint32_t slo,
                                    uint32_t shi, uint32_t thr, float scale,
                                    uint2* __restrict__ out) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n4;
       q += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = g[q];
    const float vs[4] = {v.x, v.y, v.z, v.w};
    float y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool keep = drop_hash(slo, shi, (uint64_t)(4 * q + u)) >= thr;
      y[u] = keep ? vs[u] * scale : 0.0f;
    }
    h16x4 o;
    o[0] = (h16)y[0];
    o[1] = (h16)y[1];
    o[2] = (h16)y[2];
    o[3] = (h16)y[3];
    out[q] = *reinterpret_cast<const uint2*>(&o);
  }
}

// ---- weight gradient with transposed LDS reads
constexpr int kWS = 32;                 // m rows per slice
constexpr int kWLdB = 2 * kXT + 64;     // LDS row bytes: 256 + 64 (row stride = 64 mod 256 B)

// slice rows [m, m+32) x columns [c0, c0+128) of a row-major [*, Cn] matrix -> bf16 LDS image
template <typename T>
struct WStage;

template <>
struct WStage<float> {  // Cn % 4 == 0: thread -> (column quad tid % 32, rows tid / 32 + 8 it)
  static constexpr int kIt = kWS / 8;
  float4 v[kIt];
  __device__ __forceinline__ void load(const float* __restrict__ S, int64_t mend, int Cn,
                                       int64_t m, int c0, int tid) {
    const int cq = (tid & 31) * 4;
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int64_t row = m + (tid >> 5) + 8 * it;
      v[it] = (row < mend && c0 + cq < Cn) ? *reinterpret_cast<const float4*>(S + row * Cn + c0 + cq)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // the same slice by raw buffer loads: rows past the buffer read 0, a column quad past Cn is
  // sent past the buffer too -- no branch, so the compiler counts the loads in flight exactly
  __device__ __forceinline__ void load_buf(rsrc_t r, int64_t m, int c0, int Cn, int tid, bool ok) {
    const int cq = (tid & 31) * 4;
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int64_t row = m + (tid >> 5) + 8 * it;
      const uint32_t off = ok && c0 + cq < Cn ? (uint32_t)((row * Cn + c0 + cq) * 4) : 0xfffffff0u;
      const v4i32 q = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
      v[it] = make_float4(__int_as_float(q.x), __int_as_float(q.y), __int_as_float(q.z), __int_as_float(q.w));
    }
  }
  __device__ __forceinline__ void store(char* D, int tid, float* csum) const {
    const int cq = (tid & 31) * 4;
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int r = (tid >> 5) + 8 * it;
      h16x4 o;
      o[0] = (h16)v[it].x;
      o[1] = (h16)v[it].y;
      o[2] = (h16)v[it].z;
      o[3] = (h16)v[it].w;
      *reinterpret_cast<h16x4*>(D + r * kWLdB + cq * 2) = o;
      if (csum) {  // unrounded fp32 column sums
        csum[0] += v[it].x;
        csum[1] += v[it].y;
        csum[2] += v[it].z;
        csum[3] += v[it].w;
      }
    }
  }
  static constexpr int kSumCols = 4, kRowLanes = 8;
};

template <>
struct WStage<uint16_t> {  // Cn % 8 == 0: thread -> (column octet tid % 16, rows tid / 16 + 16 it)
  static constexpr int kIt = kWS / 16;
  uint4 v[kIt];
  __device__ __forceinline__ void load(const uint16_t* __restrict__ S, int64_t mend, int Cn,
                                       int64_t m, int c0, int tid) {
    const int co = (tid & 15) * 8;
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int64_t row = m + (tid >> 4) + 16 * it;
      v[it] = (row < mend && c0 + co < Cn) ? *reinterpret_cast<const uint4*>(S + row * Cn + c0 + co)
                                           : make_uint4(0u, 0u, 0u, 0u);
    }
  }
  __device__ __forceinline__ void load_buf(rsrc_t r, int64_t m, int c0, int Cn, int tid, bool ok) {
    const int co = (tid & 15) * 8;
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int64_t row = m + (tid >> 4) + 16 * it;
      const uint32_t off = ok && c0 + co < Cn ? (uint32_t)((row * Cn + c0 + co) * 2) : 0xfffffff0u;
      v[it] = bload16(r, off, 0);
    }
  }
  __device__ __forceinline__ void store(char* D, int tid, float* csum) const {
    const int co = (tid & 15) * 8;
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int r = (tid >> 4) + 16 * it;
      *reinterpret_cast<uint4*>(D + r * kWLdB + co * 2) = v[it];
      if (csum) {
        const uint32_t w[4] = {v[it].x, v[it].y, v[it].z, v[it].w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          csum[2 * u] += h16_to_f32(w[u] & 0xffffu);
          csum[2 * u + 1] += h16_to_f32(w[u] >> 16);
        }
      }
    }
  }
  static constexpr int kSumCols = 8, kRowLanes = 16;
};

// 32x32x16 operand fragment of columns [c, c+32) x rows [k, k+16) of a [row][col] bf16 image:
// lane l gets column c + l % 32, rows k + 8 (l / 32) + 0..7 (two ds_read_b64_tr_b16)
__device__ __forceinline__ h16x8 tr_frag(const char* img, int c, int k, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const char* base = img + (k + 8 * (g >> 1) + q) * kWLdB + (c + 16 * (g & 1) + 4 * p) * 2;
  typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base));
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + 4 * kWLdB));
  h16x8 f;
  const short s[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
  for (int u = 0; u < 8; ++u) f[u] = __builtin_bit_cast(h16, s[u]);
  return f;
}

// BUF (operands < 2 GiB): branch-free buffer loads, kWPF slices in flight in registers, the LDS
// image double-buffered with one barrier per slice (slice s + 1 is stored after slice s's
// barrier, beside slice s's MFMAs).  !BUF: the pointer loads, one slice ahead, two barriers.
constexpr int kWPF = 3;
template <typename TZ, typename TX, bool BUF = false>
__global__ __launch_bounds__(256) void wgrad_ex_kernel(const TZ* __restrict__ dZ,
                                                       const TX* __restrict__ X, int64_t M, int I,
                                                       int O, int64_t rows_per_chunk, int tiles_i,
                                                       int ntile, int total, int per_xcd,
                                                       float* __restrict__ partW,
                                                       float* __restrict__ partB) {
  __shared__ __attribute__((aligned(16))) char Zs[(BUF ? 2 : 1) * kWS * kWLdB];
  __shared__ __attribute__((aligned(16))) char Xs[(BUF ? 2 : 1) * kWS * kWLdB];
  __shared__ float bred[WStage<TZ>::kRowLanes][kXT + 1];
  const int L = blockIdx.x;
  const int t = (L & 7) * per_xcd + (L >> 3);  // XCD-aware: one chunk's tiles share an L2
  if (t >= total) return;
  const int chunk = t / ntile, tile = t % ntile;
  const int o0 = (tile / tiles_i) * kXT, i0 = (tile % tiles_i) * kXT;
  const int64_t mb = (int64_t)chunk * rows_per_chunk;
  const int64_t me = mb + rows_per_chunk < M ? mb + rows_per_chunk : M;
  const bool bias = partB != nullptr && i0 == 0;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, h = lane >> 5, l32 = lane & 31;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  float csum[WStage<TZ>::kSumCols];
#pragma unroll
  for (int u = 0; u < WStage<TZ>::kSumCols; ++u) csum[u] = 0.0f;
  auto mma = [&](const char* Zb, const char* Xb) {
#pragma unroll
    for (int ks = 0; ks < kWS / 16; ++ks) {
      h16x8 a[2], b[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        a[u] = tr_frag(Zb, wr * 64 + u * 32, ks * 16, lane);
        b[u] = tr_frag(Xb, wc * 64 + u * 32, ks * 16, lane);
      }
#pragma unroll
      for (int bm = 0; bm < 2; ++bm)
#pragma unroll
        for (int bn = 0; bn < 2; ++bn)
          acc[bm][bn] = mfma32_h16(a[bm], b[bn], acc[bm][bn]);
    }
  };
  if (BUF) {
    const rsrc_t rz = make_rsrc(dZ, (uint32_t)(M * O * (int64_t)sizeof(TZ)));
    const rsrc_t rx = make_rsrc(X, (uint32_t)(M * I * (int64_t)sizeof(TX)));
    // slices, padded to whole groups of kWPF: a padding slice loads zeros (out-of-range
    // offsets), so the loop body has no branch and the loads' counts stay exact
    const int ns = (int)((me - mb + kWS - 1) / kWS);
    const int np = (ns + kWPF - 1) / kWPF * kWPF;
    WStage<TZ> gz[kWPF];
    WStage<TX> gx[kWPF];
    float* cs = csum;  // column sums of every staged dZ slice (kept for the bias tiles only)
#pragma unroll
    for (int u = 0; u < kWPF; ++u) {
      gz[u].load_buf(rz, mb + (int64_t)u * kWS, o0, O, tid, u < ns);
      gx[u].load_buf(rx, mb + (int64_t)u * kWS, i0, I, tid, u < ns);
    }
    gz[0].store(Zs, tid, cs);
    gx[0].store(Xs, tid, nullptr);
    gz[0].load_buf(rz, mb + (int64_t)kWPF * kWS, o0, O, tid, kWPF < ns);
    gx[0].load_buf(rx, mb + (int64_t)kWPF * kWS, i0, I, tid, kWPF < ns);
    for (int s0 = 0; s0 < np; s0 += kWPF) {
#pragma unroll
      for (int u = 0; u < kWPF; ++u) {
        const int sl = s0 + u;
        __syncthreads();  // slice sl landed; slice sl - 1's readers are done
        const int un = (u + 1) % kWPF, nb = (sl + 1) & 1;
        gz[un].store(Zs + nb * kWS * kWLdB, tid, cs);
        gx[un].store(Xs + nb * kWS * kWLdB, tid, nullptr);
        const int ln = sl + 1 + kWPF;
        gz[un].load_buf(rz, mb + (int64_t)ln * kWS, o0, O, tid, ln < ns);
        gx[un].load_buf(rx, mb + (int64_t)ln * kWS, i0, I, tid, ln < ns);
        mma(Zs + (sl & 1) * kWS * kWLdB, Xs + (sl & 1) * kWS * kWLdB);
      }
    }
  } else {
  WStage<TZ> gz;
  WStage<TX> gx;
  gz.load(dZ, me, O, mb, o0, tid);
  gx.load(X, me, I, mb, i0, tid);
  for (int64_t k0 = mb; k0 < me; k0 += kWS) {
    gz.store(Zs, tid, bias ? csum : nullptr);
    gx.store(Xs, tid, nullptr);
    __syncthreads();
    if (k0 + kWS < me) {
      gz.load(dZ, me, O, k0 + kWS, o0, tid);
      gx.load(X, me, I, k0 + kWS, i0, tid);
    }
    mma(Zs, Xs);
    __syncthreads();
  }
  }
  float* pw = partW + (int64_t)chunk * O * I;
#pragma unroll
  for (int bn = 0; bn < 2; ++bn) {
    const int i = i0 + wc * 64 + bn * 32 + l32;
    if (i >= I) continue;
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + wr * 64 + bm * 32 + xrow(r, h);
        if (o < O) pw[(int64_t)o * I + i] = acc[bm][bn][r];
      }
  }
  if (bias) {  // column sums of the chunk: row lanes summed in fixed order
    constexpr int SC = WStage<TZ>::kSumCols, RL = WStage<TZ>::kRowLanes;
    const int rlane = tid / (kXT / SC), cb = (tid % (kXT / SC)) * SC;
#pragma unroll
    for (int u = 0; u < SC; ++u) bred[rlane][cb + u] = csum[u];
    __syncthreads();
    if (tid < kXT && o0 + tid < O) {
      float s = 0.0f;
#pragma unroll
      for (int r = 0; r < RL; ++r) s += bred[r][tid];
      partB[(int64_t)chunk * O + o0 + tid] = s;
    }
  }
}

// Chunk partials -> dW and db in one launch: a 256-thread block covers 64 float4 elements (of
// dW, then of db); wave w folds its quarter of the chunks in order into float64 (all its loads in
// flight together), and the four quarters meet in LDS in order -- a fixed reduction tree, so the
// gradient is deterministic.
constexpr int kCombLoads = 32;  // float4 loads in flight per thread
__global__ __launch_bounds__(256) void wgrad_ex_combine_kernel(
    const float4* __restrict__ partW, int64_t nW4, const float4* __restrict__ partB, int64_t nB4,
    int chunks, float4* __restrict__ outW, float4* __restrict__ outB) {
  __shared__ double red[3][64][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t q = (int64_t)blockIdx.x * 64 + lane;
  const bool isW = q < nW4;
  const bool valid = q < nW4 + nB4;
  const float4* part = isW ? partW : partB;
  const int64_t n4 = isW ? nW4 : nB4;
  const int64_t e = isW ? q : q - nW4;
  const int lo = (w * chunks) / 4, hi = ((w + 1) * chunks) / 4;
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  if (valid) {
    for (int c0 = lo; c0 < hi; c0 += kCombLoads) {
      float4 v[kCombLoads];
#pragma unroll
      for (int u = 0; u < kCombLoads; ++u)
        if (c0 + u < hi) v[u] = part[(int64_t)(c0 + u) * n4 + e];
#pragma unroll
      for (int u = 0; u < kCombLoads; ++u)
        if (c0 + u < hi) {
          s[0] += (double)v[u].x;
          s[1] += (double)v[u].y;
          s[2] += (double)v[u].z;
          s[3] += (double)v[u].w;
        }
    }
  }
  if (w) {
#pragma unroll
    for (int u = 0; u < 4; ++u) red[w - 1][lane][u] = s[u];
  }
  __syncthreads();
  if (w == 0 && valid) {
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] += red[k][lane][u];
    const float4 r = make_float4((float)s[0], (float)s[1], (float)s[2], (float)s[3]);
    if (isW) outW[e] = r; else outB[e] = r;
  }
}

constexpr int kWgradWG = 512;  // work-groups of one weight-gradient launch

struct WgradExPlan {
  int tiles_i, tiles_o, ntile, chunks, total, per_xcd;
  int64_t rows_per_chunk;
};

static WgradExPlan wgrad_ex_plan(int64_t M, int64_t I, int64_t O) {
  WgradExPlan p;
  p.tiles_i = (int)cdiv(I, kXT);
  p.tiles_o = (int)cdiv(O, kXT);
  p.ntile = p.tiles_i * p.tiles_o;
  int64_t chunks = cdiv(kWgradWG, p.ntile);  // ~2 workgroups per CU
  chunks = std::max<int64_t>(1, std::min<int64_t>(chunks, cdiv(M, 512)));
  p.rows_per_chunk = cdiv(cdiv(M, chunks), kWS) * kWS;
  p.chunks = (int)cdiv(M, p.rows_per_chunk);
  p.total = p.chunks * p.ntile;
  p.per_xcd = (int)cdiv(p.total, 8);
  return p;
}

static uint32_t drop_threshold(float p) {
  const double t = (double)p * 4294967296.0;
  return t <= 0.0 ? 0u : (t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t);
}

#define PCST_GEMM_EX(TA, TB, EPV)                                                                  \
  hipLaunchKernelGGL((gemm_ex_kernel<TA, TB, EPV>), dim3((unsigned)(8 * per)), dim3(256), 0, s,     \
                     static_cast<const TA*>(A), M, (int)K, static_cast<const TB*>(B), (int)O,        \
                     tiles_o, ntiles, per, args)

template <typename TA, typename TB>
static void launch_gemm_ex(int ep, const void* A, int64_t M, int64_t K, const void* B, int64_t O,
                           int tiles_o, int ntiles, int per, const GemmExArgs& args, hipStream_t s) {
  switch (ep) {
    case EP_F32: PCST_GEMM_EX(TA, TB, EP_F32); break;
    case EP_BF16: PCST_GEMM_EX(TA, TB, EP_BF16); break;
    case EP_RESID_DROP: PCST_GEMM_EX(TA, TB, EP_RESID_DROP); break;
    case EP_RELU_MASK: PCST_GEMM_EX(TA, TB, EP_RELU_MASK); break;
    case EP_ADD: PCST_GEMM_EX(TA, TB, EP_ADD); break;
    case EP_RESID_DROP16: PCST_GEMM_EX(TA, TB, EP_RESID_DROP16); break;
    case EP_ADD16: PCST_GEMM_EX(TA, TB, EP_ADD16); break;
    default: PCST_GEMM_EX(TA, TB, EP_COND); break;
  }
}
#undef PCST_GEMM_EX

#define PCST_GEMM_BF(EPV)                                                                          \
  if (fast)                                                                                        \
    hipLaunchKernelGGL((gemm_bf_kernel<EPV, true>), dim3((unsigned)(8 * per)), dim3(256), 0, s,     \
                       static_cast<const uint16_t*>(A), M, (int)K, static_cast<const uint16_t*>(B),  \
                       (int)O, tiles_o, ntiles, per, args);                                          \
  else                                                                                             \
    hipLaunchKernelGGL((gemm_bf_kernel<EPV, false>), dim3((unsigned)(8 * per)), dim3(256), 0, s,    \
                       static_cast<const uint16_t*>(A), M, (int)K, static_cast<const uint16_t*>(B),  \
                       (int)O, tiles_o, ntiles, per, args)

static void launch_gemm_bf(int ep, bool fast, const void* A, int64_t M, int64_t K, const void* B,
                           int64_t O, int tiles_o, int ntiles, int per, const GemmExArgs& args,
                           hipStream_t s) {
  switch (ep) {
    case EP_F32: PCST_GEMM_BF(EP_F32); break;
    case EP_BF16: PCST_GEMM_BF(EP_BF16); break;
    case EP_RESID_DROP: PCST_GEMM_BF(EP_RESID_DROP); break;
    case EP_RELU_MASK: PCST_GEMM_BF(EP_RELU_MASK); break;
    case EP_ADD: PCST_GEMM_BF(EP_ADD); break;
    case EP_RESID_DROP16: PCST_GEMM_BF(EP_RESID_DROP16); break;
    case EP_ADD16: PCST_GEMM_BF(EP_ADD16); break;
    default: PCST_GEMM_BF(EP_COND); break;
  }
}
#undef PCST_GEMM_BF

int gemm_ex_impl(const void* A, int a_bf16, int64_t M, int64_t K, const void* B, int b_bf16,
                 int64_t O, const float* bias, int relu, int epilogue, const void* aux,
                 uint64_t seed, float drop_p, int64_t group_rows, void* C, uint16_t* C2,
                 void* stream) {
  PCST_CHECK_ARG(M >= 0 && K > 0 && O > 0 && K < (1 << 20) && O < (1 << 20), "gemm_ex: bad shape");
  PCST_CHECK_ARG(epilogue >= EP_F32 && epilogue <= EP_ADD16, "gemm_ex: bad epilogue");
  PCST_CHECK_ARG(K % (a_bf16 ? 8 : 4) == 0 && K % (b_bf16 ? 8 : 4) == 0,
                 "gemm_ex: K must be a multiple of 8 (bf16 operand) or 4 (fp32 operand)");
  PCST_CHECK_ARG(O % 4 == 0 || epilogue == EP_F32 || epilogue == EP_BF16,
                 "gemm_ex: O must be a multiple of 4 for this epilogue");
  PCST_CHECK_ARG(drop_p >= 0.0f && drop_p < 1.0f, "gemm_ex: dropout p must be in [0, 1)");
  PCST_CHECK_ARG(epilogue != EP_COND || group_rows > 0, "gemm_ex: EP_COND needs group_rows > 0");
  if (M == 0) return PCST_OK;
  PCST_CHECK_ARG(A && B && (C || (epilogue == EP_COND && C2)), "gemm_ex: null pointer");
  PCST_CHECK_ARG(!C2 || epilogue == EP_F32 || epilogue == EP_RESID_DROP || epilogue == EP_COND ||
                     ep_drop_copy(epilogue),
                 "gemm_ex: C2 is not defined for this epilogue");
  PCST_CHECK_ARG(epilogue == EP_F32 || epilogue == EP_BF16 || aux, "gemm_ex: epilogue needs aux");
  PCST_CHECK_ARG(((uintptr_t)A | (uintptr_t)B | (uintptr_t)C | (uintptr_t)C2 | (uintptr_t)aux) % 16 == 0,
                 "gemm_ex: pointers must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  const int tiles_o = (int)cdiv(O, kXT);
  const int64_t nt = cdiv(M, kXT) * tiles_o;
  PCST_CHECK_ARG(nt < (1ll << 30), "gemm_ex: too many tiles");
  const int ntiles = (int)nt, per = (int)cdiv(nt, 8);
  GemmExArgs args;
  args.bias = bias;
  args.relu = relu;
  args.aux = aux;
  args.seed_lo = (uint32_t)seed;
  args.seed_hi = (uint32_t)(seed >> 32);
  args.thr = drop_threshold(drop_p);
  args.scale = 1.0f / (1.0f - drop_p);
  args.C = C;
  args.C2 = C2;
  args.group_rows = group_rows;
  const int64_t lim = 1ll << 31;
  if (a_bf16 && b_bf16 && K % kBK == 0 && M * K * 2 < lim && O * K * 2 < lim) {
    const bool fast = O % kXT == 0 && epilogue != EP_COND && M * O * 4 < lim;
    // register staging (round 4: 140 us at K = 256 against 146 / 173 for an LDS-DMA kernel with
    // three / four stages, since removed)
    launch_gemm_bf(epilogue, fast, A, M, K, B, O, tiles_o, ntiles, per, args, s);
  } else if (a_bf16 && b_bf16)
    launch_gemm_ex<uint16_t, uint16_t>(epilogue, A, M, K, B, O, tiles_o, ntiles, per, args, s);
  else if (a_bf16)
    launch_gemm_ex<uint16_t, float>(epilogue, A, M, K, B, O, tiles_o, ntiles, per, args, s);
  else if (b_bf16)
    launch_gemm_ex<float, uint16_t>(epilogue, A, M, K, B, O, tiles_o, ntiles, per, args, s);
  else
    launch_gemm_ex<float, float>(epilogue, A, M, K, B, O, tiles_o, ntiles, per, args, s);
  PCST_LAUNCH_CHECK("gemm_ex");
  return PCST_OK;
}

int dropout_grad_impl(const float* g, int64_t n, uint64_t seed, float drop_p, uint16_t* out,
                      void* stream) {
  PCST_CHECK_ARG(n >= 0 && n % 4 == 0, "dropout_grad_bf16: n must be a multiple of 4");
  PCST_CHECK_ARG(drop_p >= 0.0f && drop_p < 1.0f, "dropout_grad_bf16: p must be in [0, 1)");
  if (n == 0) return PCST_OK;
  PCST_CHECK_ARG(g && out && ((uintptr_t)g | (uintptr_t)out) % 16 == 0, "dropout_grad_bf16: bad pointer");
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(dropout_grad_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n4, 256), 4096)),
                     dim3(256), 0, as_stream(stream), reinterpret_cast<const float4*>(g), n4,
                     (uint32_t)seed, (uint32_t)(seed >> 32), drop_threshold(drop_p),
                     1.0f / (1.0f - drop_p), reinterpret_cast<uint2*>(out));
  PCST_LAUNCH_CHECK("dropout_grad_bf16");
  return PCST_OK;
}

int wgrad_ex_workspace_impl(int64_t M, int64_t I, int64_t O, size_t* bytes) {
  PCST_CHECK_ARG(M >= 0 && I > 0 && O > 0 && bytes, "linear_wgrad_ex_workspace_size: bad args");
  const WgradExPlan p = wgrad_ex_plan(std::max<int64_t>(M, 1), I, O);
  *bytes = sizeof(float) * (size_t)p.chunks * (size_t)(O * I + O);
  return PCST_OK;
}

int wgrad_ex_impl(const void* dZ, int dz_bf16, const void* X, int x_bf16, int64_t M, int64_t I,
                  int64_t O, float* dW, float* db, void* workspace, void* stream) {
  PCST_CHECK_ARG(M >= 0 && I > 0 && O > 0 && I < (1 << 20) && O < (1 << 20), "linear_wgrad_ex: bad shape");
  PCST_CHECK_ARG(I % 8 == 0 && O % 8 == 0, "linear_wgrad_ex: I and O must be multiples of 8");
  PCST_CHECK_ARG(dW && workspace && (M == 0 || (dZ && X)), "linear_wgrad_ex: null pointer");
  PCST_CHECK_ARG(((uintptr_t)dZ | (uintptr_t)X | (uintptr_t)dW) % 16 == 0, "linear_wgrad_ex: unaligned");
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    PCST_HIP(hipMemsetAsync(dW, 0, sizeof(float) * O * I, s), "memset");
    if (db) PCST_HIP(hipMemsetAsync(db, 0, sizeof(float) * O, s), "memset");
    return PCST_OK;
  }
  const WgradExPlan p = wgrad_ex_plan(M, I, O);
  float* partW = static_cast<float*>(workspace);
  float* partB = db ? partW + (int64_t)p.chunks * O * I : nullptr;
  const dim3 grid((unsigned)(8 * p.per_xcd));
  const int64_t lim = 1ll << 31;
#define PCST_WGRAD_EX(TZ, TX)                                                                     \
  do {                                                                                            \
  if (M * O * (int64_t)sizeof(TZ) < lim && M * I * (int64_t)sizeof(TX) < lim) \
    hipLaunchKernelGGL((wgrad_ex_kernel<TZ, TX, true>), grid, dim3(256), 0, s,                     \
                       static_cast<const TZ*>(dZ), static_cast<const TX*>(X), M, (int)I, (int)O,  \
                       p.rows_per_chunk, p.tiles_i, p.ntile, p.total, p.per_xcd, partW, partB);   \
  else                                                                                            \
    hipLaunchKernelGGL((wgrad_ex_kernel<TZ, TX, false>), grid, dim3(256), 0, s,                    \
                       static_cast<const TZ*>(dZ), static_cast<const TX*>(X), M, (int)I, (int)O,  \
                       p.rows_per_chunk, p.tiles_i, p.ntile, p.total, p.per_xcd, partW, partB); \
  } while (0)
  if (dz_bf16 && x_bf16)
    PCST_WGRAD_EX(uint16_t, uint16_t);
  else if (dz_bf16)
    PCST_WGRAD_EX(uint16_t, float);
  else if (x_bf16)
    PCST_WGRAD_EX(float, uint16_t);
  else
    PCST_WGRAD_EX(float, float);
#undef PCST_WGRAD_EX
  const int64_t nW4 = O * I / 4, nB4 = db ? O / 4 : 0;
  hipLaunchKernelGGL(wgrad_ex_combine_kernel, dim3((unsigned)cdiv(nW4 + nB4, 64)), dim3(256), 0, s,
                     reinterpret_cast<const float4*>(partW), nW4,
                     reinterpret_cast<const float4*>(partB), nB4, p.chunks,
                     reinterpret_cast<float4*>(dW), reinterpret_cast<float4*>(db));
  PCST_LAUNCH_CHECK("linear_wgrad_ex");
  return PCST_OK;
}

// ---- fused residual block forward (NoisePredictorFn's 16-bit residual stream):
//   h  = 16-bit(relu(x W1^T + b1))          [M, 512]   (written: the backward's mask and dW2 operand)
//   x' = 16-bit(x + Dropout(h W2^T + b2))   [M, 256]
// = gemm_ex EP_BF16 followed by EP_RESID_DROP16 in one pass over the rows: a work-group keeps its
// 128-row x tile in LDS for all four 128-wide hidden chunks and the residual add, and each chunk
// of h goes from the accumulators through LDS straight into the second product, so h is written
// once and never read back (the two-kernel form reads it again: 246 MB per block at M = 240 000).
// Bit-identical to the two gemm_ex calls: the same 32x32x16 MFMA roles (activation rows x weight
// rows), every output's k ascending in steps of 16, the same bias / ReLU / dropout / rounding.
// 512 threads = 8 waves, wave (wr, wc) = (w & 3, w >> 2): rows [32 wr, +32) x cols [64 wc, +64) of
// each 128 x 128 output tile.  The weights stream through a double-buffered 64-deep B slice:
// per chunk 4 slices of W1 (K = 256) then 2 x 2 slices of W2 (the two output halves, K = 128).
constexpr int kRbRows = 128;   // rows per tile (512 threads, 64-deep weight slices, one work-group per CU)
constexpr int kRbThreads = kRbRows * 4;          // (rows / 32) x 2 waves
constexpr int kRbNWR = kRbRows / 32;             // wave rows
constexpr int kRbK = kRbRows == 128 ? 64 : 32;   // weight slice depth
constexpr int kRbW1S = 256 / kRbK;               // first-product slices per hidden chunk (K = 256)
constexpr int kRbW2S = 128 / kRbK;               // second-product slices per output half (K = 128)
constexpr int kRbSPC = kRbW1S + 2 * kRbW2S;      // slices per chunk
constexpr int kRbSlices = 4 * kRbSPC;
constexpr int kRbPF = 4;       // weight slices in flight (round 4: 1 / 2 / 4 = 12.15 / 11.94 / 11.94 ms)
static_assert(kRbSlices % kRbPF == 0, "kRbPF must divide the slice count");
constexpr int kRbBLd = kRbK + 8;         // B image row (16-bit elements): 144 B, conflict-free
constexpr int kRbXLd = 256 + 8;          // x tile row: 528 B
constexpr int kRbHLd = 128 + 8;          // h chunk row: 272 B
constexpr int kRbXBytes = kRbRows * kRbXLd * 2;
constexpr int kRbHBytes = kRbRows * kRbHLd * 2;
constexpr int kRbBBytes = 128 * kRbBLd * 2;
constexpr int kRbLds = kRbXBytes + kRbHBytes + 2 * kRbBBytes + kRbRows * 4 * 4;  // + mask bits

struct RbArgs {
  const uint16_t* x;   // [M, 256]   the A operand: x (forward) / dD (backward)
  const uint16_t* w1;  // [512, 256] first product's weight rows: W1 / W2^T
  const float* b1;     // [512]      (forward only)
  const uint16_t* w2;  // [256, 512] second product's weight rows: W2 / W1^T
  const float* b2;     // [256]      (forward only)
  uint16_t* h;         // [M, 512]   written: h (forward) / dZ (backward)
  uint16_t* xo;        // [M, 256]   written: x' (forward) / g' (backward)
  const uint16_t* hm;  // [M, 512]   backward: the block's h (ReLU mask)
  const uint16_t* g;   // [M, 256]   backward: the residual gradient
  uint16_t* ddo;       // [M, 256]   backward, optional: dropout copy of g' (previous block's rate)
  uint32_t* hbo;       // [M, 16]    forward (v2), optional: the ReLU mask of h as bits (bit j of word
                       //            w of row m = [h[m, 32w + j] > 0])
  const uint32_t* hbi; // [M, 16]    backward, optional: that mask, read instead of h
  int64_t M;
  uint32_t seed_lo, seed_hi, thr;
  float scale;
};

// BWD = false: the forward above.  BWD = true: the block's backward products in the same pass,
//   dZ = 16-bit((dD W2) * [h > 0])          [M, 512]   (EP_RELU_MASK; written for dW1 = dZ^T x)
//   g' = 16-bit(g + dZ W1)                   [M, 256]   (EP_ADD16)
//   dD' = 16-bit(g' keep / (1 - p))          [M, 256]   (EP_ADD16's dropout copy, optional)
// with dD in the x tile, W2^T / W1^T as the two weight streams, each chunk's mask read into the
// chunk buffer two slices before its epilogue, and g loaded into the x tile once the last
// first-product slice has read it.  Bit-identical to the two gemm_ex calls (the fast epilogue's
// "+ 0" bias included: it turns a -0 product into +0).
// MB (backward): the ReLU mask from the forward's bit array (a.hbi, 2 KiB per 128-row chunk of
// 128 units) instead of h (32 KiB): 16x fewer mask bytes
template <bool BWD, bool MB = false>
// two waves per SIMD: two 256-thread work-groups per CU (64-row tiles), or one of 512 threads
__global__ __launch_bounds__(kRbThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void resblock_kernel(
    RbArgs a, int per_xcd, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  h16* Xs = reinterpret_cast<h16*>(smem);                                   // [rows][kRbXLd]
  h16* Hs = reinterpret_cast<h16*>(smem + kRbXBytes);                       // [rows][kRbHLd]
  h16* Bs0 = reinterpret_cast<h16*>(smem + kRbXBytes + kRbHBytes);          // [128][kRbBLd]
  h16* Bs1 = reinterpret_cast<h16*>(smem + kRbXBytes + kRbHBytes + kRbBBytes);
  uint32_t* Mb = reinterpret_cast<uint32_t*>(smem + kRbXBytes + kRbHBytes + 2 * kRbBBytes);  // [rows][4]
  const int L = blockIdx.x;
  const int t = (L & 7) * per_xcd + (L >> 3);
  if (t >= ntiles) return;
  const int64_t m0 = (int64_t)t * kRbRows;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid % kRbNWR, wc = wid / kRbNWR, h = lane >> 5, l32 = lane & 31;
  const int64_t M = a.M;
  // x tile -> Xs (rows past M read 0 through the buffer bound)
  const rsrc_t rx = make_rsrc(a.x, (uint32_t)(M * 256 * 2));
#pragma unroll
  for (int it = 0; it < 8; ++it) {  // rows x 32 chunks of 16 B
    const int q = it * kRbThreads + tid, r = q >> 5, cch = (q & 31) * 8;
    const uint4 v = bload16(rx, (uint32_t)(((m0 + r) * 256 + cch) * 2), 0);
    *reinterpret_cast<uint4*>(Xs + r * kRbXLd + cch) = v;
  }
  // B slice i: chunk c = i / 8, j = i % 8: j < 4 -> W1 rows [128c, +128) k [64j, +64);
  // j >= 4 -> W2 rows [128 oh, +128) k [128c + 64s, +64) with oh = (j - 4) / 2, s = (j - 4) % 2.
  // Thread -> (row tid / 4, 16 elements at (tid % 4) * 16): two 16-byte loads.
  const rsrc_t rw1 = make_rsrc(a.w1, 512u * 256u * 2u), rw2 = make_rsrc(a.w2, 256u * 512u * 2u);
  const int br = tid / (kRbK / 16), bk = (tid % (kRbK / 16)) * 16;
  auto load_slice = [&](int i, uint4& g0, uint4& g1) {
    const int c = i / kRbSPC, j = i % kRbSPC;
    uint32_t off;
    rsrc_t r;
    if (j < kRbW1S) {
      off = (uint32_t)(((128 * c + br) * 256 + kRbK * j + bk) * 2);
      r = rw1;
    } else {
      const int oh = (j - kRbW1S) / kRbW2S, sl = (j - kRbW1S) % kRbW2S;
      off = (uint32_t)(((128 * oh + br) * 512 + 128 * c + kRbK * sl + bk) * 2);
      r = rw2;
    }
    g0 = bload16(r, off, 0);
    g1 = bload16(r, off + 16, 0);
  };
  const rsrc_t rh = make_rsrc(a.h, (uint32_t)(M * 512 * 2));
  const rsrc_t rm = make_rsrc(BWD && !MB ? a.hm : nullptr, BWD && !MB ? (uint32_t)(M * 512 * 2) : 0u);
  const rsrc_t rmb = make_rsrc(MB ? a.hbi : nullptr, MB ? (uint32_t)(M * 16 * 4) : 0u);
  const rsrc_t rg = make_rsrc(BWD ? a.g : nullptr, BWD ? (uint32_t)(M * 256 * 2) : 0u);
  uint4 mk[4], gr[8];  // backward: a chunk's mask rows, the residual gradient tile
  uint32_t mbw = 0;    // MB: one word of a chunk's mask bits (row tid / 4, word tid % 4)
  // the lane's biases, loaded up front: a load issued at its use would wait (in-order vmcnt)
  // for every weight slice in flight as well
  float bb1[4][2], bb2[4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int bn = 0; bn < 2; ++bn) bb1[c][bn] = BWD ? 0.0f : a.b1[128 * c + 64 * wc + 32 * bn + l32];
#pragma unroll
  for (int u = 0; u < 4; ++u)
    bb2[u] = BWD ? 0.0f : a.b2[128 * (u >> 1) + 64 * wc + 32 * (u & 1) + l32];
  f32x16 acc1[2], acc2[4];
#pragma unroll
  for (int u = 0; u < 2; ++u) acc1[u] = f32x16{};
#pragma unroll
  for (int u = 0; u < 4; ++u) acc2[u] = f32x16{};
  // kRbPF register stages: slice s lives in g[s % kRbPF] from its load, kRbPF slices ahead,
  // until its LDS store, one slice ahead: iteration i stores slice i + 1 into the other buffer
  // after the barrier, so the store overlaps slice i's MFMAs instead of preceding them
  uint4 g[kRbPF][2];
#pragma unroll
  for (int u = 0; u < kRbPF; ++u) load_slice(u, g[u][0], g[u][1]);
  *reinterpret_cast<uint4*>(Bs0 + br * kRbBLd + bk) = g[0][0];
  *reinterpret_cast<uint4*>(Bs0 + br * kRbBLd + bk + 8) = g[0][1];
  if (kRbPF < kRbSlices) load_slice(kRbPF, g[0][0], g[0][1]);
  const int arow = 32 * wr + l32;
  for (int i0 = 0; i0 < kRbSlices; i0 += kRbPF)
#pragma unroll
  for (int u = 0; u < kRbPF; ++u) {
    const int i = i0 + u;
    h16* Bs = (i & 1) ? Bs1 : Bs0;
    __syncthreads();  // slice i landed; slice i - 1's (and the epilogue's) readers are done
    if (i + 1 < kRbSlices) {
      const int un = (u + 1) % kRbPF;
      h16* Bn = (i & 1) ? Bs0 : Bs1;
      *reinterpret_cast<uint4*>(Bn + br * kRbBLd + bk) = g[un][0];
      *reinterpret_cast<uint4*>(Bn + br * kRbBLd + bk + 8) = g[un][1];
      if (i + 1 + kRbPF < kRbSlices) load_slice(i + 1 + kRbPF, g[un][0], g[un][1]);
    }
    const int c = i / kRbSPC, j = i % kRbSPC;
    if (MB && j == 0 && tid < 4 * kRbRows) {
      // chunk c's mask bits: rows x 4 words (units 128c .. 128c + 127)
      const int r = tid >> 2, w = tid & 3;
      mbw = __builtin_amdgcn_raw_buffer_load_b32(rmb, (int)(((m0 + r) * 16 + 4 * c + w) * 4), 0, 0);
    }
    if (MB && j == kRbW1S - 2 && tid < 4 * kRbRows) Mb[tid] = mbw;  // read by the epilogue after the next barrier
    if (BWD && !MB && j == 0) {
      // chunk c's mask rows, coalesced (rows x 16 chunks of 16 B, 4 per thread)
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int q = it * kRbThreads + tid, r = q >> 4, cch = (q & 15) * 8;
        mk[it] = bload16(rm, (uint32_t)(((m0 + r) * 512 + 128 * c + cch) * 2), 0);
      }
    }
    if (BWD && !MB && j == kRbW1S - 2) {
      // -> Hs: the previous chunk's second-product readers passed this slice's barrier; the
      // epilogue reads it after the next one
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int q = it * kRbThreads + tid, r = q >> 4, cch = (q & 15) * 8;
        *reinterpret_cast<uint4*>(Hs + r * kRbHLd + cch) = mk[it];
      }
    }
    if (BWD && i == kRbSlices - 2 * kRbW2S) {
      // g tile: Xs is read for the last time by slice 27's first product
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int q = it * kRbThreads + tid, r = q >> 5, cch = (q & 31) * 8;
        gr[it] = bload16(rg, (uint32_t)(((m0 + r) * 256 + cch) * 2), 0);
      }
    }
    if (j == kRbW1S) {
      // chunk c's h (written to Hs by every wave after slice 8c + 3) -> global h, coalesced:
      // rows x 16 chunks of 16 B, 4 per thread
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int q = it * kRbThreads + tid, r = q >> 4, cch = (q & 15) * 8;
        const uint4 v = *reinterpret_cast<const uint4*>(Hs + r * kRbHLd + cch);
        const v4i32 vv = {(int)v.x, (int)v.y, (int)v.z, (int)v.w};
        __builtin_amdgcn_raw_buffer_store_b128(vv, rh, (int)(((m0 + r) * 512 + 128 * c + cch) * 2), 0, 0);
      }
    }
#pragma unroll
    for (int ks = 0; ks < kRbK / 16; ++ks) {
      h16x8 av, b[2];
      if (j < kRbW1S)
        av = *reinterpret_cast<const h16x8*>(Xs + arow * kRbXLd + kRbK * j + 16 * ks + 8 * h);
      else
        av = *reinterpret_cast<const h16x8*>(Hs + arow * kRbHLd + kRbK * ((j - kRbW1S) % kRbW2S) +
                                             16 * ks + 8 * h);
#pragma unroll
      for (int bn = 0; bn < 2; ++bn)
        b[bn] = *reinterpret_cast<const h16x8*>(Bs + (64 * wc + 32 * bn + l32) * kRbBLd + 16 * ks + 8 * h);
      if (j < kRbW1S) {
#pragma unroll
        for (int bn = 0; bn < 2; ++bn) acc1[bn] = mfma32_h16(av, b[bn], acc1[bn]);
      } else {
        const int oh = (j - kRbW1S) / kRbW2S;
#pragma unroll
        for (int bn = 0; bn < 2; ++bn) {
          if (oh == 0) acc2[bn] = mfma32_h16(av, b[bn], acc2[bn]);
          else acc2[2 + bn] = mfma32_h16(av, b[bn], acc2[2 + bn]);
        }
      }
    }
    if (j == kRbW1S - 1) {
      // chunk c's epilogue into Hs (read by every wave after the next slice's barrier): forward
      // h = 16-bit(relu(acc1 + b1)); backward dZ = 16-bit(acc1 + 0 masked by h > 0), the mask
      // read from the lane's own element.  The accumulators restart for chunk c + 1.
#pragma unroll
      for (int bn = 0; bn < 2; ++bn) {
        const int col = 64 * wc + 32 * bn + l32;
        const float bb = bb1[c][bn];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          h16* ph = Hs + (32 * wr + xrow(r, h)) * kRbHLd + col;
          float v = acc1[bn][r] + bb;
          if (MB) v = (Mb[(32 * wr + xrow(r, h)) * 4 + (col >> 5)] >> (col & 31)) & 1u ? v : 0.0f;
          else if (BWD) v = __builtin_bit_cast(int16_t, *ph) > 0 ? v : 0.0f;
          else v = fmaxf(v, 0.0f);
          *ph = (h16)v;
        }
        acc1[bn] = f32x16{};
      }
    }
  }
  if (BWD) {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int q = it * kRbThreads + tid, r = q >> 5, cch = (q & 31) * 8;
      *reinterpret_cast<uint4*>(Xs + r * kRbXLd + cch) = gr[it];
    }
  }
  __syncthreads();  // every wave's W2 products done; Xs is read below only by its owner lanes
  // forward x' = 16-bit(x + Dropout(acc2 + b2)); backward g' = 16-bit((acc2 + 0) + g): in place
  // in Xs, then a coalesced copy out
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int oh = u >> 1, bn = u & 1;
    const int col = 128 * oh + 64 * wc + 32 * bn + l32;
    const float bb = bb2[u];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * wr + xrow(r, h);
      float y = acc2[u][r] + bb;
      if (!BWD) {
        const uint32_t e = (uint32_t)((m0 + row) * 256 + col);
        const bool keep = drop_hash(a.seed_lo, a.seed_hi, (uint64_t)e) >= a.thr;
        y = keep ? y * a.scale : 0.0f;
      }
      h16* px = Xs + row * kRbXLd + col;
      y += (float)*px;
      *px = (h16)y;
    }
  }
  __syncthreads();
  const rsrc_t ro = make_rsrc(a.xo, (uint32_t)(M * 256 * 2));
  const rsrc_t rd = make_rsrc(BWD ? a.ddo : nullptr, BWD && a.ddo ? (uint32_t)(M * 256 * 2) : 0u);
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int q = it * kRbThreads + tid, r = q >> 5, cch = (q & 31) * 8;
    const uint4 v = *reinterpret_cast<const uint4*>(Xs + r * kRbXLd + cch);
    const int off = (int)(((m0 + r) * 256 + cch) * 2);
    __builtin_amdgcn_raw_buffer_store_b128(v4i32{(int)v.x, (int)v.y, (int)v.z, (int)v.w}, ro, off, 0, 0);
    if (BWD && a.ddo) {  // dD' = 16-bit(g' keep / (1 - p)), element e = (m0 + r) * 256 + cch + u
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      uint32_t o[4];
      const uint32_t e0 = (uint32_t)((m0 + r) * 256 + cch);
#pragma unroll
      for (int u2 = 0; u2 < 4; ++u2) {
        float d[2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const uint32_t e = e0 + 2 * u2 + s2;
          const bool keep = drop_hash(a.seed_lo, a.seed_hi, (uint64_t)e) >= a.thr;
          const float yr = h16_to_f32((w[u2] >> (16 * s2)) & 0xffffu);
          d[s2] = keep ? yr * a.scale : 0.0f;
        }
        h16x2 pk;
        pk[0] = (h16)d[0];
        pk[1] = (h16)d[1];
        o[u2] = __builtin_bit_cast(uint32_t, pk);
      }
      __builtin_amdgcn_raw_buffer_store_b128(v4i32{(int)o[0], (int)o[1], (int)o[2], (int)o[3]}, rd, off, 0, 0);
    }
  }
}

// ---- fused residual block, version 2 (the forward's kernel; its backward direction is slower than
// the kernel above -- DESIGN.md §6a; bit-identical to the kernel above and to
// gemm_ex): one
// wave per SIMD, each wave keeping its 64 rows' A operand (x / dD, 64 x 256) in registers for the
// whole block, so the MFMAs read only weight fragments from LDS (one 1 KiB fragment feeds two
// MFMAs, against 1.5 fragment reads per MFMA above).  The products run transposed,
//   h^T [512, rows] = W1 x^T,   x'^T [256, rows] = W2 h^T
// (A = a weight fragment, B = the rows), so each hidden chunk's accumulators (lane = row, registers
// = 16 hidden units) become the second product's B operand in registers: v_permlane32_swap moves
// the accumulator layout (lane half h holds units {4h..4h+3, 8+4h..8+4h+3} of a 16-block) to the
// operand layout (8h..8h+7), so every output still sums k ascending in steps of 16 with the same
// products as gemm_ex -- bit-identical, as the kernel above.  Work-group = 4 waves = 256 rows; the
// weights stream per 32-unit hidden chunk (32 fragments, 32 KiB: W1 rows [32c, +32) x K 256 and
// W2 rows 0..255 x k [32c, +32)) straight into LDS (global_load_lds from the row-major weights,
// 16 B per lane), double-buffered, one barrier per chunk.
// The forward runs on this kernel (245 vs 274 us at M = 245760, r04 a31); the backward on the
// kernel above (385 vs 337 us here: it is HBM-write bound).
constexpr int kR2Rows = 256;               // rows per work-group tile
constexpr int kR2Slab = 32 * 1024;         // one hidden chunk's fragments
constexpr int kR2Keep = 8 * 256 * 4;       // dropout keep bits: [8 output blocks][256 lanes] words
constexpr int kR2Slabs = 3;                // weight ring: chunk gc + 2 loads while gc runs
constexpr int kR2Lds = kR2Slabs * kR2Slab + (512 + 256) * 4 + kR2Keep;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

// exchange lo's lanes 32..63 with hi's lanes 0..31
__device__ __forceinline__ void swap_halves(uint32_t& lo, uint32_t& hi) {
  const auto r = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
  lo = r[0];
  hi = r[1];
}
// a 16-block of 16-bit values, 8 per lane: MFMA-output layout (lane half h: {4h..4h+3, 8+4h..})
// <-> operand layout (lane half h: 8h..8h+7); the same exchange both ways
__device__ __forceinline__ u32x4 relayout(u32x4 v) {
  uint32_t a = v[0], b = v[1], c = v[2], d = v[3];
  swap_halves(a, c);
  swap_halves(b, d);
  return u32x4{a, b, c, d};
}
__device__ __forceinline__ uint32_t pack16(float lo, float hi) {
  h16x2 p;
  p[0] = (h16)lo;
  p[1] = (h16)hi;
  return __builtin_bit_cast(uint32_t, p);
}
__device__ __forceinline__ h16x8 as_h16x8(u32x4 v) { return __builtin_bit_cast(h16x8, v); }
__device__ __forceinline__ u32x4 as_u32x4(uint4 v) { return u32x4{v.x, v.y, v.z, v.w}; }

// one group of four fragment reads (asm: invisible to the compiler's LDS-DMA tracking; each
// group's wait is a counted lgkmcnt tied to its registers, as the dma_read path above)
template <int G>
__device__ __forceinline__ void r2_read4(uint32_t a0, h16x8 (&v)[4]) {
  v[0] = dma_read<(4 * G + 0) * 1024>(a0);
  v[1] = dma_read<(4 * G + 1) * 1024>(a0);
  v[2] = dma_read<(4 * G + 2) * 1024>(a0);
  v[3] = dma_read<(4 * G + 3) * 1024>(a0);
}
__device__ __forceinline__ f32x4 r2_read_f4(uint32_t addr) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

__device__ __forceinline__ h16x8 r2_read_one(uint32_t addr, int off) {
  h16x8 v;
  if (__builtin_constant_p(off) && off >= 0 && off < 65536)
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
  else
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr + off));
  return v;
}
template <int N>
__device__ __forceinline__ void r2_wait1(h16x8& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "n"(N));
}
// LDS-DMA of 16 B per lane (buffer_load_dwordx4 ... lds) in asm: the compiler, which does not
// see it, then inserts no vmcnt wait for it before barriers (it would drain the chunk-after-next
// load at every chunk); its completion is covered by the explicit counted waits.  M0 (the LDS
// destination) is saved and restored around it.
__device__ __forceinline__ void r2_dma16(rsrc_t r, uint32_t voff, uint32_t soff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(r), "s"(lds), "s"(soff)
               : "memory");
}
// 16-byte buffer load in asm (the backward's mask rows): the compiler does not track it, so it
// inserts no wait for it (its own would also drain the weight DMA behind it); the chunk-end wait
// covers it, tied to these registers
__device__ __forceinline__ u32x4 r2_load16(rsrc_t r, uint32_t voff, uint32_t soff) {
  u32x4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(v) : "v"(voff), "s"(r), "s"(soff) : "memory");
  return v;
}
__device__ __forceinline__ uint32_t r2_read_u32(uint32_t addr) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ void r2_write_u32(uint32_t addr, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1" : : "v"(addr), "v"(v) : "memory");
}

// Persistent: one work-group per CU walks tiles t = blockIdx.x, + gridDim.x, ...; the weight
// stream runs on across tiles (every tile reads the same 16 chunks), and the next tile's A rows
// load into the registers the final epilogue frees, output block by output block.
template <bool BWD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void resblock2_kernel(
    RbArgs a, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sb1 = reinterpret_cast<float*>(smem + kR2Slabs * kR2Slab);  // [512]
  float* sb2 = sb1 + 512;                                             // [256]
  uint32_t* skeep = reinterpret_cast<uint32_t*>(sb2 + 256);           // [8][256]
  int t = blockIdx.x;
  if (t >= ntiles) return;
  const int G = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t M = a.M;
  // the dropout draws are made in the loop whether or not the backward writes its dropout copy:
  // a run-time condition there would cut the loop body into blocks the scheduler cannot
  // interleave with the MFMAs (measured: the backward 88 us slower with it)
  const bool drop = true;
  const bool ddo = BWD && a.ddo != nullptr;  // backward: the dropout copy is written
  if (!BWD) {
    sb1[tid] = a.b1[tid];
    sb1[256 + tid] = a.b1[256 + tid];
    sb2[tid] = a.b2[tid];
  }
  // chunk c's fragments -> slab: f < 16: W1 rows [32c, +32) k [16f, +16); f = 16 + 2 ob + kk:
  // W2 rows [32 ob, +32) k [32c + 16kk, +16).  Waves 0, 1 load the W1 half, 2, 3 the W2 half.
  const rsrc_t rw1 = make_rsrc(a.w1, 512u * 256u * 2u), rw2 = make_rsrc(a.w2, 256u * 512u * 2u);
  const uint32_t vw = wid < 2 ? (uint32_t)((l32 * 256 + 8 * h) * 2) : (uint32_t)((l32 * 512 + 8 * h) * 2);
  const rsrc_t rwv = wid < 2 ? rw1 : rw2;
  const uint32_t lds_slab0 = (uint32_t)(uintptr_t)smem + wid * 8 * 1024;
  auto fill = [&](int c, int slab) {
    const uint32_t dst = lds_slab0 + slab * kR2Slab;
    // wave-uniform: W1 fragment f at (32c * 256 + 16 f) * 2 bytes, W2 fragment (ob, kk) at
    // (32 ob * 512 + 32c + 16 kk) * 2
    const int base = wid < 2 ? (32 * c * 256 + 16 * 8 * wid) * 2 : (32 * 4 * (wid - 2) * 512 + 32 * c) * 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int so = base + (wid < 2 ? i * 32 : (32 * (i >> 1) * 512 + 16 * (i & 1)) * 2);
      r2_dma16(rwv, vw, __builtin_amdgcn_readfirstlane(so), __builtin_amdgcn_readfirstlane(dst + i * 1024));
    }
  };
  fill(0, 0);
  fill(1, 1);
  // the A rows in operand layout: xb[p][kb] = row r0 + 32p, k [16kb + 8h, +8).  Per-lane byte
  // offsets of the rows (the columns go into the instructions' offset fields or soffset; rows
  // past M fail the buffer range check: loads read 0, stores drop)
  const rsrc_t rx = make_rsrc(a.x, (uint32_t)(M * 256 * 2));
  int64_t r0 = (int64_t)t * kR2Rows + 64 * wid + l32;  // the lane's row in set 0 (set 1: +32)
  uint32_t v256 = (uint32_t)((r0 * 256 + 8 * h) * 2);  // set p: + p * 32 * 512 bytes
  uint32_t v512 = (uint32_t)((r0 * 512 + 8 * h) * 2);  // set p: + p * 32 * 1024 bytes
  uint32_t vrow16 = (uint32_t)(r0 * 64);               // the mask-bit row (16 words): + p * 32 * 64
  const uint32_t vstep256 = (uint32_t)G * kR2Rows * 256 * 2, vstep512 = (uint32_t)G * kR2Rows * 512 * 2;
  u32x4 xb[2][16];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int kb = 0; kb < 16; ++kb)
      xb[p][kb] = as_u32x4(bload16(rx, v256 + p * 16384 + kb * 32, 0));
  const rsrc_t rh = make_rsrc(a.h, (uint32_t)(M * 512 * 2));
  const rsrc_t rhb = make_rsrc(!BWD ? a.hbo : nullptr, !BWD && a.hbo ? (uint32_t)(M * 16 * 4) : 0u);
  const rsrc_t rm = make_rsrc(BWD ? a.hm : nullptr, BWD ? (uint32_t)(M * 512 * 2) : 0u);
  const rsrc_t ro = make_rsrc(a.xo, (uint32_t)(M * 256 * 2));
  const rsrc_t rg = make_rsrc(BWD ? a.g : nullptr, BWD ? (uint32_t)(M * 256 * 2) : 0u);
  const rsrc_t rd = make_rsrc(BWD ? a.ddo : nullptr, BWD && a.ddo ? (uint32_t)(M * 256 * 2) : 0u);
  u32x4 mk[2][2];  // backward: the next chunk's mask rows (h), operand layout
  if (BWD) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        mk[p][kk] = as_u32x4(bload16(rm, v512 + p * 32768 + kk * 32, 0));
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem + lane * 16;
  const uint32_t lb1 = (uint32_t)(uintptr_t)sb1 + 16 * h;  // + 4 (32c + 8q) bytes
  const uint32_t lb2 = (uint32_t)(uintptr_t)sb2 + 16 * h;  // + 4 (32ob + 8q) bytes
  const uint32_t lkeep = (uint32_t)(uintptr_t)skeep + 4 * tid;  // + 1024 ob bytes
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // slab 0 and the biases landed
  int gc = 0;  // chunks done by this work-group
  int slab0 = 0, slab2 = 2;  // the running chunk's slab, the slab chunk gc + 2 loads into
#pragma unroll 1
  for (;;) {
    const bool more = __builtin_amdgcn_readfirstlane(t + G < ntiles ? 1 : 0) != 0;  // another tile follows
    f32x16 acc2[8][2];
#pragma unroll
    for (int ob = 0; ob < 8; ++ob)
#pragma unroll
      for (int p = 0; p < 2; ++p) acc2[ob][p] = f32x16{};
    uint32_t keep2 = 0;  // the final epilogue's dropout draws, made in the loop's MFMA shadow
#pragma unroll 1
    for (int c = 0; c < 16; ++c, ++gc) {
      const uint32_t a0 = lds0 + slab0 * kR2Slab;
      uint32_t mbits = 0;  // backward: bit 16p + r = [h > 0] of accumulator element (p, r)
      if (BWD) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            const u32x4 v = relayout(mk[p][kk]);
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              const int r = 8 * kk + 2 * d;
              mbits |= (uint32_t)((int16_t)(v[d] & 0xffffu) > 0) << (16 * p + r);
              mbits |= (uint32_t)((int16_t)(v[d] >> 16) > 0) << (16 * p + r + 1);
            }
          }
      }
      // backward: the next chunk's mask rows (this tile's c + 1, or the next tile's chunk 0)
      if (BWD && (c + 1 < 16 || more)) {
        const uint32_t vn = c + 1 < 16 ? v512 : v512 + vstep512;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            mk[p][kk] = r2_load16(rm, vn + p * 32768 + kk * 32,
                                  __builtin_amdgcn_readfirstlane((uint32_t)(64 * ((c + 1) & 15))));
      }
      // the chunk after next (this tile's c + 2 or the next tile's: the same weights) into the
      // slab chunk gc - 1 used
      const bool fill2 = c + 2 < 16 || more;
      if (fill2) fill((c + 2) & 15, slab2);
      // the chunk's 32 fragments in order: f < 16 the first product (acc1[p] += W1[32c.., 16f..]
      // x^T, k ascending), f >= 16 the second (acc2[ob][p] += W2[32ob.., 32c + 16kk ..] h^T, f =
      // 16 + 2 ob + kk); a ring of four reads in flight, the wait for fragment f counted over the
      // reads issued after it (and the forward's bias reads, issued between fragments 15 and 16)
      h16x8 fr[4];
      fr[0] = dma_read<0>(a0);
      fr[1] = dma_read<1024>(a0);
      fr[2] = dma_read<2048>(a0);
      fr[3] = dma_read<3072>(a0);
      f32x16 acc1[2] = {f32x16{}, f32x16{}};
      f32x4 bq[4];
      u32x4 hb[2][2];
      const uint32_t e0 = (uint32_t)((r0 + 32 * (c & 1)) * 256 + 32 * (c >> 1) + 4 * h);
      if (!(c & 1)) keep2 = 0;
      // one fragment step (f a constant after unrolling): wait, MFMAs, next read
      auto frag_step = [&](const int f) __attribute__((always_inline)) {
        const int younger = (31 - f < 3 ? 31 - f : 3) + (!BWD && f >= 12 && f < 16 ? 4 : 0);
        if (younger == 7) r2_wait1<7>(fr[f & 3]);
        else if (younger == 3) r2_wait1<3>(fr[f & 3]);
        else if (younger == 2) r2_wait1<2>(fr[f & 3]);
        else if (younger == 1) r2_wait1<1>(fr[f & 3]);
        else r2_wait1<0>(fr[f & 3]);
        if (f < 16) {
#pragma unroll
          for (int p = 0; p < 2; ++p) acc1[p] = mfma32_h16(fr[f & 3], as_h16x8(xb[p][f]), acc1[p]);
        } else {
          const int ob = (f - 16) >> 1, kk = f & 1;
#pragma unroll
          for (int p = 0; p < 2; ++p) acc2[ob][p] = mfma32_h16(fr[f & 3], as_h16x8(hb[p][kk]), acc2[ob][p]);
          // the final epilogue's dropout draw for output block c / 2, row set c % 2, element
          // r = f - 16 (no data dependence: it fills the MFMA shadow): bit 16 (c & 1) + r
          if (drop) {
            const int r = f - 16;
            keep2 |= (uint32_t)(drop_hash(a.seed_lo, a.seed_hi, (uint64_t)(e0 + (r & 3) + 8 * (r >> 2))) >= a.thr)
                     << (16 * (c & 1) + r);
          }
        }
        // the MFMAs of fragment f stay ahead of the next read and wait (asm statements keep
        // their order; without this the scheduler sinks MFMAs below later waits)
        __builtin_amdgcn_sched_barrier(0);
        if (f + 4 < 32) fr[f & 3] = r2_read_one(a0, (f + 4) * 1024);
        if (!BWD && f == 11) {
#pragma unroll
          for (int q = 0; q < 4; ++q) bq[q] = r2_read_f4(lb1 + 4 * (32 * c + 8 * q));
        }
            };
#pragma unroll
      for (int f = 0; f < 16; ++f) frag_step(f);
        // epilogue: forward h = 16-bit(relu(acc1 + b1)), backward dZ = 16-bit((acc1 + 0)
        // [h > 0]); to the second product's operand layout and out to global (16 B per lane)
        if (!BWD) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]));
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          float v[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            v[r] = acc1[p][r] + (BWD ? 0.0f : bq[r >> 2][r & 3]);
            if (BWD) v[r] = (mbits >> (16 * p + r)) & 1u ? v[r] : 0.0f;
            else v[r] = fmaxf(v[r], 0.0f);
          }
          uint32_t mb = 0;  // forward: this lane's half of the row's mask word for chunk c
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            const u32x4 o = {pack16(v[8 * kk + 0], v[8 * kk + 1]), pack16(v[8 * kk + 2], v[8 * kk + 3]),
                             pack16(v[8 * kk + 4], v[8 * kk + 5]), pack16(v[8 * kk + 6], v[8 * kk + 7])};
            if (!BWD) {
              // [stored 16-bit value > 0] of accumulator register r = 8kk + 2d + s, unit
              // xrow(r, h) = ((2d + s) & 3) + 16kk + 8(d >> 1) + 4h of the chunk
#pragma unroll
              for (int d = 0; d < 4; ++d) {
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                  const uint32_t half16 = (o[d] >> (16 * s2)) & 0xffffu;
                  const int bit = ((2 * d + s2) & 3) + 16 * kk + 8 * (d >> 1);
                  mb |= (half16 - 1u < 0x7fffu ? 1u : 0u) << bit;  // 1 .. 0x7fff: positive
                }
              }
            }
            hb[p][kk] = relayout(o);
            if (true)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i32, hb[p][kk]), rh,
                                                     (int)(v512 + p * 32768 + kk * 32), 64 * c, 0);
          }
          if (!BWD) {  // the two halves' bits are disjoint: one word per row, lane half 0 stores
            // (branch-free: control flow here breaks the register allocation of the loop; the
            // other half's store, and every store when hbo is NULL, fails the range check)
            mb <<= 4 * h;  // lane half h holds units + 4h
            uint32_t lo = mb, hi = mb;
            swap_halves(lo, hi);  // lo: lanes 32-63 get lanes 0-31's; hi: lanes 0-31 get 32-63's
            const uint32_t word = mb | (h ? lo : hi);
            __builtin_amdgcn_raw_buffer_store_b32(word, rhb, (int)(h ? 0x7ffffff0u : vrow16 + p * 32 * 64),
                                                  4 * c, 0);
          }
        }
#pragma unroll
      for (int f = 16; f < 32; ++f) frag_step(f);
      if (drop && (c & 1)) r2_write_u32(lkeep + 1024 * (c >> 1), keep2);
      // this wave's DMA of the next chunk (issued a chunk ago) and backward its mask rows landed;
      // the chunk-after-next DMA (8) and this chunk's h stores (4) may still be in flight
      if (BWD) {  // tied to the mask registers it guards
        if (fill2)
          asm volatile("s_waitcnt vmcnt(12)" : "+v"(mk[0][0]), "+v"(mk[0][1]), "+v"(mk[1][0]), "+v"(mk[1][1]) : : "memory");
        else
          asm volatile("s_waitcnt vmcnt(4)" : "+v"(mk[0][0]), "+v"(mk[0][1]), "+v"(mk[1][0]), "+v"(mk[1][1]) : : "memory");
      } else {  // + the two mask-bit word stores after the h stores
        if (fill2) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      }
      __syncthreads();  // every wave's DMA of chunk gc + 1 landed; every wave is done with slab0
      slab0 = slab0 == kR2Slabs - 1 ? 0 : slab0 + 1;
      slab2 = slab2 == kR2Slabs - 1 ? 0 : slab2 + 1;
    }
    // final epilogue: forward x' = 16-bit(x + Dropout(acc2 + b2)); backward g' = 16-bit((acc2 +
    // 0) + g) and the dropout copy dD' = 16-bit(g' keep / (1 - p)); 16 B stores in operand
    // layout.  Output block ob frees xb[.][2ob, 2ob + 1], which then takes the next tile's rows.
    u32x4 gres[2][2][2];  // backward: the residual gradient of blocks ob, ob + 1 (ring of two)
    if (BWD) {
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          gres[0][p][kk] = as_u32x4(bload16(rg, v256 + p * 16384 + kk * 32, 0));
    }
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) {
      if (BWD && ob + 1 < 8) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            gres[(ob + 1) & 1][p][kk] = as_u32x4(bload16(rg, v256 + p * 16384 + (ob + 1) * 64 + kk * 32, 0));
      }
      // LDS addresses recomputed per block (opaque bases): hoisted out of the tile loop they
      // would be 40 loop-invariant registers
      uint32_t lb2o = lb2, lko = lkeep;
      asm volatile("" : "+v"(lb2o), "+v"(lko));
      f32x4 bq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) bq[q] = BWD ? f32x4{0.f, 0.f, 0.f, 0.f} : r2_read_f4(lb2o + 4 * (32 * ob + 8 * q));
      uint32_t kw = drop ? r2_read_u32(lko + 1024 * ob) : 0u;
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]), "+v"(kw));
#pragma unroll
      for (int p = 0; p < 2; ++p) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          // one 8-element piece at a time: no accumulator read hoisted ahead of its piece (the
          // scheduler would otherwise read a whole block's accumulators out at once)
          __builtin_amdgcn_sched_barrier(0);
          // x (forward) / g (backward) in the accumulator layout
          const u32x4 res = relayout(BWD ? gres[ob & 1][p][kk] : xb[p][2 * ob + kk]);
          uint32_t o[4], od[4];
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            float y2[2];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
              const int r = 8 * kk + 2 * d + s2;
              float y = acc2[ob][p][r] + bq[r >> 2][r & 3];
              if (!BWD) y = (kw >> (16 * p + r)) & 1u ? y * a.scale : 0.0f;
              y += h16_to_f32((res[d] >> (16 * s2)) & 0xffffu);
              y2[s2] = y;
            }
            o[d] = pack16(y2[0], y2[1]);
            if (BWD) {
              float dv[2];
#pragma unroll
              for (int s2 = 0; s2 < 2; ++s2) {
                const int r = 8 * kk + 2 * d + s2;
                const float yr = h16_to_f32((o[d] >> (16 * s2)) & 0xffffu);
                dv[s2] = (kw >> (16 * p + r)) & 1u ? yr * a.scale : 0.0f;
              }
              od[d] = pack16(dv[0], dv[1]);
            }
          }
          const int off = (int)(v256 + p * 16384 + ob * 64 + kk * 32);
          const u32x4 on = relayout(u32x4{o[0], o[1], o[2], o[3]});
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i32, on), ro, off, 0, 0);
          if (ddo) {
            const u32x4 dn = relayout(u32x4{od[0], od[1], od[2], od[3]});
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i32, dn), rd, off, 0, 0);
          }
        }
      }
    }
    if (more) {  // the next tile's A rows
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int kb = 0; kb < 16; ++kb)
          xb[p][kb] = as_u32x4(bload16(rx, v256 + vstep256 + p * 16384 + kb * 32, 0));
    }
    if (!more) break;
    t += G;
    r0 += (int64_t)G * kR2Rows;
    v256 += vstep256;
    v512 += vstep512;
    vrow16 += (uint32_t)G * kR2Rows * 64;
  }
}

// The forward on two waves per SIMD (round 6): resblock2_kernel's dataflow -- h^T = W1 x^T and
// x'^T = W2 h^T per 32-unit hidden chunk, the chunk's accumulators relaid into the second
// product's operand in registers, the weights streamed per chunk into a 3-slab LDS ring by
// LDS-DMA, one barrier per chunk -- with 8 waves of 32 rows instead of 4 of 64.  A wave's
// accumulators are then 128 registers instead of 256, so two waves share each SIMD and one wave's
// chunk epilogue (ReLU, the h and mask-bit stores, the relayout) and its waits on fragment reads
// run in the other's MFMA shadow, where one wave per SIMD left the MFMA pipe idle (resblock2:
// 192 us per launch with the stores, refills and draws all removed, against a 52 us MFMA floor).
// Every fragment read feeds one MFMA instead of two (twice resblock2's LDS reads: 256 KiB per
// chunk and CU).  Each output's products and their order are resblock2's: the same bits.
constexpr int kR3Threads = 512;               // 8 waves x 32 rows = a 256-row tile (kR2Rows)
constexpr int kR3Keep = 8 * kR3Threads * 4;   // dropout keep bits: [8 output blocks][512 threads]
constexpr int kR3Lds = kR2Slabs * kR2Slab + (512 + 256) * 4 + kR3Keep;

__global__ __launch_bounds__(kR3Threads) __attribute__((amdgpu_waves_per_eu(2, 2))) void resblock3_kernel(
    RbArgs a, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sb1 = reinterpret_cast<float*>(smem + kR2Slabs * kR2Slab);  // [512]
  float* sb2 = sb1 + 512;                                             // [256]
  uint32_t* skeep = reinterpret_cast<uint32_t*>(sb2 + 256);           // [8][512]
  int t = blockIdx.x;
  if (t >= ntiles) return;
  const int G = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t M = a.M;
  sb1[tid] = a.b1[tid];
  if (tid < 256) sb2[tid] = a.b2[tid];
  // chunk c's fragments -> slab: f < 16: W1 rows [32c, +32) k [16f, +16); f = 16 + 2 ob + kk:
  // W2 rows [32 ob, +32) k [32c + 16kk, +16).  Waves 0-3 load the W1 half (4 fragments each),
  // waves 4-7 the W2 half.
  const bool w1half = wid < 4;
  const rsrc_t rw1 = make_rsrc(a.w1, 512u * 256u * 2u), rw2 = make_rsrc(a.w2, 256u * 512u * 2u);
  const uint32_t vw = w1half ? (uint32_t)((l32 * 256 + 8 * h) * 2) : (uint32_t)((l32 * 512 + 8 * h) * 2);
  const rsrc_t rwv = w1half ? rw1 : rw2;
  const uint32_t lds_slab0 = (uint32_t)(uintptr_t)smem + (w1half ? 4 * wid : 16 + 4 * (wid - 4)) * 1024;
  auto fill = [&](int c, int slab) {
    const uint32_t dst = lds_slab0 + slab * kR2Slab;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 4 * (w1half ? wid : wid - 4) + i;
      const int so = w1half ? (32 * c * 256 + 16 * j) * 2 : (32 * (j >> 1) * 512 + 32 * c + 16 * (j & 1)) * 2;
      r2_dma16(rwv, vw, __builtin_amdgcn_readfirstlane(so), __builtin_amdgcn_readfirstlane(dst + i * 1024));
    }
  };
  fill(0, 0);
  fill(1, 1);
  // the A rows in operand layout: xb[kb] = row r0, k [16kb + 8h, +8)
  const rsrc_t rx = make_rsrc(a.x, (uint32_t)(M * 256 * 2));
  int64_t r0 = (int64_t)t * kR2Rows + 32 * wid + l32;
  uint32_t v256 = (uint32_t)((r0 * 256 + 8 * h) * 2);
  uint32_t v512 = (uint32_t)((r0 * 512 + 8 * h) * 2);
  uint32_t vrow16 = (uint32_t)(r0 * 64);
  const uint32_t vstep256 = (uint32_t)G * kR2Rows * 256 * 2, vstep512 = (uint32_t)G * kR2Rows * 512 * 2;
  u32x4 xb[16];
#pragma unroll
  for (int kb = 0; kb < 16; ++kb) xb[kb] = as_u32x4(bload16(rx, v256 + kb * 32, 0));
  const rsrc_t rh = make_rsrc(a.h, (uint32_t)(M * 512 * 2));
  const rsrc_t rhb = make_rsrc(a.hbo, a.hbo ? (uint32_t)(M * 16 * 4) : 0u);
  const rsrc_t ro = make_rsrc(a.xo, (uint32_t)(M * 256 * 2));
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem + lane * 16;
  const uint32_t lb1 = (uint32_t)(uintptr_t)sb1 + 16 * h;
  const uint32_t lb2 = (uint32_t)(uintptr_t)sb2 + 16 * h;
  const uint32_t lkeep = (uint32_t)(uintptr_t)skeep + 4 * tid;  // + 4 * 512 ob bytes
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // slabs 0, 1 and the biases landed
  int slab0 = 0, slab2 = 2;
#pragma unroll 1
  for (;;) {
    const bool more = __builtin_amdgcn_readfirstlane(t + G < ntiles ? 1 : 0) != 0;
    f32x16 acc2[8];
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) acc2[ob] = f32x16{};
    uint32_t keep2 = 0;
#pragma unroll 1
    for (int c = 0; c < 16; ++c) {
      const uint32_t a0 = lds0 + slab0 * kR2Slab;
      const bool fill2 = c + 2 < 16 || more;
      if (fill2) fill((c + 2) & 15, slab2);
      h16x8 fr[4];
      fr[0] = dma_read<0>(a0);
      fr[1] = dma_read<1024>(a0);
      fr[2] = dma_read<2048>(a0);
      fr[3] = dma_read<3072>(a0);
      f32x16 acc1 = f32x16{};
      f32x4 bq[4];
      u32x4 hb[2];
      const uint32_t e0 = (uint32_t)(r0 * 256 + 32 * (c >> 1) + 4 * h);
      if (!(c & 1)) keep2 = 0;
      auto frag_step = [&](const int f) __attribute__((always_inline)) {
        const int younger = (31 - f < 3 ? 31 - f : 3) + (f >= 12 && f < 16 ? 4 : 0);
        if (younger == 7) r2_wait1<7>(fr[f & 3]);
        else if (younger == 3) r2_wait1<3>(fr[f & 3]);
        else if (younger == 2) r2_wait1<2>(fr[f & 3]);
        else if (younger == 1) r2_wait1<1>(fr[f & 3]);
        else r2_wait1<0>(fr[f & 3]);
        if (f < 16) {
          acc1 = mfma32_h16(fr[f & 3], as_h16x8(xb[f]), acc1);
        } else {
          const int ob = (f - 16) >> 1, kk = f & 1;
          acc2[ob] = mfma32_h16(fr[f & 3], as_h16x8(hb[kk]), acc2[ob]);
          // the final epilogue's dropout draws, in the MFMA shadow: output block c / 2, element
          // r = 8 (c & 1) + (f - 16) / 2 at every second fragment (bit r of the block's word)
          if (!(f & 1)) {
            const int r = 8 * (c & 1) + ((f - 16) >> 1);
            keep2 |= (uint32_t)(drop_hash(a.seed_lo, a.seed_hi, (uint64_t)(e0 + (r & 3) + 8 * (r >> 2))) >= a.thr)
                     << r;
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (f + 4 < 32) fr[f & 3] = r2_read_one(a0, (f + 4) * 1024);
        if (f == 11) {
#pragma unroll
          for (int q = 0; q < 4; ++q) bq[q] = r2_read_f4(lb1 + 4 * (32 * c + 8 * q));
        }
      };
#pragma unroll
      for (int f = 0; f < 16; ++f) frag_step(f);
      // chunk epilogue: h = 16-bit(relu(acc1 + b1)), to the second product's operand layout and
      // out to global (16 B per lane), and the chunk's ReLU mask word of the row
      asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]));
      {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = fmaxf(acc1[r] + bq[r >> 2][r & 3], 0.0f);
        uint32_t mb = 0;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const u32x4 o = {pack16(v[8 * kk + 0], v[8 * kk + 1]), pack16(v[8 * kk + 2], v[8 * kk + 3]),
                           pack16(v[8 * kk + 4], v[8 * kk + 5]), pack16(v[8 * kk + 6], v[8 * kk + 7])};
#pragma unroll
          for (int d = 0; d < 4; ++d) {
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
              const uint32_t half16 = (o[d] >> (16 * s2)) & 0xffffu;
              const int bit = ((2 * d + s2) & 3) + 16 * kk + 8 * (d >> 1);
              mb |= (half16 - 1u < 0x7fffu ? 1u : 0u) << bit;  // 1 .. 0x7fff: positive
            }
          }
          hb[kk] = relayout(o);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i32, hb[kk]), rh, (int)(v512 + kk * 32),
                                                 64 * c, 0);
        }
        mb <<= 4 * h;  // lane half h holds units + 4h; the halves' bits are disjoint
        uint32_t lo = mb, hi = mb;
        swap_halves(lo, hi);
        const uint32_t word = mb | (h ? lo : hi);
        __builtin_amdgcn_raw_buffer_store_b32(word, rhb, (int)(h ? 0x7ffffff0u : vrow16), 4 * c, 0);
      }
#pragma unroll
      for (int f = 16; f < 32; ++f) frag_step(f);
      if (c & 1) r2_write_u32(lkeep + 4 * kR3Threads * (c >> 1), keep2);
      // this wave's DMA of the next chunk (issued a chunk ago) landed; the chunk-after-next DMA
      // (4), this chunk's h stores (2) and its mask word (1) may still be in flight
      if (fill2) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      __syncthreads();  // every wave's DMA of the next chunk landed; every wave is done with slab0
      slab0 = slab0 == kR2Slabs - 1 ? 0 : slab0 + 1;
      slab2 = slab2 == kR2Slabs - 1 ? 0 : slab2 + 1;
    }
    // final epilogue: x' = 16-bit(x + Dropout(acc2 + b2)), 16 B stores in operand layout
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) {
      uint32_t lb2o = lb2, lko = lkeep;
      asm volatile("" : "+v"(lb2o), "+v"(lko));
      f32x4 bq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) bq[q] = r2_read_f4(lb2o + 4 * (32 * ob + 8 * q));
      uint32_t kw = r2_read_u32(lko + 4 * kR3Threads * ob);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]), "+v"(kw));
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        __builtin_amdgcn_sched_barrier(0);
        const u32x4 res = relayout(xb[2 * ob + kk]);  // x in the accumulator layout
        uint32_t o[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          float y2[2];
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const int r = 8 * kk + 2 * d + s2;
            float y = acc2[ob][r] + bq[r >> 2][r & 3];
            y = (kw >> r) & 1u ? y * a.scale : 0.0f;
            y += h16_to_f32((res[d] >> (16 * s2)) & 0xffffu);
            y2[s2] = y;
          }
          o[d] = pack16(y2[0], y2[1]);
        }
        const u32x4 on = relayout(u32x4{o[0], o[1], o[2], o[3]});
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i32, on), ro, (int)(v256 + ob * 64 + kk * 32),
                                               0, 0);
      }
    }
    if (!more) break;
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) xb[kb] = as_u32x4(bload16(rx, v256 + vstep256 + kb * 32, 0));
    t += G;
    r0 += (int64_t)G * kR2Rows;
    v256 += vstep256;
    v512 += vstep512;
    vrow16 += (uint32_t)G * kR2Rows * 64;
  }
}

// ---- batched weight casts: every 2-D weight of a step to the 16-bit format (optionally
// transposed) in one launch, instead of one cast (and, transposed, one more copy) per tensor
struct CastBatch {
  const float* src[kCastMax];
  uint16_t* dst[kCastMax];
  int32_t rows[kCastMax], cols[kCastMax], trans[kCastMax];
  int n;
};
__global__ __launch_bounds__(256) void cast16_batch_kernel(CastBatch cb) {
  const int m = blockIdx.y;
  const float* S = cb.src[m];
  uint16_t* D = cb.dst[m];
  const int R = cb.rows[m], C = cb.cols[m];
  const int64_t n = (int64_t)R * C;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const h16 v = (h16)S[e];
    const int64_t o = cb.trans[m] ? (e % C) * R + e / C : e;  // [R,C] -> [C,R]
    D[o] = __builtin_bit_cast(uint16_t, v);
  }
}

int cast16_batch_impl(const float* const* src, uint16_t* const* dst, const int32_t* rows,
                      const int32_t* cols, const int32_t* trans, int n, void* stream) {
  PCST_CHECK_ARG(n >= 0 && n <= kCastMax, "cast16_batch: 0..64 tensors");
  if (n == 0) return PCST_OK;
  CastBatch cb;
  int64_t most = 0;
  for (int i = 0; i < n; ++i) {
    PCST_CHECK_ARG(rows[i] >= 0 && cols[i] >= 0 && ((src[i] && dst[i]) || (int64_t)rows[i] * cols[i] == 0),
                   "cast16_batch: bad tensor");
    cb.src[i] = src[i];
    cb.dst[i] = dst[i];
    cb.rows[i] = rows[i];
    cb.cols[i] = cols[i];
    cb.trans[i] = trans[i] ? 1 : 0;
    most = std::max<int64_t>(most, (int64_t)rows[i] * cols[i]);
  }
  cb.n = n;
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(most, 256), 64));
  hipLaunchKernelGGL(cast16_batch_kernel, dim3(gx, (unsigned)n), dim3(256), 0, as_stream(stream), cb);
  PCST_LAUNCH_CHECK("cast16_batch");
  return PCST_OK;
}

// persistent grid of the fused residual-block kernel: one work-group per CU of the current device
// (queried per call: the library keeps no process-global state)
static int r2_grid() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
}

int resblock_fwd_impl(const uint16_t* x, int64_t M, const uint16_t* w1, const float* b1,
                      const uint16_t* w2, const float* b2, uint64_t seed, float drop_p,
                      uint16_t* h, uint16_t* xo, uint32_t* hbits, void* stream) {
  PCST_CHECK_ARG(M >= 0 && M * 512 * 2 < (1ll << 31), "resblock_fwd: bad M");
  PCST_CHECK_ARG(drop_p >= 0.0f && drop_p < 1.0f, "resblock_fwd: dropout p must be in [0, 1)");
  if (M == 0) return PCST_OK;
  PCST_CHECK_ARG(x && w1 && b1 && w2 && b2 && h && xo, "resblock_fwd: null pointer");
  PCST_CHECK_ARG(((uintptr_t)x | (uintptr_t)w1 | (uintptr_t)w2 | (uintptr_t)h | (uintptr_t)xo) % 16 == 0,
                 "resblock_fwd: pointers must be 16-byte aligned");
  PCST_CHECK_ARG(xo != x, "resblock_fwd: out of place only");
  RbArgs a;
  a.x = x; a.w1 = w1; a.b1 = b1; a.w2 = w2; a.b2 = b2; a.h = h; a.xo = xo; a.M = M;
  a.seed_lo = (uint32_t)seed;
  a.seed_hi = (uint32_t)(seed >> 32);
  a.thr = drop_threshold(drop_p);
  a.scale = 1.0f / (1.0f - drop_p);
  a.hm = nullptr; a.g = nullptr; a.ddo = nullptr;
  a.hbo = hbits; a.hbi = nullptr;
  const int ntiles = (int)cdiv(M, kR2Rows);
#ifndef PCST_RB_FWD_V2  // experiment builds: 1 = the one-wave-per-SIMD forward (resblock2_kernel)
#define PCST_RB_FWD_V2 0
#endif
  if (PCST_RB_FWD_V2)
    hipLaunchKernelGGL(resblock2_kernel<false>, dim3((unsigned)std::min(ntiles, r2_grid())), dim3(256),
                       kR2Lds, as_stream(stream), a, ntiles);
  else
    hipLaunchKernelGGL(resblock3_kernel, dim3((unsigned)std::min(ntiles, r2_grid())), dim3(kR3Threads),
                       kR3Lds, as_stream(stream), a, ntiles);
  PCST_LAUNCH_CHECK("resblock_fwd");
  return PCST_OK;
}

int resblock_bwd_impl(const uint16_t* dd, int64_t M, const uint16_t* w2t, const uint16_t* w1t,
                      const uint16_t* h, const uint16_t* g, uint64_t seed, float drop_p,
                      uint16_t* dz, uint16_t* g_out, uint16_t* dd_out, const uint32_t* hbits,
                      void* stream) {
  PCST_CHECK_ARG(M >= 0 && M * 512 * 2 < (1ll << 31), "resblock_bwd: bad M");
  PCST_CHECK_ARG(drop_p >= 0.0f && drop_p < 1.0f, "resblock_bwd: dropout p must be in [0, 1)");
  if (M == 0) return PCST_OK;
  PCST_CHECK_ARG(dd && w2t && w1t && (h || hbits) && g && dz && g_out, "resblock_bwd: null pointer");
  PCST_CHECK_ARG(((uintptr_t)hbits % 4) == 0, "resblock_bwd: hbits must be 4-byte aligned");
  PCST_CHECK_ARG(((uintptr_t)dd | (uintptr_t)w2t | (uintptr_t)w1t | (uintptr_t)h | (uintptr_t)g |
                  (uintptr_t)dz | (uintptr_t)g_out | (uintptr_t)dd_out) % 16 == 0,
                 "resblock_bwd: pointers must be 16-byte aligned");
  PCST_CHECK_ARG(g_out != dd && dz != h, "resblock_bwd: out of place only");
  RbArgs a;
  a.x = dd; a.w1 = w2t; a.b1 = nullptr; a.w2 = w1t; a.b2 = nullptr; a.h = dz; a.xo = g_out;
  a.hm = h; a.g = g; a.ddo = dd_out; a.M = M;
  a.hbo = nullptr; a.hbi = hbits;
  a.seed_lo = (uint32_t)seed;
  a.seed_hi = (uint32_t)(seed >> 32);
  a.thr = drop_threshold(drop_p);
  a.scale = 1.0f / (1.0f - drop_p);
  const int ntiles = (int)cdiv(M, kRbRows), per = (int)cdiv(ntiles, 8);
  if (hbits)
    hipLaunchKernelGGL((resblock_kernel<true, true>), dim3((unsigned)(8 * per)), dim3(kRbThreads), kRbLds,
                       as_stream(stream), a, per, ntiles);
  else
    hipLaunchKernelGGL(resblock_kernel<true>, dim3((unsigned)(8 * per)), dim3(kRbThreads), kRbLds,
                       as_stream(stream), a, per, ntiles);
  PCST_LAUNCH_CHECK("resblock_bwd");
  return PCST_OK;
}

}  // namespace PCST_H16_NS
}  // namespace pcst

#if !PCST_H16_F16
// C entry points (include/pcst.h): the 16-bit storage flags (a_bf16, ...) mark 16-bit operands,
// `f16` picks their format -- 0 bf16, 1 fp16 -- for the operands rounded while staged too.
extern "C" int pcst_gemm_ex(const void* A, int a_bf16, int64_t M, int64_t K, const void* B,
                            int b_bf16, int64_t O, const float* bias, int relu, int epilogue,
                            const void* aux, uint64_t seed, float drop_p, int64_t group_rows,
                            void* C, uint16_t* C2, int f16, void* stream) {
  return f16 ? pcst::f16m::gemm_ex_impl(A, a_bf16, M, K, B, b_bf16, O, bias, relu, epilogue, aux,
                                        seed, drop_p, group_rows, C, C2, stream)
             : pcst::bf16m::gemm_ex_impl(A, a_bf16, M, K, B, b_bf16, O, bias, relu, epilogue, aux,
                                         seed, drop_p, group_rows, C, C2, stream);
}

extern "C" int pcst_resblock_fwd16(const uint16_t* x, int64_t M, const uint16_t* w1, const float* b1,
                                   const uint16_t* w2, const float* b2, uint64_t seed, float drop_p,
                                   uint16_t* h, uint16_t* x_out, uint32_t* hbits, int f16, void* stream) {
  return f16 ? pcst::f16m::resblock_fwd_impl(x, M, w1, b1, w2, b2, seed, drop_p, h, x_out, hbits, stream)
             : pcst::bf16m::resblock_fwd_impl(x, M, w1, b1, w2, b2, seed, drop_p, h, x_out, hbits, stream);
}

extern "C" int pcst_cast16_batch(const float* const* src, uint16_t* const* dst, const int32_t* rows,
                                 const int32_t* cols, const int32_t* transpose, int n, int f16,
                                 void* stream) {
  return f16 ? pcst::f16m::cast16_batch_impl(src, dst, rows, cols, transpose, n, stream)
             : pcst::bf16m::cast16_batch_impl(src, dst, rows, cols, transpose, n, stream);
}

extern "C" int pcst_resblock_bwd16(const uint16_t* dd, int64_t M, const uint16_t* w2t,
                                   const uint16_t* w1t, const uint16_t* h, const uint16_t* g,
                                   uint64_t seed, float drop_p, uint16_t* dz, uint16_t* g_out,
                                   uint16_t* dd_out, const uint32_t* hbits, int f16, void* stream) {
  return f16 ? pcst::f16m::resblock_bwd_impl(dd, M, w2t, w1t, h, g, seed, drop_p, dz, g_out, dd_out, hbits, stream)
             : pcst::bf16m::resblock_bwd_impl(dd, M, w2t, w1t, h, g, seed, drop_p, dz, g_out, dd_out, hbits, stream);
}

extern "C" int pcst_dropout_grad_bf16(const float* g, int64_t n, uint64_t seed, float drop_p,
                                      uint16_t* out, int f16, void* stream) {
  return f16 ? pcst::f16m::dropout_grad_impl(g, n, seed, drop_p, out, stream)
             : pcst::bf16m::dropout_grad_impl(g, n, seed, drop_p, out, stream);
}

extern "C" int pcst_linear_wgrad_ex_workspace_size(int64_t M, int64_t I, int64_t O, size_t* bytes) {
  return pcst::bf16m::wgrad_ex_workspace_impl(M, I, O, bytes);  // the same plan in both formats
}

extern "C" int pcst_linear_wgrad_ex(const void* dZ, int dz_bf16, const void* X, int x_bf16,
                                    int64_t M, int64_t I, int64_t O, float* dW, float* db,
                                    void* workspace, int f16, void* stream) {
  return f16 ? pcst::f16m::wgrad_ex_impl(dZ, dz_bf16, X, x_bf16, M, I, O, dW, db, workspace, stream)
             : pcst::bf16m::wgrad_ex_impl(dZ, dz_bf16, X, x_bf16, M, I, O, dW, db, workspace, stream);
}
#endif
