// SetAbstraction grouped MLP + max-pool (models/pointnet2_encoder.py:106-112) and the other
// small per-point linear layers of the style encoder, on exact-f32 MFMA
// (v_mfma_f32_32x32x2_f32: a k-ordered fmaf chain, so results match an fp32 reference to
// summation order only).
//
//   Y[m, o] = act(scale[o] * (X[m, :] . W[o, :]) + shift[o])      (Conv2d 1x1 + BN + ReLU)
//   pooled: Y[g, o] = max over rows m in group g (g = m / ns)      (torch.max(points, 3))
//
// Eval-mode BN is folded into (scale, shift) by the host.  Train-mode BN needs batch
// statistics of the pre-BN activations: linear pass with (1, bias), channel_stats (deterministic
// two-level float64 reduction), then affine_act (+pool).
//
// Tile: 64 rows x 64 channels per 256-thread workgroup (2x2 waves of 32x32), K staged through
// LDS in 32-deep slices (rows padded to 33 floats: conflict-free column reads).
// Max-pool after ReLU: every candidate is >= 0, so the max is an order-independent
// atomicMax on the float bits into a zero-initialised output.
#include "common.h"

namespace pcst {

typedef __attribute__((ext_vector_type(16))) float f32x16;
constexpr int kBM = 64, kBN = 64, kBK = 32, kLd = kBK + 1;

__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <bool POOL>
__global__ __launch_bounds__(256) void pw_linear_kernel(const float* __restrict__ X, int64_t M,
                                                        int K, const float* __restrict__ W, int O,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ shift, int relu,
                                                        int64_t ns, float* __restrict__ Y) {
  __shared__ float As[kBM][kLd];
  __shared__ float Bs[kBN][kLd];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, h = lane >> 5, l32 = lane & 31;
  const int64_t m0 = (int64_t)blockIdx.x * kBM;
  const int o0 = blockIdx.y * kBN;
  f32x16 acc = f32x16{};
  for (int k0 = 0; k0 < K; k0 += kBK) {
    for (int e = tid; e < kBM * kBK; e += 256) {
      const int r = e / kBK, k = e % kBK;
      const int64_t m = m0 + r;
      As[r][k] = (m < M && k0 + k < K) ? X[m * K + k0 + k] : 0.0f;
      const int o = o0 + r;
      Bs[r][k] = (o < O && k0 + k < K) ? W[(int64_t)o * K + k0 + k] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kBK; kk += 2) {
      const float a = As[wr * 32 + l32][kk + h];
      const float b = Bs[wc * 32 + l32][kk + h];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  // C layout: column (channel) = lane & 31, row (point) = crow(r, h)
  const int o = o0 + wc * 32 + l32;
  const float sc = (o < O && scale) ? scale[o] : 1.0f;
  const float sh = (o < O && shift) ? shift[o] : 0.0f;
  const int64_t mb = m0 + wr * 32;
  if (!POOL) {
    if (o < O) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = mb + crow(r, h);
        float v = fmaf(acc[r], sc, sh);
        if (relu) v = fmaxf(v, 0.0f);
        if (m < M) Y[m * O + o] = v;
      }
    }
    return;
  }
  // pooled (relu required): groups of ns consecutive rows
  if (ns % 32 == 0) {
    float mx = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t m = mb + crow(r, h);
      const float v = fmaxf(fmaf(acc[r], sc, sh), 0.0f);
      if (m < M) mx = fmaxf(mx, v);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    if (h == 0 && o < O && mb < M)
      atomicMax(reinterpret_cast<unsigned int*>(&Y[(mb / ns) * O + o]), __float_as_uint(mx));
  } else if (o < O) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t m = mb + crow(r, h);
      const float v = fmaxf(fmaf(acc[r], sc, sh), 0.0f);
      if (m < M) atomicMax(reinterpret_cast<unsigned int*>(&Y[(m / ns) * O + o]), __float_as_uint(v));
    }
  }
}

// Deterministic per-channel statistics of Z [M, O]: one pass of float64 partial sums and sums
// of squares over row chunks (an fp32 value's square is exact in float64), then a fixed-order
// combine.  mean[o], var[o] = E[z^2] - mean^2 (biased, as BatchNorm normalises with; in float64
// the cancellation costs ~1e-16 * (mean^2 + var) / var relative, far below the fp32 outputs).
// A 256-thread block covers TQ = min(O / W, 64) groups of W channels (W = 4: float4 loads when
// O % 4 == 0) x (256 / TQ) row lanes of one chunk; the lanes fold in a fixed order.
constexpr int kStatChunks = 256;

template <int W>
__global__ __launch_bounds__(256) void channel_partial_kernel(const float* __restrict__ Z, int64_t M,
                                                              int O, double* __restrict__ part) {
  const int G = O / W;  // channel groups (O % W == 0)
  const int TQ = G < 64 ? G : 64;
  const int RL = 256 / TQ;
  const int cg = threadIdx.x % TQ, rl = threadIdx.x / TQ;
  const int o0 = (blockIdx.y * TQ + cg) * W;
  const int chunk = blockIdx.x;
  const int64_t per = (M + kStatChunks - 1) / kStatChunks;
  const int64_t a = chunk * per, e = a + per < M ? a + per : M;
  __shared__ double s1[W][256], s2[W][256];
  double t1[W], t2[W];
#pragma unroll
  for (int w = 0; w < W; ++w) t1[w] = t2[w] = 0.0;
  if (rl < RL && o0 < O) {
    for (int64_t m = a + rl; m < e; m += RL) {
      float v[W];
      if constexpr (W == 4) {
        const float4 q = *reinterpret_cast<const float4*>(Z + m * O + o0);
        v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
      } else {
        v[0] = Z[m * O + o0];
      }
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const double d = (double)v[w];
        t1[w] += d;
        t2[w] = fma(d, d, t2[w]);
      }
    }
  }
#pragma unroll
  for (int w = 0; w < W; ++w) {
    s1[w][threadIdx.x] = t1[w];
    s2[w][threadIdx.x] = t2[w];
  }
  __syncthreads();
  if (rl == 0 && o0 < O) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
      double u1 = 0.0, u2 = 0.0;
      for (int q = 0; q < RL; ++q) {
        u1 += s1[w][q * TQ + cg];
        u2 += s2[w][q * TQ + cg];
      }
      part[((int64_t)chunk * 2 + 0) * O + o0 + w] = u1;
      part[((int64_t)chunk * 2 + 1) * O + o0 + w] = u2;
    }
  }
}

// one wave per channel: lane j folds chunks j, j + 64, ... in order, then a fixed butterfly
__device__ __forceinline__ double chunk_fold(const double* __restrict__ part, int64_t stride, int lane) {
  double t = 0.0;
  for (int c = lane; c < kStatChunks; c += 64) t += part[(int64_t)c * stride];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) t += __shfl_xor(t, d);
  return t;
}

__global__ __launch_bounds__(256) void channel_combine_kernel(const double* __restrict__ part, int64_t M,
                                                              int O, double* __restrict__ mean,
                                                              double* __restrict__ var) {
  const int o = blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (o >= O) return;
  const double s = chunk_fold(part + o, 2 * (int64_t)O, lane);
  const double q = chunk_fold(part + O + o, 2 * (int64_t)O, lane);
  if (lane == 0) {
    const double mu = s / (double)M;
    const double v = q / (double)M - mu * mu;
    mean[o] = mu;
    var[o] = v > 0.0 ? v : 0.0;
  }
}

// channel_combine_kernel followed by sa_train.hip's bn_coeffs_kernel in one launch (the
// BatchNorm forward's statistics, affine coefficients and running-stat update): the same
// operations, fp contraction off as in that file, so the same bits
__global__ __launch_bounds__(256) void bn_stats_coeffs_kernel(
    const double* __restrict__ part, int64_t M, int O, double* __restrict__ mean,
    double* __restrict__ var, const float* __restrict__ gamma, const float* __restrict__ beta,
    double eps, double momentum, float* __restrict__ run_mean, float* __restrict__ run_var,
    float* __restrict__ scale, float* __restrict__ shift, double* __restrict__ invstd) {
  const int o = blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (o >= O) return;
  const double s = chunk_fold(part + o, 2 * (int64_t)O, lane);
  const double q = chunk_fold(part + O + o, 2 * (int64_t)O, lane);
  if (lane) return;
  // the statistics as channel_combine_kernel (this file's flags)
  const double mu = s / (double)M;
  const double v0 = q / (double)M - mu * mu;
  const double vd = v0 > 0.0 ? v0 : 0.0;
  mean[o] = mu;
  var[o] = vd;
  {  // the coefficients as bn_coeffs_kernel (sa_train.hip: fp contraction off)
#pragma clang fp contract(off)
    const float v = (float)vd, muf = (float)mu;
    const float sc = gamma[o] / sqrtf(v + (float)eps);
    scale[o] = sc;
    shift[o] = beta[o] - muf * sc;
    invstd[o] = 1.0 / sqrt(vd + eps);
    if (run_mean) {
      const double unb = M > 1 ? vd * ((double)M / (double)(M - 1)) : vd;
      run_mean[o] = (float)((1.0 - momentum) * run_mean[o] + momentum * mu);
      run_var[o] = (float)((1.0 - momentum) * run_var[o] + momentum * unb);
    }
  }
}

__global__ void affine_act_kernel(const float* __restrict__ Z, int64_t M, int O,
                                  const float* __restrict__ scale, const float* __restrict__ shift,
                                  int relu, int64_t ns, float* __restrict__ Y) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < M * O;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(e % O);
    const int64_t m = e / O;
    float v = fmaf(Z[e], scale[o], shift[o]);
    if (relu) v = fmaxf(v, 0.0f);
    if (ns > 0) atomicMax(reinterpret_cast<unsigned int*>(&Y[(m / ns) * O + o]), __float_as_uint(v));
    else Y[e] = v;
  }
}

// Weight gradient of a per-point linear layer (training path, models/_autograd.py):
//   dW[o, i] = sum_m dZ[m, o] * X[m, i]      db[o] = sum_m dZ[m, o]
// dZ [M, O] and X [M, I] are read in their natural row-major layout (no transposed copies).
// The reduction over the M rows (240k for the noise predictor at B=8) is split into chunks:
// grid = (O tiles x I tiles, chunks); each workgroup reduces its rows on exact-f32 MFMA into a
// partial [O, I] tile, and wgrad_combine sums the partials in chunk order in float64, so the
// gradient is deterministic.  The MFMA A operand is dZ^T (lane = o), B is X (lane = i); both
// tiles are staged k-major in LDS (row stride 96 floats: the two half-waves read rows kk and
// kk+1 from disjoint bank ranges).
constexpr int kWgLd = 96;

__global__ __launch_bounds__(256) void wgrad_partial_kernel(const float* __restrict__ dZ,
                                                            const float* __restrict__ X, int64_t M,
                                                            int I, int O, int64_t rows_per_chunk,
                                                            int tiles_i, float* __restrict__ partW,
                                                            float* __restrict__ partB) {
  __shared__ float As[kBK][kWgLd];  // dZ[m][o]
  __shared__ float Bs[kBK][kWgLd];  // X[m][i]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, h = lane >> 5, l32 = lane & 31;
  const int o0 = (blockIdx.x / tiles_i) * kBN, i0 = (blockIdx.x % tiles_i) * kBN;
  const int chunk = blockIdx.y;
  const int64_t mb = (int64_t)chunk * rows_per_chunk;
  const int64_t me = mb + rows_per_chunk < M ? mb + rows_per_chunk : M;
  const bool bias = partB != nullptr && i0 == 0;
  f32x16 acc = f32x16{};
  float bsum = 0.0f;
  for (int64_t k0 = mb; k0 < me; k0 += kBK) {
#pragma unroll
    for (int e = tid; e < kBK * kBN; e += 256) {
      const int r = e >> 6, c = e & 63;
      const int64_t m = k0 + r;
      const bool mv = m < me;
      As[r][c] = (mv && o0 + c < O) ? dZ[m * O + o0 + c] : 0.0f;
      Bs[r][c] = (mv && i0 + c < I) ? X[m * I + i0 + c] : 0.0f;
    }
    __syncthreads();
    if (bias && tid < kBN) {
#pragma unroll 8
      for (int r = 0; r < kBK; ++r) bsum += As[r][tid];
    }
#pragma unroll
    for (int kk = 0; kk < kBK; kk += 2) {
      const float a = As[kk + h][wr * 32 + l32];
      const float b = Bs[kk + h][wc * 32 + l32];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  // C layout: column (i) = lane & 31, row (o) = crow(r, h)
  const int i = i0 + wc * 32 + l32;
  float* pw = partW + (int64_t)chunk * O * I;
  if (i < I) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = o0 + wr * 32 + crow(r, h);
      if (o < O) pw[(int64_t)o * I + i] = acc[r];
    }
  }
  if (bias && tid < kBN && o0 + tid < O) partB[(int64_t)chunk * O + o0 + tid] = bsum;
}

// out[e] = sum over chunks of part[c][e], in chunk order, float64
__global__ void wgrad_combine_kernel(const float* __restrict__ part, int64_t n, int chunks,
                                     float* __restrict__ out) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int c = 0; c < chunks; ++c) s += (double)part[(int64_t)c * n + e];
    out[e] = (float)s;
  }
}

// ReLU backward of the training path: dz = dy * [y > 0] in one pass (the product form keeps
// torch's semantics: -0 and NaN propagate as in dy * mask)
__global__ void relu_bwd_kernel(const float4* __restrict__ dy, const float4* __restrict__ y,
                                int64_t n4, float4* __restrict__ dz) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n4;
       e += (int64_t)gridDim.x * blockDim.x) {
    const float4 g = dy[e], v = y[e];
    dz[e] = make_float4(g.x * (v.x > 0.f ? 1.f : 0.f), g.y * (v.y > 0.f ? 1.f : 0.f),
                        g.z * (v.z > 0.f ? 1.f : 0.f), g.w * (v.w > 0.f ? 1.f : 0.f));
  }
}

__global__ void relu_bwd_tail_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                     int64_t b0, int64_t n, float* __restrict__ dz) {
  const int64_t e = b0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e < n) dz[e] = dy[e] * (y[e] > 0.f ? 1.f : 0.f);
}

struct WgradPlan {
  int tiles_i, tiles_o, chunks;
  int64_t rows_per_chunk;
};

// enough workgroups to fill 256 CUs several times over; chunks of >= 256 rows
static WgradPlan wgrad_plan(int64_t M, int64_t I, int64_t O) {
  WgradPlan p;
  p.tiles_i = (int)cdiv(I, kBN);
  p.tiles_o = (int)cdiv(O, kBN);
  const int64_t tiles = (int64_t)p.tiles_i * p.tiles_o;
  int64_t chunks = cdiv(2048, tiles);
  chunks = std::max<int64_t>(1, std::min<int64_t>(chunks, cdiv(M, 256)));
  p.rows_per_chunk = cdiv(cdiv(M, chunks), kBK) * kBK;
  p.chunks = (int)cdiv(M, p.rows_per_chunk);
  return p;
}

}  // namespace pcst

using namespace pcst;

extern "C" int pcst_pointwise_linear(const float* X, int64_t M, int64_t K, const float* W,
                                     int64_t O, const float* scale, const float* shift, int relu,
                                     int64_t pool_ns, float* Y, void* stream) {
  PCST_CHECK_ARG(M >= 0 && K > 0 && O > 0 && K < (1 << 20) && O < (1 << 20), "pointwise_linear: bad shape");
  PCST_CHECK_ARG(pool_ns == 0 || (relu && M % pool_ns == 0),
                 "pointwise_linear: pooling needs relu and M %% ns == 0");
  if (M == 0) return PCST_OK;
  PCST_CHECK_ARG(X && W && Y, "pointwise_linear: null pointer");
  hipStream_t s = as_stream(stream);
  if (pool_ns > 0) PCST_HIP(hipMemsetAsync(Y, 0, sizeof(float) * (M / pool_ns) * O, s), "memset");
  dim3 grid((unsigned)cdiv(M, kBM), (unsigned)cdiv(O, kBN));
  if (pool_ns > 0)
    hipLaunchKernelGGL(pw_linear_kernel<true>, grid, dim3(256), 0, s, X, M, (int)K, W, (int)O,
                       scale, shift, relu, pool_ns, Y);
  else
    hipLaunchKernelGGL(pw_linear_kernel<false>, grid, dim3(256), 0, s, X, M, (int)K, W, (int)O,
                       scale, shift, relu, (int64_t)0, Y);
  PCST_LAUNCH_CHECK("pointwise_linear");
  return PCST_OK;
}

extern "C" int pcst_channel_stats_workspace_size(int64_t O, size_t* bytes) {
  *bytes = sizeof(double) * (size_t)(2 * kStatChunks * O);
  return PCST_OK;
}

extern "C" int pcst_channel_stats(const float* Z, int64_t M, int64_t O, double* mean, double* var,
                                  void* workspace, void* stream) {
  PCST_CHECK_ARG(M > 0 && O > 0, "channel_stats: bad shape");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  if (O % 4 == 0 && (uintptr_t)Z % 16 == 0) {
    const int64_t G = O / 4;
    hipLaunchKernelGGL(channel_partial_kernel<4>, dim3(kStatChunks, (unsigned)cdiv(G, G < 64 ? G : 64)),
                       dim3(256), 0, s, Z, M, (int)O, part);
  } else {
    hipLaunchKernelGGL(channel_partial_kernel<1>, dim3(kStatChunks, (unsigned)cdiv(O, O < 64 ? O : 64)),
                       dim3(256), 0, s, Z, M, (int)O, part);
  }
  hipLaunchKernelGGL(channel_combine_kernel, dim3((unsigned)cdiv(O, 4)), dim3(256), 0, s, part, M,
                     (int)O, mean, var);
  PCST_LAUNCH_CHECK("channel_stats");
  return PCST_OK;
}

extern "C" int pcst_bn_train_stats(const float* Z, int64_t M, int64_t O, const float* gamma,
                                   const float* beta, double eps, double momentum,
                                   float* running_mean, float* running_var, double* mean, double* var,
                                   float* scale, float* shift, double* invstd, void* workspace,
                                   void* stream) {
  PCST_CHECK_ARG(M > 0 && O > 0, "bn_train_stats: bad shape");
  PCST_CHECK_ARG(Z && gamma && beta && mean && var && scale && shift && invstd && workspace,
                 "bn_train_stats: null pointer");
  PCST_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr),
                 "bn_train_stats: running mean and var go together");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  if (O % 4 == 0 && (uintptr_t)Z % 16 == 0) {
    const int64_t G = O / 4;
    hipLaunchKernelGGL(channel_partial_kernel<4>, dim3(kStatChunks, (unsigned)cdiv(G, G < 64 ? G : 64)),
                       dim3(256), 0, s, Z, M, (int)O, part);
  } else {
    hipLaunchKernelGGL(channel_partial_kernel<1>, dim3(kStatChunks, (unsigned)cdiv(O, O < 64 ? O : 64)),
                       dim3(256), 0, s, Z, M, (int)O, part);
  }
  hipLaunchKernelGGL(bn_stats_coeffs_kernel, dim3((unsigned)cdiv(O, 4)), dim3(256), 0, s, part, M,
                     (int)O, mean, var, gamma, beta, eps, momentum, running_mean, running_var, scale,
                     shift, invstd);
  PCST_LAUNCH_CHECK("bn_train_stats");
  return PCST_OK;
}

extern "C" int pcst_affine_act(const float* Z, int64_t M, int64_t O, const float* scale,
                               const float* shift, int relu, int64_t pool_ns, float* Y,
                               void* stream) {
  PCST_CHECK_ARG(M >= 0 && O > 0, "affine_act: bad shape");
  PCST_CHECK_ARG(pool_ns == 0 || (relu && M % pool_ns == 0), "affine_act: pooling needs relu");
  if (M == 0) return PCST_OK;
  hipStream_t s = as_stream(stream);
  if (pool_ns > 0) PCST_HIP(hipMemsetAsync(Y, 0, sizeof(float) * (M / pool_ns) * O, s), "memset");
  const int64_t g = std::min<int64_t>(cdiv(M * O, 256), 8192);
  hipLaunchKernelGGL(affine_act_kernel, dim3((unsigned)g), dim3(256), 0, s, Z, M, (int)O, scale,
                     shift, relu, pool_ns, Y);
  PCST_LAUNCH_CHECK("affine_act");
  return PCST_OK;
}

extern "C" int pcst_linear_wgrad_workspace_size(int64_t M, int64_t I, int64_t O, size_t* bytes) {
  PCST_CHECK_ARG(M >= 0 && I > 0 && O > 0 && bytes, "linear_wgrad_workspace_size: bad args");
  const WgradPlan p = wgrad_plan(std::max<int64_t>(M, 1), I, O);
  *bytes = sizeof(float) * (size_t)p.chunks * (size_t)(O * I + O);
  return PCST_OK;
}

extern "C" int pcst_linear_wgrad(const float* dZ, const float* X, int64_t M, int64_t I,
                                 int64_t O, float* dW, float* db, void* workspace, void* stream) {
  PCST_CHECK_ARG(M >= 0 && I > 0 && O > 0 && I < (1 << 20) && O < (1 << 20),
                 "linear_wgrad: bad shape");
  PCST_CHECK_ARG(dW && workspace && (M == 0 || (dZ && X)), "linear_wgrad: null pointer");
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    PCST_HIP(hipMemsetAsync(dW, 0, sizeof(float) * O * I, s), "memset");
    if (db) PCST_HIP(hipMemsetAsync(db, 0, sizeof(float) * O, s), "memset");
    return PCST_OK;
  }
  const WgradPlan p = wgrad_plan(M, I, O);
  float* partW = static_cast<float*>(workspace);
  float* partB = db ? partW + (int64_t)p.chunks * O * I : nullptr;
  hipLaunchKernelGGL(wgrad_partial_kernel, dim3((unsigned)(p.tiles_i * p.tiles_o), (unsigned)p.chunks),
                     dim3(256), 0, s, dZ, X, M, (int)I, (int)O, p.rows_per_chunk, p.tiles_i, partW,
                     partB);
  const int64_t n = O * I;
  hipLaunchKernelGGL(wgrad_combine_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 2048)),
                     dim3(256), 0, s, partW, n, p.chunks, dW);
  if (db)
    hipLaunchKernelGGL(wgrad_combine_kernel, dim3((unsigned)cdiv(O, 256)), dim3(256), 0, s, partB,
                       O, p.chunks, db);
  PCST_LAUNCH_CHECK("linear_wgrad");
  return PCST_OK;
}

extern "C" int pcst_relu_bwd(const float* dy, const float* y, int64_t n, float* dz, void* stream) {
  PCST_CHECK_ARG(n >= 0, "relu_bwd: bad size");
  if (n == 0) return PCST_OK;
  PCST_CHECK_ARG(dy && y && dz, "relu_bwd: null pointer");
  hipStream_t s = as_stream(stream);
  const bool vec = ((uintptr_t)dy % 16 == 0) && ((uintptr_t)y % 16 == 0) && ((uintptr_t)dz % 16 == 0);
  const int64_t n4 = vec ? n / 4 : 0;
  if (n4 > 0)
    hipLaunchKernelGGL(relu_bwd_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n4, 256), 8192)),
                       dim3(256), 0, s, reinterpret_cast<const float4*>(dy),
                       reinterpret_cast<const float4*>(y), n4, reinterpret_cast<float4*>(dz));
  if (n4 * 4 < n)
    hipLaunchKernelGGL(relu_bwd_tail_kernel, dim3((unsigned)cdiv(n - n4 * 4, 256)), dim3(256), 0, s,
                       dy, y, n4 * 4, n, dz);
  PCST_LAUNCH_CHECK("relu_bwd");
  return PCST_OK;
}
