// Training half of SetAbstraction (models/pointnet2_encoder.py:92-112): train-mode BatchNorm2d
// + ReLU (+ max over nsample) forward and backward, and the backward of the grouped-feature
// gather, replacing F.batch_norm / F.relu / torch.max / advanced-index backward on the trainer's
// path.  Everything is deterministic: per-channel reductions are fixed row chunks combined in
// chunk order in float64, and the gather backward sums every destination's contributions in
// ascending entry order after a stable radix sort (no float atomics).
//
//   forward   stats     mean, var (biased) of Z [M, O]               pcst_channel_stats
//             coeffs    scale = g / sqrt(var + eps), shift = b - mean scale, invstd; running
//                       stats (momentum, unbiased var) updated on the device   pcst_bn_train_coeffs
//             act       Y = relu(scale Z + shift)                    pcst_affine_act
//                       or pooled P[g] = max over the ns rows of group g, with the first row
//                       of the maximum                               pcst_bn_relu_maxpool
//   backward  dyp = dY * [scale Z + shift > 0]   (dY dense, or dP routed to the argmax rows)
//             S1 = sum_m dyp, S2 = sum_m dyp xhat, xhat = (Z - mean) invstd
//             dZ = g invstd (dyp - S1/M - xhat S2/M); dgamma = S2, dbeta = S1
//                                                                    pcst_bn_relu_bwd
//   gather    grouped[b, s, k, 3 + c] = P[b, clamp(idx[b, s, k]), c]  (pcst_group_gather)
//             dP[b, n, c] = sum over entries e with idx == n of dG[b, e, 3 + c]
//                                                                    pcst_group_gather_bwd
#include <hip/hip_fp16.h>

#include "common.h"
#include "sort.h"

namespace pcst {

constexpr int kBnChunks = 256;  // row chunks of the per-channel reductions

__global__ void bn_coeffs_kernel(const double* __restrict__ mean, const double* __restrict__ var,
                                 int64_t M, int O, const float* __restrict__ gamma,
                                 const float* __restrict__ beta, double eps, double momentum,
                                 float* __restrict__ run_mean, float* __restrict__ run_var,
                                 float* __restrict__ scale, float* __restrict__ shift,
                                 double* __restrict__ invstd) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= O) return;
  // fp32 steps of the training path (pointnet2_encoder.py via F.batch_norm): invstd from the
  // fp32 variance, scale / shift in fp32
  const float v = (float)var[o], mu = (float)mean[o];
  const float sc = gamma[o] / sqrtf(v + (float)eps);
  scale[o] = sc;
  shift[o] = beta[o] - mu * sc;
  invstd[o] = 1.0 / sqrt(var[o] + eps);
  if (run_mean) {
    const double unb = M > 1 ? var[o] * ((double)M / (double)(M - 1)) : var[o];
    run_mean[o] = (float)((1.0 - momentum) * run_mean[o] + momentum * mean[o]);
    run_var[o] = (float)((1.0 - momentum) * run_var[o] + momentum * unb);
  }
}

// pooled[g, o] = max_{r < ns} relu(scale Z[g ns + r, o] + shift), arg = first r of the max
__global__ void bn_relu_maxpool_kernel(const float* __restrict__ Z, int64_t G, int64_t ns, int O,
                                       const float* __restrict__ scale,
                                       const float* __restrict__ shift, float* __restrict__ Y,
                                       int32_t* __restrict__ arg) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < G * O;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(e % O);
    const int64_t g = e / O;
    const float sc = scale[o], sh = shift[o];
    const float* z = Z + g * ns * O + o;
    float best = -1.0f;
    int bi = 0;
    for (int64_t r = 0; r < ns; ++r) {
      const float v = fmaxf(fmaf(z[r * O], sc, sh), 0.0f);
      if (v > best) { best = v; bi = (int)r; }
    }
    Y[e] = best;
    arg[e] = bi;
  }
}

// Per-channel partial sums over row chunks: a 256-thread block covers TQ = min(O / W, 64)
// groups of W channels (W = 4: 16-byte loads when O % 4 == 0) x (256 / TQ) row lanes; lanes are
// folded in a fixed order, chunks combined in a fixed order later.
template <int W>
struct Vec;
template <>
struct Vec<4> {
  float v[4];
  __device__ __forceinline__ void load(const float* __restrict__ p) {
    const float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
  }
};
template <>
struct Vec<1> {
  float v[1];
  __device__ __forceinline__ void load(const float* __restrict__ p) { v[0] = *p; }
};

// dyp[w] = dY * [scale z + shift > 0] for channels o..o+W-1 of row m (z returned)
template <int W>
__device__ __forceinline__ void bn_dyp(const float* __restrict__ Z, const float* __restrict__ dY,
                                       const float* __restrict__ dP, const int32_t* __restrict__ arg,
                                       int64_t ns, int O, int64_t m, int o, const float* sc,
                                       const float* sh, float (&z)[W], float (&dyp)[W]) {
  Vec<W> zv, dv;
  zv.load(Z + m * O + o);
  if (dY) {
    dv.load(dY + m * O + o);
  } else {
    const int64_t g = m / ns;
    const int r = (int)(m - g * ns);
    dv.load(dP + g * O + o);
#pragma unroll
    for (int w = 0; w < W; ++w)
      if (arg[g * O + o + w] != r) dv.v[w] = 0.0f;
  }
#pragma unroll
  for (int w = 0; w < W; ++w) {
    z[w] = zv.v[w];
    dyp[w] = fmaf(z[w], sc[w], sh[w]) > 0.0f ? dv.v[w] : 0.0f;
  }
}

template <int W>
__global__ __launch_bounds__(256) void bn_bwd_partial_kernel(
    const float* __restrict__ Z, const float* __restrict__ dY, const float* __restrict__ dP,
    const int32_t* __restrict__ arg, int64_t M, int64_t ns, int O, const float* __restrict__ scale,
    const float* __restrict__ shift, const double* __restrict__ mean,
    const double* __restrict__ invstd, double* __restrict__ part) {
  const int G = O / W;
  const int TQ = G < 64 ? G : 64;
  const int RL = 256 / TQ;                 // row lanes
  const int cg = threadIdx.x % TQ, rl = threadIdx.x / TQ;
  const int o = (blockIdx.y * TQ + cg) * W;
  const int chunk = blockIdx.x;
  const int64_t per = (M + kBnChunks - 1) / kBnChunks;
  const int64_t a = chunk * per, e = a + per < M ? a + per : M;
  __shared__ double s1[W][256], s2[W][256];
  double t1[W], t2[W];
#pragma unroll
  for (int w = 0; w < W; ++w) t1[w] = t2[w] = 0.0;
  if (rl < RL && o < O) {
    float sc[W], sh[W];
    double mu[W], is[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      sc[w] = scale[o + w];
      sh[w] = shift[o + w];
      mu[w] = mean[o + w];
      is[w] = invstd[o + w];
    }
    for (int64_t m = a + rl; m < e; m += RL) {
      float z[W], dyp[W];
      bn_dyp<W>(Z, dY, dP, arg, ns, O, m, o, sc, sh, z, dyp);
#pragma unroll
      for (int w = 0; w < W; ++w) {
        t1[w] += dyp[w];
        t2[w] += dyp[w] * (((double)z[w] - mu[w]) * is[w]);
      }
    }
  }
#pragma unroll
  for (int w = 0; w < W; ++w) {
    s1[w][threadIdx.x] = t1[w];
    s2[w][threadIdx.x] = t2[w];
  }
  __syncthreads();
  if (rl == 0 && o < O) {
#pragma unroll
    for (int w = 0; w < W; ++w) {
      double u1 = 0.0, u2 = 0.0;
      for (int q = 0; q < RL; ++q) {
        u1 += s1[w][q * TQ + cg];
        u2 += s2[w][q * TQ + cg];
      }
      part[((int64_t)chunk * 2 + 0) * O + o + w] = u1;
      part[((int64_t)chunk * 2 + 1) * O + o + w] = u2;
    }
  }
}

// one wave per channel: lane j folds chunks j, j + 64, ... in order, then a fixed butterfly
__device__ __forceinline__ double bn_chunk_fold(const double* __restrict__ part, int64_t stride,
                                                int lane) {
  double t = 0.0;
  for (int c = lane; c < kBnChunks; c += 64) t += part[(int64_t)c * stride];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) t += __shfl_xor(t, d);
  return t;
}

// S1, S2 over the chunks -> dgamma = S2, dbeta = S1 and the per-channel coefficients of dZ
__global__ __launch_bounds__(256) void bn_bwd_combine_kernel(const double* __restrict__ part, int64_t M,
                                                             int O, const float* __restrict__ gamma,
                                                             const double* __restrict__ invstd,
                                                             double* __restrict__ coef,
                                                             float* __restrict__ dgamma,
                                                             float* __restrict__ dbeta) {
  const int o = blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (o >= O) return;
  const double u1 = bn_chunk_fold(part + o, 2 * (int64_t)O, lane);
  const double u2 = bn_chunk_fold(part + O + o, 2 * (int64_t)O, lane);
  if (lane) return;
  if (dgamma) dgamma[o] = (float)u2;
  if (dbeta) dbeta[o] = (float)u1;
  coef[o * 3 + 0] = (double)gamma[o] * invstd[o];
  coef[o * 3 + 1] = u1 / (double)M;
  coef[o * 3 + 2] = u2 / (double)M;
}

// dZ = g invstd (dyp - S1/M - xhat S2/M), W channels of one row per thread
template <int W>
__global__ void bn_bwd_apply_kernel(const float* __restrict__ Z, const float* __restrict__ dY,
                                    const float* __restrict__ dP, const int32_t* __restrict__ arg,
                                    int64_t M, int64_t ns, int O, const float* __restrict__ scale,
                                    const float* __restrict__ shift, const double* __restrict__ mean,
                                    const double* __restrict__ invstd,
                                    const double* __restrict__ coef, float* __restrict__ dZ) {
  const int G = O / W;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < M * G;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = q / G;
    const int o = (int)(q - m * G) * W;
    float sc[W], sh[W], z[W], dyp[W], out[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      sc[w] = scale[o + w];
      sh[w] = shift[o + w];
    }
    bn_dyp<W>(Z, dY, dP, arg, ns, O, m, o, sc, sh, z, dyp);
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const double xh = ((double)z[w] - mean[o + w]) * invstd[o + w];
      out[w] = (float)(coef[(o + w) * 3 + 0] *
                       ((double)dyp[w] - coef[(o + w) * 3 + 1] - xh * coef[(o + w) * 3 + 2]));
    }
    if constexpr (W == 4)
      *reinterpret_cast<float4*>(dZ + m * O + o) = make_float4(out[0], out[1], out[2], out[3]);
    else
      dZ[m * O + o] = out[0];
  }
}

// ---- gather backward
__global__ void gather_keys_kernel(const int64_t* __restrict__ gidx, int64_t E, int64_t N,
                                   uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const int b = blockIdx.y;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    int64_t n = gidx[b * E + e];
    n = n < 0 ? 0 : (n > N - 1 ? N - 1 : n);
    keys[b * E + e] = (uint32_t)n;
    vals[b * E + e] = (uint32_t)e;
  }
}

// one workgroup per destination (n, b): its entries are one run of the sorted keys, summed in
// ascending entry order (the sort is stable)
__global__ void gather_bwd_kernel(const float* __restrict__ dG, const uint32_t* __restrict__ keys,
                                  const uint32_t* __restrict__ vals, int64_t E, int64_t C,
                                  int64_t N, float* __restrict__ dP) {
  const int64_t n = blockIdx.x;
  const int b = blockIdx.y;
  const uint32_t* K = keys + b * E;
  // lower bounds of n and n + 1 (uniform: every thread searches the same)
  int64_t lo = 0, hi = E;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (K[mid] < (uint32_t)n) lo = mid + 1; else hi = mid;
  }
  const int64_t s0 = lo;
  hi = E;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (K[mid] <= (uint32_t)n) lo = mid + 1; else hi = mid;
  }
  const int64_t s1 = lo;
  const uint32_t* V = vals + b * E;
  const float* G = dG + (int64_t)b * E * (3 + C) + 3;
  for (int64_t c = threadIdx.x; c < C; c += blockDim.x) {
    float acc = 0.0f;
    for (int64_t i = s0; i < s1; ++i) acc += G[(int64_t)V[i] * (3 + C) + c];
    dP[((int64_t)b * N + n) * C + c] = acc;
  }
}

struct GatherWS {
  uint32_t *k, *v, *kt, *vt, *hist;
  size_t bytes;
};

static GatherWS carve_gather(void* base, int64_t B, int64_t E) {
  Carver c(base);
  GatherWS w;
  w.k = c.take<uint32_t>(B * E);
  w.v = c.take<uint32_t>(B * E);
  w.kt = c.take<uint32_t>(B * E);
  w.vt = c.take<uint32_t>(B * E);
  w.hist = c.take<uint32_t>(radix_hist_words((int)B, E));
  w.bytes = c.bytes();
  return w;
}

static unsigned grid1d(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n, 256), 8192)); }

}  // namespace pcst

using namespace pcst;

extern "C" int pcst_bn_train_coeffs(const double* mean, const double* var, int64_t M, int64_t O,
                                    const float* gamma, const float* beta, double eps,
                                    double momentum, float* running_mean, float* running_var,
                                    float* scale, float* shift, double* invstd, void* stream) {
  PCST_CHECK_ARG(M > 0 && O > 0, "bn_train_coeffs: bad shape");
  PCST_CHECK_ARG(mean && var && gamma && beta && scale && shift && invstd,
                 "bn_train_coeffs: null pointer");
  PCST_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr),
                 "bn_train_coeffs: running mean and var go together");
  hipLaunchKernelGGL(bn_coeffs_kernel, dim3((unsigned)cdiv(O, 256)), dim3(256), 0,
                     as_stream(stream), mean, var, M, (int)O, gamma, beta, eps, momentum,
                     running_mean, running_var, scale, shift, invstd);
  PCST_LAUNCH_CHECK("bn_train_coeffs");
  return PCST_OK;
}

extern "C" int pcst_bn_relu_maxpool(const float* Z, int64_t M, int64_t O, const float* scale,
                                    const float* shift, int64_t ns, float* Y, int32_t* arg,
                                    void* stream) {
  PCST_CHECK_ARG(M >= 0 && O > 0 && ns > 0 && M % ns == 0, "bn_relu_maxpool: bad shape");
  if (M == 0) return PCST_OK;
  PCST_CHECK_ARG(Z && scale && shift && Y && arg, "bn_relu_maxpool: null pointer");
  const int64_t G = M / ns;
  hipLaunchKernelGGL(bn_relu_maxpool_kernel, dim3(grid1d(G * O)), dim3(256), 0, as_stream(stream),
                     Z, G, ns, (int)O, scale, shift, Y, arg);
  PCST_LAUNCH_CHECK("bn_relu_maxpool");
  return PCST_OK;
}

extern "C" int pcst_bn_relu_bwd_workspace_size(int64_t O, size_t* bytes) {
  PCST_CHECK_ARG(O > 0 && bytes, "bn_relu_bwd_workspace_size: bad args");
  *bytes = sizeof(double) * (size_t)(2 * kBnChunks * O + 3 * O);
  return PCST_OK;
}

extern "C" int pcst_bn_relu_bwd(const float* Z, int64_t M, int64_t O, const float* scale,
                                const float* shift, const double* mean, const double* invstd,
                                const float* gamma, const float* dY, const float* dP,
                                const int32_t* arg, int64_t ns, float* dZ, float* dgamma,
                                float* dbeta, void* workspace, void* stream) {
  PCST_CHECK_ARG(M > 0 && O > 0, "bn_relu_bwd: bad shape");
  PCST_CHECK_ARG(Z && scale && shift && mean && invstd && gamma && dZ && workspace,
                 "bn_relu_bwd: null pointer");
  PCST_CHECK_ARG(dY ? (dP == nullptr) : (dP && arg && ns > 0 && M % ns == 0),
                 "bn_relu_bwd: give dY (dense) or dP + arg + ns (pooled)");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  double* coef = part + 2 * kBnChunks * O;
  const bool vec = O % 4 == 0 && ((uintptr_t)Z | (uintptr_t)dY | (uintptr_t)dP | (uintptr_t)dZ) % 16 == 0;
  if (vec) {
    const int64_t G = O / 4;
    hipLaunchKernelGGL(bn_bwd_partial_kernel<4>, dim3(kBnChunks, (unsigned)cdiv(G, G < 64 ? G : 64)),
                       dim3(256), 0, s, Z, dY, dP, arg, M, ns, (int)O, scale, shift, mean, invstd, part);
  } else {
    hipLaunchKernelGGL(bn_bwd_partial_kernel<1>, dim3(kBnChunks, (unsigned)cdiv(O, O < 64 ? O : 64)),
                       dim3(256), 0, s, Z, dY, dP, arg, M, ns, (int)O, scale, shift, mean, invstd, part);
  }
  hipLaunchKernelGGL(bn_bwd_combine_kernel, dim3((unsigned)cdiv(O, 4)), dim3(256), 0, s, part, M,
                     (int)O, gamma, invstd, coef, dgamma, dbeta);
  if (vec)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<4>, dim3(grid1d(M * O / 4)), dim3(256), 0, s, Z, dY, dP,
                       arg, M, ns, (int)O, scale, shift, mean, invstd, coef, dZ);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<1>, dim3(grid1d(M * O)), dim3(256), 0, s, Z, dY, dP, arg,
                       M, ns, (int)O, scale, shift, mean, invstd, coef, dZ);
  PCST_LAUNCH_CHECK("bn_relu_bwd");
  return PCST_OK;
}

extern "C" int pcst_group_gather_bwd_workspace_size(int64_t B, int64_t E, size_t* bytes) {
  PCST_CHECK_ARG(B >= 0 && E >= 0 && bytes, "group_gather_bwd_workspace_size: bad args");
  *bytes = carve_gather(nullptr, B, E).bytes;
  return PCST_OK;
}

extern "C" int pcst_group_gather_bwd(const float* dgrouped, const int64_t* group_idx, int64_t B,
                                     int64_t S, int64_t ns, int64_t N, int64_t C, float* dpoints,
                                     void* workspace, void* stream) {
  PCST_CHECK_ARG(B >= 0 && S >= 0 && ns >= 0 && N > 0 && C > 0, "group_gather_bwd: bad shape");
  const int64_t E = S * ns;
  PCST_CHECK_ARG(N <= 65536 && E <= 262144, "group_gather_bwd: N <= 65536 and S*ns <= 262144");
  hipStream_t s = as_stream(stream);
  if (B == 0) return PCST_OK;
  PCST_CHECK_ARG(dpoints && workspace && (E == 0 || (dgrouped && group_idx)),
                 "group_gather_bwd: null pointer");
  if (E == 0) {
    PCST_HIP(hipMemsetAsync(dpoints, 0, sizeof(float) * B * N * C, s), "memset");
    return PCST_OK;
  }
  GatherWS w = carve_gather(workspace, B, E);
  hipLaunchKernelGGL(gather_keys_kernel, dim3((unsigned)std::min<int64_t>(cdiv(E, 256), 1024), (unsigned)B),
                     dim3(256), 0, s, group_idx, E, N, w.k, w.v);
  int rc = radix_sort_pairs(w.k, w.v, w.kt, w.vt, w.hist, (int)B, E, SegCounts{nullptr, (int32_t)E},
                            0, 16, s);
  if (rc) return rc;
  hipLaunchKernelGGL(gather_bwd_kernel, dim3((unsigned)N, (unsigned)B), dim3(C >= 128 ? 128 : 64), 0, s,
                     dgrouped, w.k, w.v, E, C, N, dpoints);
  PCST_LAUNCH_CHECK("group_gather_bwd");
  return PCST_OK;
}

// ---- per-cloud column sums of a 16-bit matrix (NoisePredictorFn's dL/dtf = dL/dsf) ----------
// out[b][c] = f32(h16(sum over the N rows of cloud b of G[b*N + n][c])): the reduction autograd
// makes for the broadcast time / style rows of x = (pf + tf) + sf (diffusion_model.py:56-58)
// under autocast -- float accumulation, the 16-bit output rounding of torch's half sum.
// Deterministic: slice s of cloud b sums rows [s*rows_per, ...) in row order per lane, the 8
// row lanes of a work-group meet in LDS in lane order, and the slices are combined in slice order.
namespace pcst {
constexpr int kColsumSlices = 64;
constexpr int kColsumCols = 256;  // columns per work-group: 32 lanes x 8 (16-byte loads)

__device__ __forceinline__ float h16_to_f(uint16_t v, int f16) {
  if (f16) return __half2float(__ushort_as_half(v));
  return __uint_as_float((uint32_t)v << 16);
}
__device__ __forceinline__ float h16_round(float v, int f16) {
  if (f16) return __half2float(__float2half_rn(v));
  return (float)(__bf16)v;
}

__global__ __launch_bounds__(256) void colsum16_partial_kernel(const uint16_t* __restrict__ G,
                                                               int f16, int64_t N, int64_t C,
                                                               float* __restrict__ part) {
  const int b = blockIdx.z, s = blockIdx.y;
  const int64_t c0 = (int64_t)blockIdx.x * kColsumCols + (threadIdx.x & 31) * 8;
  const int rl = threadIdx.x >> 5;  // row lane 0..7
  const int64_t per = (N + kColsumSlices - 1) / kColsumSlices;
  const int64_t r0 = s * per, r1 = r0 + per < N ? r0 + per : N;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < C) {
    const uint16_t* base = G + ((int64_t)b * N) * C + c0;
    for (int64_t r = r0 + rl; r < r1; r += 8) {
      const uint4 v = *reinterpret_cast<const uint4*>(base + r * C);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[2 * j] += h16_to_f((uint16_t)(w[j] & 0xffffu), f16);
        acc[2 * j + 1] += h16_to_f((uint16_t)(w[j] >> 16), f16);
      }
    }
  }
  __shared__ float sh[8][kColsumCols + 4];
#pragma unroll
  for (int j = 0; j < 8; ++j) sh[rl][(threadIdx.x & 31) * 8 + j] = acc[j];
  __syncthreads();
  const int64_t c = (int64_t)blockIdx.x * kColsumCols + threadIdx.x;
  if (c < C) {
    float t = sh[0][threadIdx.x];
#pragma unroll
    for (int k = 1; k < 8; ++k) t += sh[k][threadIdx.x];
    part[((int64_t)b * kColsumSlices + s) * C + c] = t;
  }
}

__global__ __launch_bounds__(256) void colsum16_combine_kernel(const float* __restrict__ part,
                                                               int f16, int64_t B, int64_t C,
                                                               float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= B * C) return;
  const int64_t b = i / C, c = i % C;
  float t = 0.f;
  for (int s = 0; s < kColsumSlices; ++s) t += part[(b * kColsumSlices + s) * C + c];
  out[i] = h16_round(t, f16);
}
}  // namespace pcst

extern "C" int pcst_group_colsum16_workspace_size(int64_t B, int64_t C, size_t* bytes) {
  PCST_CHECK_ARG(bytes && B >= 0 && C >= 0, "group_colsum16_workspace_size: bad arguments");
  *bytes = (size_t)(B * pcst::kColsumSlices * C) * sizeof(float);
  return PCST_OK;
}

extern "C" int pcst_group_colsum16(const uint16_t* G, int f16, int64_t B, int64_t N, int64_t C,
                                   float* out, void* workspace, void* stream) {
  PCST_CHECK_ARG(B >= 0 && N >= 0 && C >= 0, "group_colsum16: bad shape");
  PCST_CHECK_ARG(C % 8 == 0, "group_colsum16: C must be a multiple of 8 (16-byte rows)");
  if (B == 0 || C == 0) return PCST_OK;
  PCST_CHECK_ARG(G && out && workspace, "group_colsum16: null pointer");
  PCST_CHECK_ARG(((uintptr_t)G & 15) == 0, "group_colsum16: G must be 16-byte aligned");
  PCST_CHECK_ARG(B <= 65535, "group_colsum16: too many clouds");
  hipStream_t s = pcst::as_stream(stream);
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(pcst::colsum16_partial_kernel,
                     dim3((unsigned)pcst::cdiv(C, pcst::kColsumCols), pcst::kColsumSlices, (unsigned)B),
                     dim3(256), 0, s, G, f16, N, C, part);
  hipLaunchKernelGGL(pcst::colsum16_combine_kernel, dim3((unsigned)pcst::cdiv(B * C, 256)), dim3(256),
                     0, s, part, f16, B, C, out);
  PCST_LAUNCH_CHECK("group_colsum16");
  return PCST_OK;
}
