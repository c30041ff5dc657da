// Squared Chamfer distance of chamfer_distance_chunked_optimized (models/losses.py:8-63) and
// the L1 noise loss of DiffusionLoss (losses.py:90), forward and backward.
//
// Forward, per direction: D = (|p|^2 + |q|^2) + (-2 p.q) with the reference's rounding
// (dot = K=3 sgemm fma chain, unfused norms; -2*dot is exact so the final add is one fma),
// clamp >= 0, row min with the first index on ties.  Targets stream through LDS in tiles of
// 2048 points; each thread owns one query.  Never materialises the N x M matrix (the reference
// chunks 1024 rows to bound it).  Means are reduced deterministically (fixed-order float64).
//
// Backward (autograd of the reference formula): for a row i with argmin j and raw D >= 0,
// dL/dp_i += g/N * 2(p_i - q_j) and dL/dq_j -= the same.  The scatter onto the argmin side is
// made deterministic without float atomics: (argmin, row) pairs are radix-sorted (stable) and
// every destination sums its contributions in ascending row order.
#include "common.h"
#include "sort.h"

namespace pcst {

constexpr int kCdTile = 2048;

__device__ __forceinline__ float cd_dist(float px, float py, float pz, float np_, float qx,
                                         float qy, float qz, float nq) {
  const float dot = dot3(px, py, pz, qx, qy, qz);
  return ffma(-2.0f, dot, fadd(np_, nq));
}

// one direction: for every query row of P [B,N,3], min over Q [B,M,3]
__global__ __launch_bounds__(256) void chamfer_rowmin_kernel(const float* __restrict__ P,
                                                             const float* __restrict__ Q, int N,
                                                             int M, float* __restrict__ mind,
                                                             int32_t* __restrict__ argm) {
  __shared__ float4 sq[kCdTile];
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const bool valid = i < N;
  const float* p = P + ((int64_t)b * N + (valid ? i : 0)) * 3;
  const float px = p[0], py = p[1], pz = p[2];
  const float np_ = sqnorm3(px, py, pz);
  float best = INFINITY;
  int bj = 0;
  const float* Qb = Q + (int64_t)b * M * 3;
  for (int t0 = 0; t0 < M; t0 += kCdTile) {
    const int tn = min(kCdTile, M - t0);
    __syncthreads();
    for (int k = threadIdx.x; k < tn; k += 256) {
      const float* q = Qb + (int64_t)(t0 + k) * 3;
      const float qx = q[0], qy = q[1], qz = q[2];
      sq[k] = make_float4(qx, qy, qz, sqnorm3(qx, qy, qz));
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < tn; ++k) {
      const float4 q = sq[k];
      float d = cd_dist(px, py, pz, np_, q.x, q.y, q.z, q.w);
      d = d < 0.0f ? 0.0f : d;
      if (d < best) { best = d; bj = t0 + k; }
    }
  }
  if (valid) {
    mind[(int64_t)b * N + i] = best;
    argm[(int64_t)b * N + i] = bj;
  }
}

// out[b] = mean(m1[b]) + mean(m2[b]), fixed-order float64 reduction (one workgroup per cloud)
__global__ __launch_bounds__(256) void chamfer_mean_kernel(const float* __restrict__ m1, int N,
                                                           const float* __restrict__ m2, int M,
                                                           float* __restrict__ out) {
  const int b = blockIdx.x;
  __shared__ double s1[256], s2[256];
  double a = 0.0, c = 0.0;
  for (int i = threadIdx.x; i < N; i += 256) a += m1[(int64_t)b * N + i];
  for (int j = threadIdx.x; j < M; j += 256) c += m2[(int64_t)b * M + j];
  s1[threadIdx.x] = a;
  s2[threadIdx.x] = c;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      s1[threadIdx.x] += s1[threadIdx.x + off];
      s2[threadIdx.x] += s2[threadIdx.x + off];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out[b] = (float)(s1[0] / N + s2[0] / M);
}

// raw (unclamped) D of the pair, recomputed exactly as in the forward
__device__ __forceinline__ float raw_pair(const float* p, const float* q) {
  return cd_dist(p[0], p[1], p[2], sqnorm3(p[0], p[1], p[2]), q[0], q[1], q[2],
                 sqnorm3(q[0], q[1], q[2]));
}

// direct term: row i of P gets g/N * 2(p_i - q_arg) (if raw D >= 0)
__global__ void chamfer_direct_kernel(const float* __restrict__ P, const float* __restrict__ Q,
                                      int N, int M, const int32_t* __restrict__ argm,
                                      const float* __restrict__ gout, float sign,
                                      float* __restrict__ grad) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  const float* p = P + ((int64_t)b * N + i) * 3;
  const float* q = Q + ((int64_t)b * M + argm[(int64_t)b * N + i]) * 3;
  const float s = raw_pair(p, q) >= 0.0f ? gout[b] * 2.0f / (float)N : 0.0f;
  float* g = grad + ((int64_t)b * N + i) * 3;
  for (int c = 0; c < 3; ++c) g[c] += sign * s * (p[c] - q[c]);
}

// keys = argmin (the destination), vals = row, for the stable sort
__global__ void chamfer_keys_kernel(const int32_t* __restrict__ argm, int R, uint32_t* keys,
                                    uint32_t* vals) {
  const int b = blockIdx.y;
  for (int r = blockIdx.x * 256 + threadIdx.x; r < R; r += gridDim.x * 256) {
    keys[(int64_t)b * R + r] = (uint32_t)argm[(int64_t)b * R + r];
    vals[(int64_t)b * R + r] = (uint32_t)r;
  }
}

// scattered term: destination d (a row of D-side cloud, D_pts [B,ND,3]) sums
// sign * g/NR * 2(src_r - dst_d) over source rows r with argmin(r) == d.  A group of 16 lanes
// serves one destination: lane j sums the contributions lo+j, lo+j+16, ... of d's sorted segment
// in order, then the 16 partials are combined by a fixed xor tree, so the result is
// deterministic and a destination with many sources (a point many rows collapse onto) costs
// len/16 rounds instead of len.
constexpr int kGatherLanes = 16;
__global__ void chamfer_gather_kernel(const float* __restrict__ Dp, int ND,
                                      const float* __restrict__ Sp, int NR,
                                      const uint32_t* __restrict__ skeys,
                                      const uint32_t* __restrict__ svals,
                                      const float* __restrict__ gout, float sign,
                                      float* __restrict__ grad) {
  const int b = blockIdx.y;
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int d = t / kGatherLanes, j = t % kGatherLanes;
  const bool valid = d < ND;  // whole 16-lane groups share validity (256 % 16 == 0)
  const uint32_t* K = skeys + (int64_t)b * NR;
  int lo = 0, hi = valid ? NR : 0;  // lower bound of d
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (K[mid] < (uint32_t)d) lo = mid + 1; else hi = mid;
  }
  const float* q = Dp + ((int64_t)b * ND + (valid ? d : 0)) * 3;
  const float g = gout[b] * 2.0f / (float)NR;
  float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
  if (valid) {
    for (int k = lo + j; k < NR && K[k] == (uint32_t)d; k += kGatherLanes) {
      const int r = (int)svals[(int64_t)b * NR + k];
      const float* p = Sp + ((int64_t)b * NR + r) * 3;
      if (raw_pair(p, q) >= 0.0f) {
        a0 += g * (p[0] - q[0]);
        a1 += g * (p[1] - q[1]);
        a2 += g * (p[2] - q[2]);
      }
    }
  }
#pragma unroll
  for (int off = kGatherLanes / 2; off > 0; off >>= 1) {
    a0 += __shfl_xor(a0, off);
    a1 += __shfl_xor(a1, off);
    a2 += __shfl_xor(a2, off);
  }
  if (valid && j == 0) {
    float* o = grad + ((int64_t)b * ND + d) * 3;
    o[0] += -sign * a0;
    o[1] += -sign * a1;
    o[2] += -sign * a2;
  }
}

// ---- L1 (F.l1_loss, mean reduction): deterministic two-level float64 sum
constexpr int kL1Blocks = 512;
__global__ __launch_bounds__(256) void l1_partial_kernel(const float* __restrict__ a,
                                                         const float* __restrict__ b, int64_t n,
                                                         double* __restrict__ part) {
  __shared__ double s[256];
  double acc = 0.0;
  for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
    acc += fabs((double)a[e] - (double)b[e]);
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) s[threadIdx.x] += s[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = s[0];
}
__global__ void l1_final_kernel(const double* __restrict__ part, int np_, int64_t n,
                                float* __restrict__ out) {
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < np_; ++i) s += part[i];
    out[0] = (float)(s / (double)n);
  }
}
__global__ void l1_bwd_kernel(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                              const float* __restrict__ gout, float* __restrict__ ga) {
  const float g = gout[0] / (float)n;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const float d = a[e] - b[e];
    ga[e] = d > 0.0f ? g : (d < 0.0f ? -g : 0.0f);
  }
}

struct CdWS {
  uint32_t *kA, *vA, *kB, *vB, *hist;
  size_t bytes;
};
static CdWS carve_cd(void* base, int64_t B, int64_t R) {
  Carver c(base);
  CdWS w;
  w.kA = c.take<uint32_t>(B * R);
  w.vA = c.take<uint32_t>(B * R);
  w.kB = c.take<uint32_t>(B * R);
  w.vB = c.take<uint32_t>(B * R);
  w.hist = c.take<uint32_t>(radix_hist_words((int)B, R));
  w.bytes = c.bytes();
  return w;
}

}  // namespace pcst

using namespace pcst;

extern "C" int pcst_chamfer_fwd(const float* pred, const float* target, int64_t B, int64_t N,
                                int64_t M, float* min1, int32_t* arg1, float* min2,
                                int32_t* arg2, float* out, void* stream) {
  PCST_CHECK_ARG(B >= 0 && N > 0 && M > 0 && N < (1ll << 31) && M < (1ll << 31), "chamfer_fwd: bad shape");
  if (B == 0) return PCST_OK;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(chamfer_rowmin_kernel, dim3((unsigned)cdiv(N, 256), (unsigned)B), dim3(256), 0,
                     s, pred, target, (int)N, (int)M, min1, arg1);
  hipLaunchKernelGGL(chamfer_rowmin_kernel, dim3((unsigned)cdiv(M, 256), (unsigned)B), dim3(256), 0,
                     s, target, pred, (int)M, (int)N, min2, arg2);
  if (out)
    hipLaunchKernelGGL(chamfer_mean_kernel, dim3((unsigned)B), dim3(256), 0, s, min1, (int)N, min2,
                       (int)M, out);
  PCST_LAUNCH_CHECK("chamfer_fwd");
  return PCST_OK;
}

extern "C" int pcst_chamfer_bwd_workspace_size(int64_t B, int64_t N, int64_t M, size_t* bytes) {
  *bytes = carve_cd(nullptr, B, std::max(N, M)).bytes;
  return PCST_OK;
}

// grad_pred / grad_target (either may be NULL) are ACCUMULATED into (zero them first).
extern "C" int pcst_chamfer_bwd(const float* pred, const float* target, int64_t B, int64_t N,
                                int64_t M, const int32_t* arg1, const int32_t* arg2,
                                const float* grad_out, float* grad_pred, float* grad_target,
                                void* workspace, void* stream) {
  PCST_CHECK_ARG(B >= 0 && N > 0 && M > 0, "chamfer_bwd: bad shape");
  if (B == 0) return PCST_OK;
  hipStream_t s = as_stream(stream);
  CdWS w = carve_cd(workspace, B, std::max(N, M));
  const unsigned b = (unsigned)B;
  // direction 1 (pred rows -> target argmin): direct on pred, scattered on target
  if (grad_pred)
    hipLaunchKernelGGL(chamfer_direct_kernel, dim3((unsigned)cdiv(N, 256), b), dim3(256), 0, s,
                       pred, target, (int)N, (int)M, arg1, grad_out, 1.0f, grad_pred);
  if (grad_target) {
    hipLaunchKernelGGL(chamfer_keys_kernel, dim3((unsigned)std::min<int64_t>(cdiv(N, 256), 1024), b),
                       dim3(256), 0, s, arg1, (int)N, w.kA, w.vA);
    int rc = radix_sort_pairs(w.kA, w.vA, w.kB, w.vB, w.hist, (int)B, N, SegCounts{nullptr, (int32_t)N},
                              0, 32, s);
    if (rc) return rc;
    hipLaunchKernelGGL(chamfer_gather_kernel, dim3((unsigned)cdiv(M * kGatherLanes, 256), b),
                       dim3(256), 0, s, target, (int)M, pred, (int)N, w.kA, w.vA, grad_out, 1.0f,
                       grad_target);
  }
  // direction 2 (target rows -> pred argmin): direct on target, scattered on pred
  if (grad_target)
    hipLaunchKernelGGL(chamfer_direct_kernel, dim3((unsigned)cdiv(M, 256), b), dim3(256), 0, s,
                       target, pred, (int)M, (int)N, arg2, grad_out, 1.0f, grad_target);
  if (grad_pred) {
    hipLaunchKernelGGL(chamfer_keys_kernel, dim3((unsigned)std::min<int64_t>(cdiv(M, 256), 1024), b),
                       dim3(256), 0, s, arg2, (int)M, w.kA, w.vA);
    int rc = radix_sort_pairs(w.kA, w.vA, w.kB, w.vB, w.hist, (int)B, M, SegCounts{nullptr, (int32_t)M},
                              0, 32, s);
    if (rc) return rc;
    hipLaunchKernelGGL(chamfer_gather_kernel, dim3((unsigned)cdiv(N * kGatherLanes, 256), b),
                       dim3(256), 0, s, pred, (int)N, target, (int)M, w.kA, w.vA, grad_out, 1.0f,
                       grad_pred);
  }
  PCST_LAUNCH_CHECK("chamfer_bwd");
  return PCST_OK;
}

extern "C" int pcst_l1_workspace_size(size_t* bytes) {
  *bytes = sizeof(double) * kL1Blocks;
  return PCST_OK;
}

extern "C" int pcst_l1_fwd(const float* a, const float* b, int64_t n, float* out, void* workspace,
                           void* stream) {
  PCST_CHECK_ARG(n > 0 && a && b && out && workspace, "l1_fwd: bad args");
  hipStream_t s = as_stream(stream);
  const int g = (int)std::min<int64_t>(cdiv(n, 256), kL1Blocks);
  hipLaunchKernelGGL(l1_partial_kernel, dim3(g), dim3(256), 0, s, a, b, n, (double*)workspace);
  hipLaunchKernelGGL(l1_final_kernel, dim3(1), dim3(64), 0, s, (const double*)workspace, g, n, out);
  PCST_LAUNCH_CHECK("l1_fwd");
  return PCST_OK;
}

extern "C" int pcst_l1_bwd(const float* a, const float* b, int64_t n, const float* grad_out,
                           float* grad_a, void* stream) {
  PCST_CHECK_ARG(n > 0 && a && b && grad_out && grad_a, "l1_bwd: bad args");
  const int64_t g = std::min<int64_t>(cdiv(n, 256), 4096);
  hipLaunchKernelGGL(l1_bwd_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), a, b, n,
                     grad_out, grad_a);
  PCST_LAUNCH_CHECK("l1_bwd");
  return PCST_OK;
}
