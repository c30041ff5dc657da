// Evaluation metrics on the device: evaluation/metrics.py:20-203 and
// compare.py:6-43 all reduce to nearest-neighbour distances between two clouds, which the
// reference gets from torch.cdist (an N x M matrix: 57.6 GB at 120k) or sklearn / cKDTree on the
// host.  Two kernels:
//
//  * knn_dist: for every query row of P [B,N,3], its K nearest rows of Q [B,M,3] (K <= 16),
//    refs streamed through LDS in tiles, one query per thread.  Screening uses fp32 squared
//    distances from direct differences (no |p|^2+|q|^2-2pq cancellation); the K survivors'
//    Euclidean distances are then recomputed in float64, as sklearn / cKDTree / scipy compute
//    them from the fp32 inputs.  Ties go to the lower index.
//
//  * emd_greedy: earth_mover_distance's greedy matching (metrics.py:46-90), one 1024-thread
//    workgroup per cloud: for i in order, the nearest still-unused target j (scipy cdist
//    float64 distance sqrt((dx^2 + dy^2) + dz^2), strict < over ascending j, so the lowest j
//    wins ties), then mark j used.  The running total is summed in i order in float64, exactly
//    like the Python loop, and out[b] = float(total / N).
#include "common.h"

namespace pcst {

constexpr int kMtTile = 2048;

__device__ __forceinline__ float sq_direct(float px, float py, float pz, float qx, float qy,
                                           float qz) {
  const float dx = fsub(px, qx), dy = fsub(py, qy), dz = fsub(pz, qz);
  return fadd(fadd(fmul(dx, dx), fmul(dy, dy)), fmul(dz, dz));
}

__device__ __forceinline__ double dist_f64(const float* p, const float* q) {
  const double dx = dsub((double)p[0], (double)q[0]);
  const double dy = dsub((double)p[1], (double)q[1]);
  const double dz = dsub((double)p[2], (double)q[2]);
  return __dsqrt_rn(dadd(dadd(dmul(dx, dx), dmul(dy, dy)), dmul(dz, dz)));
}

template <int K>
__global__ __launch_bounds__(256) void knn_dist_kernel(const float* __restrict__ P,
                                                       const float* __restrict__ Q, int N, int M,
                                                       int k, double* __restrict__ dist,
                                                       int32_t* __restrict__ idx) {
  __shared__ float4 sq[kMtTile];
  const int b = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const bool valid = i < N;
  const float* p = P + ((int64_t)b * N + (valid ? i : 0)) * 3;
  const float px = p[0], py = p[1], pz = p[2];
  float bd[K];
  int bi[K];
#pragma unroll
  for (int s = 0; s < K; ++s) {
    bd[s] = INFINITY;
    bi[s] = -1;
  }
  const float* Qb = Q + (int64_t)b * M * 3;
  for (int t0 = 0; t0 < M; t0 += kMtTile) {
    const int tn = min(kMtTile, M - t0);
    __syncthreads();
    for (int e = threadIdx.x; e < tn; e += 256) {
      const float* q = Qb + (int64_t)(t0 + e) * 3;
      sq[e] = make_float4(q[0], q[1], q[2], 0.0f);
    }
    __syncthreads();
#pragma unroll 4
    for (int e = 0; e < tn; ++e) {
      const float4 q = sq[e];
      const float d = sq_direct(px, py, pz, q.x, q.y, q.z);
      if (d < bd[K - 1]) {  // sorted insertion; equal distances keep the earlier (lower) index
        const int j = t0 + e;
#pragma unroll
        for (int s = K - 1; s > 0; --s) {
          const bool shift = d < bd[s - 1];
          const bool place = !shift && d < bd[s];
          bd[s] = shift ? bd[s - 1] : (place ? d : bd[s]);
          bi[s] = shift ? bi[s - 1] : (place ? j : bi[s]);
        }
        if (d < bd[0]) {
          bd[0] = d;
          bi[0] = j;
        }
      }
    }
  }
  if (!valid) return;
  // exact float64 distances of the survivors, re-ranked (ties to the lower index)
  double dd[K];
#pragma unroll
  for (int s = 0; s < K; ++s) dd[s] = bi[s] >= 0 ? dist_f64(p, Qb + (int64_t)bi[s] * 3) : INFINITY;
#pragma unroll
  for (int a = 1; a < K; ++a) {
#pragma unroll
    for (int s = a; s > 0; --s) {
      const bool sw = dd[s] < dd[s - 1] || (dd[s] == dd[s - 1] && (unsigned)bi[s] < (unsigned)bi[s - 1]);
      if (sw) {
        const double td = dd[s];
        dd[s] = dd[s - 1];
        dd[s - 1] = td;
        const int ti = bi[s];
        bi[s] = bi[s - 1];
        bi[s - 1] = ti;
      }
    }
  }
  const int64_t o = ((int64_t)b * N + i) * k;
#pragma unroll
  for (int s = 0; s < K; ++s) {
    if (s < k) {
      dist[o + s] = dd[s];
      if (idx) idx[o + s] = bi[s];
    }
  }
}

constexpr int kEmdThreads = 1024;

__device__ __forceinline__ bool emd_better(double d, int j, double bd, int bj) {
  return d < bd || (d == bd && (unsigned)j < (unsigned)bj);
}

constexpr int kEmdMaxM = 1 << 18;  // the used-target bitmap lives in LDS (32 KB)

__global__ __launch_bounds__(kEmdThreads) void emd_greedy_kernel(const float* __restrict__ P,
                                                                 const float* __restrict__ Q,
                                                                 int N, int M,
                                                                 float* __restrict__ out) {
  __shared__ uint32_t used[kEmdMaxM / 32];
  __shared__ double wd[kEmdThreads / 64];
  __shared__ int wj[kEmdThreads / 64];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int words = (M + 31) >> 5;
  for (int w = tid; w < words; w += kEmdThreads) used[w] = 0u;
  __syncthreads();
  const float* Pb = P + (int64_t)b * N * 3;
  const float* Qb = Q + (int64_t)b * M * 3;
  double total = 0.0;
  for (int i = 0; i < N; ++i) {
    const float* p = Pb + (int64_t)i * 3;
    double bd = INFINITY;
    int bj = -1;
    for (int j = tid; j < M; j += kEmdThreads) {
      if ((used[j >> 5] >> (j & 31)) & 1u) continue;
      const double d = dist_f64(p, Qb + (int64_t)j * 3);
      if (d < bd) {  // ascending j per thread: strict < keeps the lowest
        bd = d;
        bj = j;
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double od = __shfl_xor(bd, off);
      const int oj = __shfl_xor(bj, off);
      if (oj >= 0 && (bj < 0 || emd_better(od, oj, bd, bj))) {
        bd = od;
        bj = oj;
      }
    }
    if (lane == 0) {
      wd[wid] = bd;
      wj[wid] = bj;
    }
    __syncthreads();
    if (tid == 0) {
      double fd = INFINITY;
      int fj = -1;
      for (int w = 0; w < kEmdThreads / 64; ++w)
        if (wj[w] >= 0 && (fj < 0 || emd_better(wd[w], wj[w], fd, fj))) {
          fd = wd[w];
          fj = wj[w];
        }
      if (fj >= 0) {
        total = dadd(total, fd);
        used[fj >> 5] |= 1u << (fj & 31);
      }
    }
    __syncthreads();
  }
  if (tid == 0) out[b] = (float)(total / (double)N);
}

}  // namespace pcst

using namespace pcst;

extern "C" int pcst_knn_dist(const float* P, const float* Q, int64_t B, int64_t N, int64_t M,
                             int64_t k, double* dist, int32_t* idx, void* stream) {
  PCST_CHECK_ARG(B >= 0 && N >= 0 && M > 0 && N < (1ll << 31) && M < (1ll << 31),
                 "knn_dist: bad shape");
  PCST_CHECK_ARG(k >= 1 && k <= 16 && k <= M, "knn_dist: need 1 <= k <= min(16, M)");
  if (B == 0 || N == 0) return PCST_OK;
  PCST_CHECK_ARG(P && Q && dist, "knn_dist: null pointer");
  hipStream_t s = as_stream(stream);
  dim3 g((unsigned)cdiv(N, 256), (unsigned)B);
  if (k == 1)
    hipLaunchKernelGGL(knn_dist_kernel<1>, g, dim3(256), 0, s, P, Q, (int)N, (int)M, (int)k, dist, idx);
  else if (k <= 4)
    hipLaunchKernelGGL(knn_dist_kernel<4>, g, dim3(256), 0, s, P, Q, (int)N, (int)M, (int)k, dist, idx);
  else if (k <= 9)
    hipLaunchKernelGGL(knn_dist_kernel<9>, g, dim3(256), 0, s, P, Q, (int)N, (int)M, (int)k, dist, idx);
  else
    hipLaunchKernelGGL(knn_dist_kernel<16>, g, dim3(256), 0, s, P, Q, (int)N, (int)M, (int)k, dist, idx);
  PCST_LAUNCH_CHECK("knn_dist");
  return PCST_OK;
}

extern "C" int pcst_emd_greedy(const float* P, const float* Q, int64_t B, int64_t N, int64_t M,
                               float* out, void* stream) {
  PCST_CHECK_ARG(B >= 0 && N > 0 && M > 0 && M <= kEmdMaxM, "emd_greedy: bad shape (M <= 262144)");
  if (B == 0) return PCST_OK;
  PCST_CHECK_ARG(P && Q && out, "emd_greedy: null pointer");
  hipLaunchKernelGGL(emd_greedy_kernel, dim3((unsigned)B), dim3(kEmdThreads), 0, as_stream(stream),
                     P, Q, (int)N, (int)M, out);
  PCST_LAUNCH_CHECK("emd_greedy");
  return PCST_OK;
}
