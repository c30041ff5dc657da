// Squared Chamfer distance of chamfer_distance_chunked_optimized (models/losses.py:8-63) and
// the L1 noise loss of DiffusionLoss (losses.py:90), forward and backward.
//
// Forward, per direction: D = (|p|^2 + |q|^2) + (-2 p.q) with the reference's rounding
// (dot = K=3 sgemm fma chain, unfused norms; -2*dot is exact so the final add is one fma),
// clamp >= 0, row min with the first index on ties.  Each thread owns one query row; the other
// cloud streams through scalar loads in packed point pairs (v_pk_* math, see below).  Never
// materialises the N x M matrix (the reference chunks 1024 rows to bound it).  Means are reduced deterministically (fixed-order float64).
//
// Backward (autograd of the reference formula): for a row i with argmin j and raw D >= 0,
// dL/dp_i += g/N * 2(p_i - q_j) and dL/dq_j -= the same.  The scatter onto the argmin side is
// made deterministic without float atomics: (argmin, row) pairs are radix-sorted (stable) and
// every destination sums its contributions in ascending row order.
#include "common.h"
#include "sort.h"

namespace pcst {

__device__ __forceinline__ float cd_dist(float px, float py, float pz, float np_, float qx,
                                         float qy, float qz, float nq) {
  const float dot = dot3(px, py, pz, qx, qy, qz);
  return ffma(-2.0f, dot, fadd(np_, nq));
}

// Row minima on packed fp32 math.  The D-side cloud is first repacked per point pair as
// {x0,x1,y0,y1} {z0,z1,n0,n1} (n = |q|^2; padding pairs carry n = +inf), so every v_pk_* op
// evaluates two pairs.  With m = -2p (a power-of-two scaling: every rounding step of the sgemm
// dot commutes with it), D = (|p|^2 + n) + fma(mz, z, fma(my, y, mx * x)) is bit-identical to
// cd_dist.  Since clamp(., 0) is monotone, min_k clamp(D_k) = clamp(min_k D_k): the inner loop
// keeps one raw minimum (v_min3 over two pairs) per chunk of kCdChunk points, the row keeps the
// first chunk reaching its best clamped value, and that chunk is re-scanned for the first index
// with clamp(D) == best -- the reference's first-index argmin of the clamped matrix.  The packed
// pairs are wave-uniform, so they arrive by scalar loads and cost no LDS traffic.
typedef float cd_f2 __attribute__((ext_vector_type(2)));
constexpr int kCdChunk = 256;  // points per argmin chunk (128 pairs)

__global__ void chamfer_pack_kernel(const float* __restrict__ Q, int M, int Mp,
                                    float4* __restrict__ Qp) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;  // pair index
  if (2 * j >= Mp) return;
  float v[2][4];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int k = 2 * j + u;
    if (k < M) {
      const float* q = Q + ((int64_t)b * M + k) * 3;
      v[u][0] = q[0];
      v[u][1] = q[1];
      v[u][2] = q[2];
      v[u][3] = sqnorm3(v[u][0], v[u][1], v[u][2]);
    } else {
      v[u][0] = v[u][1] = v[u][2] = 0.0f;
      v[u][3] = INFINITY;
    }
  }
  float4* o = Qp + ((int64_t)b * (Mp / 2) + j) * 2;
  o[0] = make_float4(v[0][0], v[1][0], v[0][1], v[1][1]);
  o[1] = make_float4(v[0][2], v[1][2], v[0][3], v[1][3]);
}

// raw D of 4 packed pairs (8 points) against R rows, folded into cmin[R]
template <int R>
__device__ __forceinline__ void cd_minpairs(const float4 (&q)[8], const cd_f2 (&mx2)[R],
                                            const cd_f2 (&my2)[R], const cd_f2 (&mz2)[R],
                                            const cd_f2 (&np2)[R], float (&cmin)[R]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float4 a = q[2 * u], e = q[2 * u + 1];
    const cd_f2 x = {a.x, a.y}, y = {a.z, a.w}, z = {e.x, e.y}, n = {e.z, e.w};
#pragma unroll
    for (int w = 0; w < R; ++w) {
      cd_f2 t = mx2[w] * x;
      t = __builtin_elementwise_fma(my2[w], y, t);
      t = __builtin_elementwise_fma(mz2[w], z, t);
      const cd_f2 d = (np2[w] + n) + t;
      cmin[w] = fminf(cmin[w], fminf(d.x, d.y));
    }
  }
}

// Block = S segments x 256 threads; a thread owns R rows (r + 256 w) of the block's 256 R rows
// against segment s's chunks [s*per, (s+1)*per).  R rows share every scalar load; S segments
// put more waves in flight.  The block combines the segments' (best, first chunk) in segment
// order, and the winning chunk's re-scan is split over the S segments the same way.
template <int S, int R>
__global__ __launch_bounds__(256 * S) void chamfer_rowmin_kernel(const float* __restrict__ P,
                                                                 const float4* __restrict__ Qp,
                                                                 int N, int M, int Mp,
                                                                 float* __restrict__ mind,
                                                                 int32_t* __restrict__ argm) {
  __shared__ float sbest[S][256 * R];
  __shared__ int sidx[S][256 * R];
  const int b = blockIdx.y;
  const int r = threadIdx.x & 255;
  const int seg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);  // wave-uniform
  float mx[R], my[R], mz[R], np_[R];
  cd_f2 mx2[R], my2[R], mz2[R], np2[R];
#pragma unroll
  for (int w = 0; w < R; ++w) {
    const int i = blockIdx.x * 256 * R + w * 256 + r;
    const float* p = P + ((int64_t)b * N + (i < N ? i : 0)) * 3;
    const float px = p[0], py = p[1], pz = p[2];
    np_[w] = sqnorm3(px, py, pz);
    mx[w] = -2.0f * px;
    my[w] = -2.0f * py;
    mz[w] = -2.0f * pz;
    mx2[w] = cd_f2{mx[w], mx[w]};
    my2[w] = cd_f2{my[w], my[w]};
    mz2[w] = cd_f2{mz[w], mz[w]};
    np2[w] = cd_f2{np_[w], np_[w]};
  }
  const float4* __restrict__ Qb = Qp + (int64_t)b * Mp;  // Mp/2 pairs x 2 float4
  const int chunks = Mp / kCdChunk;
  const int per = (chunks + S - 1) / S;
  const int c0 = seg * per, c1 = c0 + per < chunks ? c0 + per : chunks;
  float best[R];
  int bchunk[R];
#pragma unroll
  for (int w = 0; w < R; ++w) {
    best[w] = INFINITY;
    bchunk[w] = 0;
  }
  for (int c = c0; c < c1; ++c) {
    const float4* __restrict__ Qc = Qb + c * kCdChunk;
    float cmin[R];
#pragma unroll
    for (int w = 0; w < R; ++w) cmin[w] = INFINITY;
    // two 4-pair stages ping-pong in scalar registers
    float4 A[8], Bq[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) A[u] = Qc[u];
    for (int k = 0; k < kCdChunk / 2; k += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) Bq[u] = Qc[2 * (k + 4) + u];
      cd_minpairs<R>(A, mx2, my2, mz2, np2, cmin);
      const int kn = k + 8 < kCdChunk / 2 ? k + 8 : k;  // the last reload is a harmless repeat
#pragma unroll
      for (int u = 0; u < 8; ++u) A[u] = Qc[2 * kn + u];
      cd_minpairs<R>(Bq, mx2, my2, mz2, np2, cmin);
    }
#pragma unroll
    for (int w = 0; w < R; ++w) {
      const float cm = fmaxf(cmin[w], 0.0f);
      if (cm < best[w]) {
        best[w] = cm;
        bchunk[w] = c;
      }
    }
  }
  if (S > 1) {
#pragma unroll
    for (int w = 0; w < R; ++w) {
      sbest[seg][w * 256 + r] = best[w];
      sidx[seg][w * 256 + r] = bchunk[w];
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < R; ++w) {
      best[w] = INFINITY;
      bchunk[w] = 0;
#pragma unroll
      for (int t = 0; t < S; ++t)
        if (sbest[t][w * 256 + r] < best[w]) {  // strict: the earliest segment wins ties
          best[w] = sbest[t][w * 256 + r];
          bchunk[w] = sidx[t][w * 256 + r];
        }
    }
    __syncthreads();
  }
  // first index of the winning chunk whose clamped distance equals best; segment s scans its
  // 256/S points of the chunk
  constexpr int kPer = kCdChunk / S;
  int found[R];
#pragma unroll
  for (int w = 0; w < R; ++w) {
    found[w] = kCdChunk;
    const float4* Qc = Qb + bchunk[w] * kCdChunk;
    for (int k = seg * kPer; k < (seg + 1) * kPer; ++k) {
      const float4 a = Qc[2 * (k >> 1)], e = Qc[2 * (k >> 1) + 1];
      const int u = k & 1;
      const float x = u ? a.y : a.x, y = u ? a.w : a.z, z = u ? e.y : e.x, n = u ? e.w : e.z;
      const float t = ffma(mz[w], z, ffma(my[w], y, fmul(mx[w], x)));
      const float d = fadd(fadd(np_[w], n), t);
      if (fmaxf(d, 0.0f) == best[w]) {
        found[w] = k;
        break;
      }
    }
  }
  if (S > 1) {
#pragma unroll
    for (int w = 0; w < R; ++w) sidx[seg][w * 256 + r] = found[w];
    __syncthreads();
    if (seg != 0) return;
#pragma unroll
    for (int w = 0; w < R; ++w)
#pragma unroll
      for (int t = 1; t < S; ++t) found[w] = min(found[w], sidx[t][w * 256 + r]);
  }
#pragma unroll
  for (int w = 0; w < R; ++w) {
    const int i = blockIdx.x * 256 * R + w * 256 + r;
    const int bj = bchunk[w] * kCdChunk + (found[w] < kCdChunk ? found[w] : 0);
    if (i < N) {
      mind[(int64_t)b * N + i] = best[w];
      argm[(int64_t)b * N + i] = bj < M ? bj : 0;
    }
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

static inline int64_t cd_padded(int64_t n) { return cdiv(n, kCdChunk) * kCdChunk; }

extern "C" int pcst_chamfer_fwd_workspace_size(int64_t B, int64_t N, int64_t M, size_t* bytes) {
  PCST_CHECK_ARG(B >= 0 && N > 0 && M > 0 && bytes, "chamfer_fwd_workspace_size: bad args");
  *bytes = sizeof(float) * 4 * (size_t)B * (size_t)(cd_padded(N) + cd_padded(M));
  return PCST_OK;
}

extern "C" int pcst_chamfer_fwd(const float* pred, const float* target, int64_t B, int64_t N,
                                int64_t M, float* min1, int32_t* arg1, float* min2,
                                int32_t* arg2, float* out, void* workspace, void* stream) {
  PCST_CHECK_ARG(B >= 0 && N > 0 && M > 0 && N < (1ll << 30) && M < (1ll << 30), "chamfer_fwd: bad shape");
  if (B == 0) return PCST_OK;
  PCST_CHECK_ARG(pred && target && min1 && arg1 && min2 && arg2 && workspace, "chamfer_fwd: null pointer");
  hipStream_t s = as_stream(stream);
  const int64_t Np = cd_padded(N), Mp = cd_padded(M);
  float4* Pp = static_cast<float4*>(workspace);  // pred packed, B x Np/2 pairs x 2
  float4* Tp = Pp + B * Np;                       // target packed
  const unsigned b = (unsigned)B;
  hipLaunchKernelGGL(chamfer_pack_kernel, dim3((unsigned)cdiv(Np / 2, 256), b), dim3(256), 0, s,
                     pred, (int)N, (int)Np, Pp);
  hipLaunchKernelGGL(chamfer_pack_kernel, dim3((unsigned)cdiv(Mp / 2, 256), b), dim3(256), 0, s,
                     target, (int)M, (int)Mp, Tp);
  static const int variant = [] {  // S x R experiment knob: 11, 21, 41, 12, 22, 14
    const char* e = getenv("PCST_CD_VARIANT");
    return e ? atoi(e) : 21;
  }();
  auto rowmin = [&](const float* P, const float4* Qp, int64_t n, int64_t m, int64_t mp, float* md,
                    int32_t* am) {
#define PCST_CD_LAUNCH(S_, R_)                                                                  \
  hipLaunchKernelGGL((chamfer_rowmin_kernel<S_, R_>), dim3((unsigned)cdiv(n, 256 * R_), b),    \
                     dim3(256 * S_), 0, s, P, Qp, (int)n, (int)m, (int)mp, md, am)
    switch (variant) {
      case 11: PCST_CD_LAUNCH(1, 1); break;
      case 41: PCST_CD_LAUNCH(4, 1); break;
      case 12: PCST_CD_LAUNCH(1, 2); break;
      case 22: PCST_CD_LAUNCH(2, 2); break;
      case 14: PCST_CD_LAUNCH(1, 4); break;
      case 42: PCST_CD_LAUNCH(4, 2); break;
      default: PCST_CD_LAUNCH(2, 1); break;
    }
#undef PCST_CD_LAUNCH
  };
  rowmin(pred, Tp, N, M, Mp, min1, arg1);
  rowmin(target, Pp, M, N, Np, min2, arg2);
  if (out)
    hipLaunchKernelGGL(chamfer_mean_kernel, dim3(b), dim3(256), 0, s, min1, (int)N, min2, (int)M,
                       out);
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
