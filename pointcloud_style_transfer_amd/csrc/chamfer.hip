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
  auto row_of = [&](int w) {  // the row of slot w, or N (none)
    const int k = blockIdx.x * 256 * R + w * 256 + r;
    return k < N ? k : N;
  };
  float mx[R], my[R], mz[R], np_[R];
  cd_f2 mx2[R], my2[R], mz2[R], np2[R];
#pragma unroll
  for (int w = 0; w < R; ++w) {
    const int i = row_of(w);
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
    const int i = row_of(w);
    const int bj = bchunk[w] * kCdChunk + (found[w] < kCdChunk ? found[w] : 0);
    if (i < N) {
      mind[(int64_t)b * N + i] = best[w];
      argm[(int64_t)b * N + i] = bj < M ? bj : 0;
    }
  }
}

// out[b] = mean(m1[b]) + mean(m2[b]), fixed-order float64 reduction (one workgroup per cloud;
// 1024 threads, 8 loads in flight per thread)
__device__ __forceinline__ double cd_block_sum(const float* __restrict__ m, int n) {
  double a = 0.0;
  int i = threadIdx.x;
  for (; i + 7 * 1024 < n; i += 8 * 1024) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = m[i + u * 1024];
#pragma unroll
    for (int u = 0; u < 8; ++u) a += (double)v[u];
  }
  for (; i < n; i += 1024) a += (double)m[i];
  return a;
}

__global__ __launch_bounds__(1024) void chamfer_mean_kernel(const float* __restrict__ m1, int N,
                                                            const float* __restrict__ m2, int M,
                                                            float* __restrict__ out) {
  const int b = blockIdx.x;
  __shared__ double s1[1024], s2[1024];
  s1[threadIdx.x] = cd_block_sum(m1 + (int64_t)b * N, N);
  s2[threadIdx.x] = cd_block_sum(m2 + (int64_t)b * M, M);
  __syncthreads();
  for (int off = 512; off > 0; off >>= 1) {
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

// The same sums as a segmented reduction over the sorted (destination, row) pairs, so a
// destination that many rows share (a noisy predicted x0: thousands of target rows on one
// predicted point) costs one pass over its entries in parallel instead of a serial loop of 16
// lanes.  chamfer_segsum_kernel: kSegE consecutive entries per block; a segmented inclusive scan
// (thread-serial over 4 entries, then a block scan of (head seen, sum) pairs) gives every
// segment end its sum since max(segment head, block start).  A segment that starts and ends in
// the block is written by it (its only writer).  The block records its first segment's partial
// when that segment began in an earlier block and ends here, and its last segment's partial when
// that segment runs on past the block.  chamfer_segfix_kernel: the block holding a spanning
// segment's end adds the earlier blocks' partials, walking back to the segment's head.  The
// summation order is fixed, so the gradient is deterministic.
constexpr int kSegPer = 4;
constexpr int kSegE = 256 * kSegPer;  // entries per block
__device__ __forceinline__ void seg_op(int& f, float (&a)[3], int f2, const float (&b)[3]) {
  // (f, a) (+) (f2, b): b restarts at a head
#pragma unroll
  for (int c = 0; c < 3; ++c) a[c] = f2 ? b[c] : a[c] + b[c];
  f |= f2;
}
__global__ __launch_bounds__(256) void chamfer_segsum_kernel(
    const float* __restrict__ Dp, int ND, const float* __restrict__ Sp, int NR,
    const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ svals,
    const float* __restrict__ gout, float sign, float* __restrict__ grad, int nblk,
    float4* __restrict__ part, int* __restrict__ pflag) {
  const int b = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x;
  const int base = blk * kSegE;
  const uint32_t* K = skeys + (int64_t)b * NR;
  const uint32_t* V = svals + (int64_t)b * NR;
  const float g = gout[b] * 2.0f / (float)NR;
  // this thread's entries: values and head flags
  float v[kSegPer][3];
  int hd[kSegPer];
  uint32_t key[kSegPer];
  const int k0 = base + tid * kSegPer;
#pragma unroll
  for (int u = 0; u < kSegPer; ++u) {
    const int k = k0 + u;
    v[u][0] = v[u][1] = v[u][2] = 0.0f;
    hd[u] = 1;
    key[u] = 0xffffffffu;
    if (k < NR) {
      key[u] = K[k];
      hd[u] = k == 0 || K[k - 1] != key[u];
      const int d = (int)key[u], r = (int)V[k];
      const float* q = Dp + ((int64_t)b * ND + (d < ND ? d : 0)) * 3;
      const float* p = Sp + ((int64_t)b * NR + r) * 3;
      if (raw_pair(p, q) >= 0.0f) {
        v[u][0] = g * (p[0] - q[0]);
        v[u][1] = g * (p[1] - q[1]);
        v[u][2] = g * (p[2] - q[2]);
      }
    }
  }
  // thread-serial segmented scan, then the thread aggregates across the block
  float s[kSegPer][3];
  int f = hd[0];
  float acc[3] = {v[0][0], v[0][1], v[0][2]};
#pragma unroll
  for (int c = 0; c < 3; ++c) s[0][c] = acc[c];
#pragma unroll
  for (int u = 1; u < kSegPer; ++u) {
    seg_op(f, acc, hd[u], v[u]);
#pragma unroll
    for (int c = 0; c < 3; ++c) s[u][c] = acc[c];
  }
  // inclusive block scan of (f, acc) over threads (wave shuffles, then the waves in LDS)
  const int lane = tid & 63, wv = tid >> 6;
  int fi = f;
  float ai[3] = {acc[0], acc[1], acc[2]};
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int fo = __shfl_up(fi, off);
    float ao[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) ao[c] = __shfl_up(ai[c], off);
    if (lane >= off) {  // (fo, ao) (+) (fi, ai)
      float r[3] = {ao[0], ao[1], ao[2]};
      int fr = fo;
      seg_op(fr, r, fi, ai);
      fi = fr;
#pragma unroll
      for (int c = 0; c < 3; ++c) ai[c] = r[c];
    }
  }
  __shared__ float wsum[4][3];
  __shared__ int wflag[4];
  if (lane == 63) {
    wflag[wv] = fi;
#pragma unroll
    for (int c = 0; c < 3; ++c) wsum[wv][c] = ai[c];
  }
  __syncthreads();
  // exclusive prefix for this thread: the waves before, then the lanes before
  int fx = 0;
  float ax[3] = {0.0f, 0.0f, 0.0f};
  for (int w = 0; w < wv; ++w) {
    float t[3] = {wsum[w][0], wsum[w][1], wsum[w][2]};
    seg_op(fx, ax, wflag[w], t);
  }
  {
    const int fl = __shfl_up(fi, 1);
    float al[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) al[c] = __shfl_up(ai[c], 1);
    if (lane > 0) seg_op(fx, ax, fl, al);
  }
  // the block's first segment began in an earlier block and ends in this one: segfix completes
  // it (a flag per block, written every call)
  if (tid == 0 && base < NR) {
    const uint32_t k0key = K[base];
    const int last = min(base + kSegE, NR) - 1;
    const bool spans_in = base > 0 && K[base - 1] == k0key;
    const bool runs_on = K[last] == k0key && last + 1 < NR && K[last + 1] == k0key;
    pflag[b * nblk + blk] = spans_in && !runs_on;
  }
  // entries: carry-in until the thread's first head
#pragma unroll
  for (int u = 0; u < kSegPer; ++u) {
    const int k = k0 + u;
    if (k >= NR) break;
    // sum of this entry's segment since max(head, block start) up to k
    bool head_seen = false;  // a head among this thread's entries 0..u
#pragma unroll
    for (int w = 0; w <= u; ++w) head_seen |= hd[w] != 0;
    float tot[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) tot[c] = head_seen ? s[u][c] : ax[c] + s[u][c];
    const bool head_in_block = head_seen || fx != 0;  // the segment's head lies in this block
    const bool seg_end = k == NR - 1 || K[k + 1] != key[u];
    if (seg_end) {
      if (head_in_block) {
        float* o = grad + ((int64_t)b * ND + key[u]) * 3;
        o[0] += -sign * tot[0];
        o[1] += -sign * tot[1];
        o[2] += -sign * tot[2];
      } else {  // began in an earlier block: this block holds its end (segfix completes it)
        part[((int64_t)b * nblk + blk) * 2] = make_float4(tot[0], tot[1], tot[2], 0.0f);
      }
    } else if (k == base + kSegE - 1) {  // runs on past the block: this block's portion
      part[((int64_t)b * nblk + blk) * 2 + 1] = make_float4(tot[0], tot[1], tot[2], 0.0f);
    }
  }
}

__global__ void chamfer_segfix_kernel(int ND, int NR, const uint32_t* __restrict__ skeys, float sign,
                                      float* __restrict__ grad, int nblk,
                                      const float4* __restrict__ part, int* __restrict__ pflag) {
  const int b = blockIdx.y, blk = blockIdx.x * 256 + threadIdx.x;
  if (blk >= nblk || !pflag[b * nblk + blk]) return;
  const uint32_t* K = skeys + (int64_t)b * NR;
  const float4 e = part[((int64_t)b * nblk + blk) * 2];
  float t[3] = {e.x, e.y, e.z};
  const uint32_t key = K[blk * kSegE];
  // walk back over the blocks the segment runs through: each contributes its last portion
  for (int j = blk - 1; j >= 0; --j) {
    const float4 q = part[((int64_t)b * nblk + j) * 2 + 1];
    t[0] += q.x;
    t[1] += q.y;
    t[2] += q.z;
    if (j == 0 || K[j * kSegE - 1] != key) break;  // the segment's head is in block j
  }
  float* o = grad + ((int64_t)b * ND + key) * 3;
  o[0] += -sign * t[0];
  o[1] += -sign * t[1];
  o[2] += -sign * t[2];
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
  float4* part;  // [B][blocks][2] segmented-sum partials (chamfer_segsum_kernel)
  int* pflag;    // [B][blocks]
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
  w.part = c.take<float4>(B * cdiv(R, kSegE) * 2);
  w.pflag = c.take<int>(B * cdiv(R, kSegE));
  w.bytes = c.bytes();
  return w;
}


// ---- Grid-pruned exact row minima (large clouds).  Each cloud is counting-sorted into a
// uniform grid (~kCgPerCell points per cell); a row searches Chebyshev rings of cells around
// its own cell, nearest first, and skips a cell (or stops the search) when a conservative
// lower bound of the COMPUTED distance there exceeds its best so far.  The bound is the exact
// box distance shrunk by the fp32 error of the expanded formula (|D_computed - D| <= ~7u
// (|p|^2 + |q|^2) + u|D|, bounded with 16u (|p|^2 + max|q|^2)), so no pair that could reach the
// row's clamped minimum is skipped; pairs are scored by cd_dist itself and ranked by
// (clamped value, original index): bit-identical to the exhaustive first-index argmin, in any
// visiting order.  A row's rings cost ~27 cells x kCgPerCell pairs instead of M.
constexpr int kCgPerCell = 8;        // points per cell at the density an average point sees
constexpr int kCgMaxCells = 262144;  // per cloud
constexpr int kCgTile = 1024;        // scan tile (cells)
constexpr int kCgHist = 16;          // bins per axis of the density histogram
constexpr float kCgU = 5.9604645e-08f;  // 2^-24

struct CgGrid {
  float o[3];
  float h, inv_h, slack, nmax;
  int d[3];
};

__global__ __launch_bounds__(1024) void cg_stats_kernel(const float* __restrict__ P,
                                                        const float* __restrict__ Q, int N, int M,
                                                        CgGrid* __restrict__ grids) {
  const int b = blockIdx.x, side = blockIdx.y;  // side 0: pred (P), 1: target (Q)
  const int n = side ? M : N;
  const float* X = (side ? Q + (int64_t)b * M * 3 : P + (int64_t)b * N * 3);
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY}, nm = 0.0f;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const float x = X[i * 3], y = X[i * 3 + 1], z = X[i * 3 + 2];
    lo[0] = fminf(lo[0], x); lo[1] = fminf(lo[1], y); lo[2] = fminf(lo[2], z);
    hi[0] = fmaxf(hi[0], x); hi[1] = fmaxf(hi[1], y); hi[2] = fmaxf(hi[2], z);
    nm = fmaxf(nm, sqnorm3(x, y, z));
  }
  __shared__ float red[7][32];
  float v[7] = {lo[0], lo[1], lo[2], -hi[0], -hi[1], -hi[2], -nm};
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    for (int off = 32; off >= 1; off >>= 1) v[k] = fminf(v[k], __shfl_xor(v[k], off));
    if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = v[k];
  }
  __syncthreads();
  __shared__ float bb[7];
  __shared__ int hist[kCgHist * kCgHist * kCgHist];
  for (int i = threadIdx.x; i < kCgHist * kCgHist * kCgHist; i += 1024) hist[i] = 0;
  if (threadIdx.x == 0) {
    for (int k = 0; k < 7; ++k) {
      float r = red[k][0];
      for (int w = 1; w < 16; ++w) r = fminf(r, red[k][w]);
      bb[k] = r;
    }
  }
  __syncthreads();
  // density histogram over the bounding box: the cell size follows the PEAK density
  {
    float hinv[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float e = fmaxf(-bb[3 + a] - bb[a], 1e-30f);
      hinv[a] = kCgHist / e;
    }
    for (int i = threadIdx.x; i < n; i += 1024) {
      int c[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const float f = (X[i * 3 + a] - bb[a]) * hinv[a];
        c[a] = f >= 0.0f ? (int)fminf(f, (float)(kCgHist - 1)) : 0;
      }
      atomicAdd(&hist[(c[2] * kCgHist + c[1]) * kCgHist + c[0]], 1);
    }
  }
  __syncthreads();
  // sum of count^2 over the bins: n x the bin occupancy an average POINT sees
  double hsq = 0.0;
  for (int i = threadIdx.x; i < kCgHist * kCgHist * kCgHist; i += 1024) hsq += (double)hist[i] * hist[i];
  for (int off = 32; off >= 1; off >>= 1) hsq += __shfl_xor(hsq, off);
  __shared__ double hred[16];
  if ((threadIdx.x & 63) == 0) hred[threadIdx.x >> 6] = hsq;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; ++w) hsq += hred[w];
    float r[7];
    for (int k = 0; k < 7; ++k) r[k] = bb[k];
    CgGrid g;
    float ext[3], vol = 1.0f, span = 0.0f;
    for (int a = 0; a < 3; ++a) {
      g.o[a] = r[a];
      ext[a] = fmaxf(-r[3 + a] - r[a], 0.0f);
      span = fmaxf(span, ext[a] + fabsf(r[a]));
    }
    const float emax = fmaxf(fmaxf(ext[0], ext[1]), fmaxf(ext[2], 1e-30f));
    for (int a = 0; a < 3; ++a) vol *= fmaxf(ext[a], emax * 1e-3f);
    // the density an average point sees (point-weighted over the histogram bins); cells hold
    // ~kCgPerCell points there: dense regions get more per cell, sparse rows fewer rings
    const float bin_vol = vol / (float)(kCgHist * kCgHist * kCgHist);
    const float dens = (float)fmax(hsq / fmax((double)n, 1.0), 1.0) / bin_vol;
    float h = cbrtf((float)kCgPerCell / dens);
    if (!(h > 1e-30f) || !(h < INFINITY)) h = fmaxf(emax, 1.0f);  // degenerate cloud
    for (int it = 0; it < 64; ++it) {  // grow h until the cell count fits
      int64_t c = 1;
      for (int a = 0; a < 3; ++a) c *= (int64_t)fminf(ceilf(ext[a] / h) + 1.0f, 4096.0f);
      if (c <= kCgMaxCells) break;
      h *= 1.25f;
    }
    g.h = h;
    g.inv_h = 1.0f / h;
    for (int a = 0; a < 3; ++a) g.d[a] = (int)fminf(ceilf(ext[a] / h) + 1.0f, 4096.0f);
    // cell assignment uses (x - o) * inv_h in fp32; boxes are widened by this slack
    g.slack = 1e-3f * h + 4e-6f * span;
    g.nmax = -r[6];
    grids[b * 2 + side] = g;
  }
}

__device__ __forceinline__ int cg_cell_coord(float x, float o, float inv_h, int d) {
  const float f = (x - o) * inv_h;  // clamped in float: no out-of-range int conversion
  return f >= 0.0f ? (int)fminf(f, (float)(d - 1)) : 0;
}

// per point: its cell and rank in the cell (one atomic on the cell's count)
__global__ void cg_count_kernel(const float* __restrict__ P, const float* __restrict__ Q, int N,
                                int M, const CgGrid* __restrict__ grids, int* __restrict__ counts,
                                int2* __restrict__ crank) {
  const int b = blockIdx.y, side = blockIdx.z;
  const int n = side ? M : N;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* X = side ? Q + ((int64_t)b * M + i) * 3 : P + ((int64_t)b * N + i) * 3;
  const CgGrid g = grids[b * 2 + side];
  const int cx = cg_cell_coord(X[0], g.o[0], g.inv_h, g.d[0]);
  const int cy = cg_cell_coord(X[1], g.o[1], g.inv_h, g.d[1]);
  const int cz = cg_cell_coord(X[2], g.o[2], g.inv_h, g.d[2]);
  const int cell = (cz * g.d[1] + cy) * g.d[0] + cx;
  const int rank = atomicAdd(&counts[(int64_t)(b * 2 + side) * (kCgMaxCells + 1) + cell], 1);
  crank[(int64_t)(b * 2 + side) * (N > M ? N : M) + i] = make_int2(cell, rank);
}

// exclusive scan of one cloud's cell counts, in two launches: per-tile sums, then each tile
// adds the sums of the tiles before it (<= kCgMaxCells / kCgTile of them) to its own block scan
// (starts in a separate array; starts[C] = n for every C <= kCgMaxCells past the last cell)
__global__ __launch_bounds__(kCgTile) void cg_tilesum_kernel(const int* __restrict__ counts,
                                                             int* __restrict__ tsum) {
  const int64_t slot = blockIdx.y;
  const int v = counts[slot * (kCgMaxCells + 1) + (int64_t)blockIdx.x * kCgTile + threadIdx.x];
  int s = v;
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
  __shared__ int ws[kCgTile / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kCgTile / 64; ++w) t += ws[w];
    tsum[slot * (kCgMaxCells / kCgTile) + blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kCgTile) void cg_scan_kernel(const int* __restrict__ counts,
                                                          const int* __restrict__ tsum,
                                                          int* __restrict__ starts) {
  const int64_t slot = blockIdx.y;
  constexpr int T = kCgMaxCells / kCgTile;
  __shared__ int ws[kCgTile / 64];
  __shared__ int base_s;
  if (threadIdx.x < 64) {  // offset of this tile: sum of the earlier tiles' sums
    int b = 0;
    for (int t = threadIdx.x; t < (int)blockIdx.x; t += 64) b += tsum[slot * T + t];
    for (int off = 32; off >= 1; off >>= 1) b += __shfl_xor(b, off);
    if (threadIdx.x == 0) base_s = b;
  }
  const int64_t e = (int64_t)blockIdx.x * kCgTile + threadIdx.x;
  const int v = counts[slot * (kCgMaxCells + 1) + e];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int inc = v;
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(inc, off);
    if (lane >= off) inc += t;
  }
  if (lane == 63) ws[wv] = inc;
  __syncthreads();
  int pre = base_s;
  for (int w = 0; w < wv; ++w) pre += ws[w];
  starts[slot * (kCgMaxCells + 1) + e] = pre + inc - v;
  if (blockIdx.x == T - 1 && threadIdx.x == kCgTile - 1)
    starts[slot * (kCgMaxCells + 1) + kCgMaxCells] = pre + inc;
}

__global__ void cg_fill_kernel(const float* __restrict__ P, const float* __restrict__ Q, int N,
                               int M, const int* __restrict__ starts,
                               const int2* __restrict__ crank, float4* __restrict__ sorted,
                               int* __restrict__ sidx) {
  const int b = blockIdx.y, side = blockIdx.z;
  const int n = side ? M : N;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t slot = (int64_t)(b * 2 + side);
  const int NM = N > M ? N : M;
  const float* X = side ? Q + ((int64_t)b * M + i) * 3 : P + ((int64_t)b * N + i) * 3;
  const int2 cr = crank[slot * NM + i];
  const int pos = starts[slot * (kCgMaxCells + 1) + cr.x] + cr.y;
  const float x = X[0], y = X[1], z = X[2];
  sorted[slot * NM + pos] = make_float4(x, y, z, sqnorm3(x, y, z));
  sidx[slot * NM + pos] = i;
}

__device__ __forceinline__ float cg_axis_gap(float p, float lo, float hi) {
  return p < lo ? lo - p : (p > hi ? p - hi : 0.0f);
}

// rows: side s's sorted points; grid: side 1-s.  Writes min/arg at the row's original index.
// ring_budget > 0 (the hybrid mode): a row still open after that many rings around its cell
// (a row far from the other cloud, whose search would sweep a thin shell of the whole grid)
// is appended to its overflow list instead (ovf_rows[b*2+side][*], count ovf_count[b*2+side];
// list order is irrelevant) and the exhaustive row-min serves it.
__global__ __launch_bounds__(256) void cg_rowmin_kernel(int N, int M,
                                                        const CgGrid* __restrict__ grids,
                                                        const int* __restrict__ starts,
                                                        const float4* __restrict__ sorted,
                                                        const int* __restrict__ sidx,
                                                        float* __restrict__ min1,
                                                        int32_t* __restrict__ arg1,
                                                        float* __restrict__ min2,
                                                        int32_t* __restrict__ arg2,
                                                        int ring_budget,
                                                        int* __restrict__ ovf_count,
                                                        int* __restrict__ ovf_rows) {
  const int b = blockIdx.y, side = blockIdx.z;  // side 0: pred rows vs target grid
  const int n = side ? M : N;
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int NM = N > M ? N : M;
  const int64_t rs = (int64_t)(b * 2 + side), ts = (int64_t)(b * 2 + 1 - side);
  const float4 p = sorted[rs * NM + r];
  const int row = sidx[rs * NM + r];
  const CgGrid g = grids[ts];
  const int* S = starts + ts * (kCgMaxCells + 1);
  const float4* T = sorted + ts * NM;
  const int* TI = sidx + ts * NM;
  const float px = p.x, py = p.y, pz = p.z, np_ = p.w;
  const float err = 16.0f * kCgU * (np_ + g.nmax) + 1e-30f;
  const float shrink = 1.0f - 8.0f * kCgU;
  const int cx = cg_cell_coord(px, g.o[0], g.inv_h, g.d[0]);
  const int cy = cg_cell_coord(py, g.o[1], g.inv_h, g.d[1]);
  const int cz = cg_cell_coord(pz, g.o[2], g.inv_h, g.d[2]);
  float best = INFINITY;
  int bi = 0x7fffffff;
  const int rmax = max(max(g.d[0], g.d[1]), g.d[2]);
  for (int ring = 0; ring <= rmax; ++ring) {
    if (ring > 0 && best != INFINITY) {
      // distance from p to the outside of the box of rings < ring (interior faces only)
      // lower bound for every unvisited cell: the box distance from p to the slab of the
      // grid beyond each interior face of the box of rings < ring (p may lie outside the grid)
      float lb = INFINITY;
      bool any = false;
      const int c3[3] = {cx, cy, cz};
      const float p3[3] = {px, py, pz};
      float glo[3], ghi[3], gin[3];  // grid box and p's gap to it per axis
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        glo[a] = g.o[a] - g.slack;
        ghi[a] = g.o[a] + g.d[a] * g.h + g.slack;
        gin[a] = cg_axis_gap(p3[a], glo[a], ghi[a]);
      }
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const int lo = c3[a] - (ring - 1), hi = c3[a] + (ring - 1);
        const float o2 = gin[(a + 1) % 3] * gin[(a + 1) % 3] + gin[(a + 2) % 3] * gin[(a + 2) % 3];
        if (lo > 0) {
          any = true;
          const float ga = cg_axis_gap(p3[a], glo[a], g.o[a] + lo * g.h + g.slack);
          lb = fminf(lb, ga * ga + o2);
        }
        if (hi < g.d[a] - 1) {
          any = true;
          const float ga = cg_axis_gap(p3[a], g.o[a] + (hi + 1) * g.h - g.slack, ghi[a]);
          lb = fminf(lb, ga * ga + o2);
        }
      }
      if (!any) break;  // the rings so far cover the whole grid
      if (lb * shrink - err > best) break;
    }
    if (ring_budget > 0 && ring > ring_budget) {  // over budget: the exhaustive pass takes it
      const int at = atomicAdd(&ovf_count[rs], 1);
      ovf_rows[rs * NM + at] = row;
      return;
    }
    const int z0 = max(cz - ring, 0), z1 = min(cz + ring, g.d[2] - 1);
    const int y0 = max(cy - ring, 0), y1 = min(cy + ring, g.d[1] - 1);
    const int x0 = max(cx - ring, 0), x1 = min(cx + ring, g.d[0] - 1);
    auto visit = [&](int x, int y, int z) {
      const float gx = cg_axis_gap(px, g.o[0] + x * g.h - g.slack, g.o[0] + (x + 1) * g.h + g.slack);
      const float gy = cg_axis_gap(py, g.o[1] + y * g.h - g.slack, g.o[1] + (y + 1) * g.h + g.slack);
      const float gz = cg_axis_gap(pz, g.o[2] + z * g.h - g.slack, g.o[2] + (z + 1) * g.h + g.slack);
      if (best != INFINITY && (gx * gx + gy * gy + gz * gz) * shrink - err > best) return;
      const int cell = (z * g.d[1] + y) * g.d[0] + x;
      const int k1 = S[cell + 1];
      for (int k = S[cell]; k < k1; ++k) {
        const float4 q = T[k];
        float v = cd_dist(px, py, pz, np_, q.x, q.y, q.z, q.w);
        v = v < 0.0f ? 0.0f : v;
        const int j = TI[k];
        if (v < best || (v == best && j < bi)) {
          best = v;
          bi = j;
        }
      }
    };
    // the cells at Chebyshev distance exactly `ring` from the row's cell, inside the grid
    for (int z = z0; z <= z1; ++z)
      for (int y = y0; y <= y1; ++y) {
        if (z == cz - ring || z == cz + ring || y == cy - ring || y == cy + ring) {
          for (int x = x0; x <= x1; ++x) visit(x, y, z);
        } else {
          if (cx - ring >= 0) visit(cx - ring, y, z);
          if (cx + ring <= g.d[0] - 1) visit(cx + ring, y, z);
        }
      }
  }
  if (bi == 0x7fffffff) bi = 0;  // no comparable pair (NaN row): the exhaustive kernel's answer
  if (side == 0) {
    min1[(int64_t)b * N + row] = best;
    arg1[(int64_t)b * N + row] = bi;
  } else {
    min2[(int64_t)b * M + row] = best;
    arg2[(int64_t)b * M + row] = bi;
  }
}

// ---- The rows over the ring budget (hybrid mode) by box pruning.  Each cloud's cell-sorted
// points are cut into boxes of kCgBoxPts consecutive points (a run of neighbouring cells) with
// their exact bounding boxes, and the boxes into superboxes of kCgSbBoxes.  One wave per row:
// the superboxes' distance lower bounds (lane = superbox), the nearest box of the nearest
// superbox scanned for a first best (lane = point), then, eight kept superboxes at a time (lane =
// one of their boxes), every box the ring search's own conservative test (lb * shrink - err >
// best) cannot rule out.  Pairs are scored by cd_dist and ranked by (clamped value, original
// index) as in cg_rowmin_kernel: the exhaustive first-index argmin, bit for bit, in any visiting
// order.  A far row scans a few boxes (5-6 on average, tools/cd_box_probe.py) instead of M points.
constexpr int kCgBoxPts = 64;
constexpr int kCgSbBoxes = 8;

// boxes[slot][box] = {lo.xyz, hi.xyz} of sorted points [64 box, 64 box + 64), sboxes[slot][sb]
// the same over boxes [8 sb, 8 sb + 8) (NaN points drop out).  One 512-thread block per superbox.
__global__ __launch_bounds__(512) void cg_box_kernel(int N, int M, const float4* __restrict__ sorted,
                                                     float4* __restrict__ boxes,
                                                     float4* __restrict__ sboxes) {
  const int b = blockIdx.y, side = blockIdx.z;
  const int n = side ? M : N;
  const int NM = N > M ? N : M;
  const int nbs = (NM + kCgBoxPts - 1) / kCgBoxPts;
  const int nss = (nbs + kCgSbBoxes - 1) / kCgSbBoxes;
  const int sb = blockIdx.x;
  if (sb * kCgSbBoxes * kCgBoxPts >= n) return;  // block-uniform
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int box = sb * kCgSbBoxes + w;
  const int i = box * kCgBoxPts + lane;
  const int64_t slot = b * 2 + side;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  if (i < n) {
    const float4 q = sorted[slot * NM + i];
    lo[0] = hi[0] = q.x;
    lo[1] = hi[1] = q.y;
    lo[2] = hi[2] = q.z;
  }
#pragma unroll
  for (int a = 0; a < 3; ++a)
    for (int off = 32; off >= 1; off >>= 1) {
      lo[a] = fminf(lo[a], __shfl_xor(lo[a], off));
      hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off));
    }
  __shared__ float red[kCgSbBoxes][6];
  if (lane == 0) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      red[w][a] = lo[a];
      red[w][3 + a] = hi[a];
    }
    if (box * kCgBoxPts < n) {
      boxes[(slot * nbs + box) * 2] = make_float4(lo[0], lo[1], lo[2], 0.0f);
      boxes[(slot * nbs + box) * 2 + 1] = make_float4(hi[0], hi[1], hi[2], 0.0f);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int v = 1; v < kCgSbBoxes; ++v)
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        lo[a] = fminf(lo[a], red[v][a]);
        hi[a] = fmaxf(hi[a], red[v][3 + a]);
      }
    sboxes[(slot * nss + sb) * 2] = make_float4(lo[0], lo[1], lo[2], 0.0f);
    sboxes[(slot * nss + sb) * 2 + 1] = make_float4(hi[0], hi[1], hi[2], 0.0f);
  }
}

// (v, j) into (best, bi) by (value, index); NaN never enters
__device__ __forceinline__ void cg_take(float v, int j, float& best, int& bi) {
  if (v < best || (v == best && j < bi)) {
    best = v;
    bi = j;
  }
}

template <int kFrom = 32>
__device__ __forceinline__ void cg_wave_argmin(float& best, int& bi) {
  for (int off = kFrom; off >= 1; off >>= 1) {
    const float ov = __shfl_xor(best, off);
    const int oj = __shfl_xor(bi, off);
    cg_take(ov, oj, best, bi);
  }
}

// grid (blocks, B, 2): the waves of (cloud b, side) stride over that side's overflow list
__global__ __launch_bounds__(256) void cg_list_box_kernel(
    const float* __restrict__ P, const float* __restrict__ Q, int N, int M,
    const CgGrid* __restrict__ grids, const float4* __restrict__ sorted,
    const int* __restrict__ sidx, const float4* __restrict__ boxes,
    const float4* __restrict__ sboxes, const int* __restrict__ ovf_count,
    const int* __restrict__ ovf_rows, float* __restrict__ min1, int32_t* __restrict__ arg1,
    float* __restrict__ min2, int32_t* __restrict__ arg2) {
  const int b = blockIdx.y, side = blockIdx.z;  // side 0: pred rows vs the target's boxes
  const int NM = N > M ? N : M;
  const int nbs = (NM + kCgBoxPts - 1) / kCgBoxPts;
  const int nss = (nbs + kCgSbBoxes - 1) / kCgSbBoxes;
  const int64_t rs = b * 2 + side, ts = b * 2 + 1 - side;
  const int m = side ? N : M;  // the other cloud's points
  const int nbox = (m + kCgBoxPts - 1) / kCgBoxPts;
  const int nsb = (nbox + kCgSbBoxes - 1) / kCgSbBoxes;
  const int lane = threadIdx.x & 63;
  const int count = ovf_count[rs];
  const int* __restrict__ L = ovf_rows + rs * NM;
  const float4* __restrict__ T = sorted + ts * NM;
  const int* __restrict__ TI = sidx + ts * NM;
  const float4* __restrict__ Bx = boxes + ts * nbs * 2;
  const float4* __restrict__ Sx = sboxes + ts * nss * 2;
  const float gnmax = grids[ts].nmax;
  const float shrink = 1.0f - 8.0f * kCgU;
  const int waves = gridDim.x * 4;
  for (int k = blockIdx.x * 4 + (int)(threadIdx.x >> 6); k < count; k += waves) {
    const int row = L[k];
    const float* X = side ? Q + ((int64_t)b * M + row) * 3 : P + ((int64_t)b * N + row) * 3;
    const float px = X[0], py = X[1], pz = X[2];
    const float np_ = sqnorm3(px, py, pz);
    const float err = 16.0f * kCgU * (np_ + gnmax) + 1e-30f;
    auto lbound = [&](const float4* __restrict__ Bs, int c) {
      const float4 lo = Bs[2 * c], hi = Bs[2 * c + 1];
      const float gx = cg_axis_gap(px, lo.x, hi.x), gy = cg_axis_gap(py, lo.y, hi.y);
      const float gz = cg_axis_gap(pz, lo.z, hi.z);
      return gx * gx + gy * gy + gz * gz;
    };
    float best = INFINITY;
    int bi = 0x7fffffff;
    auto scan = [&](int c) {  // lane = point of box c
      const int kk = c * kCgBoxPts + lane;
      if (kk < m) {
        const float4 q = T[kk];
        float v = cd_dist(px, py, pz, np_, q.x, q.y, q.z, q.w);
        v = v < 0.0f ? 0.0f : v;
        cg_take(v, TI[kk], best, bi);
      }
    };
    // the first best: the nearest box (by bound) of the nearest superbox
    float lmin = INFINITY;
    int smin = 0;
    float slb = INFINITY;  // this lane's superbox bound among the first 64 (reused below)
    for (int c = lane; c < nsb; c += 64) {
      const float v = lbound(Sx, c);
      if (c < 64) slb = v;
      cg_take(v, c, lmin, smin);
    }
    cg_wave_argmin(lmin, smin);
    smin = __builtin_amdgcn_readfirstlane(smin);
    lmin = INFINITY;
    int cmin = smin * kCgSbBoxes;
    {
      const int c = smin * kCgSbBoxes + (lane & (kCgSbBoxes - 1));
      if (c < nbox) cg_take(lbound(Bx, c), c, lmin, cmin);
    }
    cg_wave_argmin<kCgSbBoxes / 2>(lmin, cmin);
    cmin = __builtin_amdgcn_readfirstlane(cmin);
    scan(cmin);
    // the superboxes the bound keeps, eight at a time: lane group g takes the g-th kept one
    for (int s0 = 0; s0 < nsb; s0 += 64) {
      cg_wave_argmin(best, bi);
      const int sc = s0 + lane;
      uint64_t smask = __ballot(sc < nsb && !((s0 ? lbound(Sx, sc) : slb) * shrink - err > best));
      while (smask) {
        cg_wave_argmin(best, bi);  // the tightest bound so far for this batch's boxes
        uint64_t mg = smask;
        for (int g = 0; g < (lane >> 3); ++g) mg &= mg - 1;
#pragma unroll
        for (int g = 0; g < 64 / kCgSbBoxes; ++g) smask &= smask - 1;
        const int c = mg ? (s0 + __builtin_ctzll(mg)) * kCgSbBoxes + (lane & (kCgSbBoxes - 1)) : nbox;
        uint64_t bmask = __ballot(c < nbox && c != cmin && !(lbound(Bx, c) * shrink - err > best));
        while (bmask) {
          const int bit = __builtin_ctzll(bmask);
          bmask &= bmask - 1;
          scan(__builtin_amdgcn_readlane(c, bit));
        }
      }
    }
    cg_wave_argmin(best, bi);
    if (lane == 0) {
      if (bi == 0x7fffffff) bi = 0;  // no comparable pair (NaN row)
      if (side == 0) {
        min1[(int64_t)b * N + row] = best;
        arg1[(int64_t)b * N + row] = bi;
      } else {
        min2[(int64_t)b * M + row] = best;
        arg2[(int64_t)b * M + row] = bi;
      }
    }
  }
}

struct CgWS {
  CgGrid* grids;
  int* counts;     // [B][2][kCgMaxCells + 1]
  int* starts;     // [B][2][kCgMaxCells + 1]
  int* tsum;       // [B][2][kCgMaxCells / kCgTile]
  int2* crank;     // [B][2][NM]
  float4* sorted;  // [B][2][NM]
  int* sidx;       // [B][2][NM]
  int* ovf_count;  // [B][2]       hybrid mode: rows over the ring budget
  int* ovf_rows;   // [B][2][NM]
  float4* boxes;   // [B][2][NM / kCgBoxPts][2]  hybrid mode: sorted-point boxes (lo, hi)
  float4* sboxes;  // [B][2][boxes / kCgSbBoxes][2]  and their superboxes
  size_t bytes;
};
static CgWS carve_cg(void* base, int64_t B, int64_t N, int64_t M) {
  Carver c(base);
  const int64_t NM = std::max(N, M);
  CgWS w;
  w.grids = c.take<CgGrid>(B * 2);
  w.counts = c.take<int>(B * 2 * (kCgMaxCells + 1));
  w.starts = c.take<int>(B * 2 * (kCgMaxCells + 1));
  w.tsum = c.take<int>(B * 2 * (kCgMaxCells / kCgTile));
  w.crank = c.take<int2>(B * 2 * NM);
  w.sorted = c.take<float4>(B * 2 * NM);
  w.sidx = c.take<int>(B * 2 * NM);
  w.ovf_count = c.take<int>(B * 2);
  w.ovf_rows = c.take<int>(B * 2 * NM);
  w.boxes = c.take<float4>(B * 2 * cdiv(NM, kCgBoxPts) * 2);
  w.sboxes = c.take<float4>(B * 2 * cdiv(cdiv(NM, kCgBoxPts), kCgSbBoxes) * 2);
  w.bytes = c.bytes();
  return w;
}

}  // namespace pcst

using namespace pcst;

static inline int64_t cd_padded(int64_t n) { return cdiv(n, kCdChunk) * kCdChunk; }

// The grid path wins when the two clouds overlap (8 x 30000 lidar-like pairs 2.0 -> 0.32 ms),
// but a row far outside the other cloud's grid has to search the thin shell of points within
// its nearest distance, which grows with the distance: a noisy predicted x0 against its target
// (the trainer's early timesteps) measured 46-60 ms.  The hybrid mode (3, and the default 0)
// bounds that: the grid search gives up after kCgRingBudget rings and the rows it gave up on (a
// list per cloud and side) are served by box pruning (cg_list_box_kernel; round 4 measured it
// against the exhaustive row-min over the list).  Measured on the trainer's pair (a predicted x0
// = lidar-like target + noise, 8 x 30000 per side, tools/cd_sweep.sh): noise 0.02: exhaustive
// 2.08 ms, grid 0.32, hybrid 0.34; noise 0.2: 2.10 / 1.34 / 1.43; noise 1: 2.09 / 16.9 / 1.25;
// noise 4: 2.10 / 62.5 / 1.28.  All modes give bit-identical minima and first-index argmins.
// blocks (4 waves) per cloud and side of cg_list_box_kernel (r04 a48: 512 9.61-9.65 ms per trainer
// step, 128 9.80-9.89)
constexpr int kCgListBlocks = 512;
constexpr int kCgRingBudget = 2;  // rings the grid search tries before a row joins the list (r04 a47)
static bool cd_use_grid(int mode) { return mode == 0 || mode == 2 || mode == 3; }
static size_t cd_exh_bytes(int64_t B, int64_t N, int64_t M) {
  return (sizeof(float) * 4 * (size_t)B * (size_t)(cd_padded(N) + cd_padded(M)) + 255) / 256 * 256;
}

extern "C" int pcst_chamfer_fwd_workspace_size(int64_t B, int64_t N, int64_t M, size_t* bytes) {
  PCST_CHECK_ARG(B >= 0 && N > 0 && M > 0 && bytes, "chamfer_fwd_workspace_size: bad args");
  *bytes = cd_exh_bytes(B, N, M) + carve_cg(nullptr, B, N, M).bytes;
  return PCST_OK;
}

extern "C" int pcst_chamfer_fwd(const float* pred, const float* target, int64_t B, int64_t N,
                                int64_t M, float* min1, int32_t* arg1, float* min2,
                                int32_t* arg2, float* out, int mode, void* workspace,
                                void* stream) {
  PCST_CHECK_ARG(B >= 0 && N > 0 && M > 0 && N < (1ll << 30) && M < (1ll << 30), "chamfer_fwd: bad shape");
  PCST_CHECK_ARG(mode >= 0 && mode <= 3,
                 "chamfer_fwd: mode is 0 (auto), 1 (exhaustive), 2 (grid) or 3 (hybrid)");
  if (B == 0) return PCST_OK;
  PCST_CHECK_ARG(pred && target && min1 && arg1 && min2 && arg2 && workspace, "chamfer_fwd: null pointer");
  hipStream_t s = as_stream(stream);
  const unsigned b = (unsigned)B;
  const int64_t Np = cd_padded(N), Mp = cd_padded(M);
  float4* Pp = static_cast<float4*>(workspace);  // pred packed, B x Np/2 pairs x 2
  float4* Tp = Pp + B * Np;                       // target packed
  auto pack = [&]() {
    hipLaunchKernelGGL(chamfer_pack_kernel, dim3((unsigned)cdiv(Np / 2, 256), b), dim3(256), 0, s,
                       pred, (int)N, (int)Np, Pp);
    hipLaunchKernelGGL(chamfer_pack_kernel, dim3((unsigned)cdiv(Mp / 2, 256), b), dim3(256), 0, s,
                       target, (int)M, (int)Mp, Tp);
  };
  if (cd_use_grid(mode)) {
    const bool hybrid = mode != 2;
    CgWS w = carve_cg(static_cast<char*>(workspace) + cd_exh_bytes(B, N, M), B, N, M);
    const int64_t NM = std::max(N, M);
    PCST_HIP(hipMemsetAsync(w.counts, 0, sizeof(int) * B * 2 * (kCgMaxCells + 1), s), "memset");
    if (hybrid) PCST_HIP(hipMemsetAsync(w.ovf_count, 0, sizeof(int) * B * 2, s), "memset");
    hipLaunchKernelGGL(cg_stats_kernel, dim3(b, 2), dim3(1024), 0, s, pred, target, (int)N, (int)M,
                       w.grids);
    const dim3 pg((unsigned)cdiv(NM, 256), b, 2);
    hipLaunchKernelGGL(cg_count_kernel, pg, dim3(256), 0, s, pred, target, (int)N, (int)M, w.grids,
                       w.counts, w.crank);
    const dim3 tg((unsigned)(kCgMaxCells / kCgTile), b * 2);
    hipLaunchKernelGGL(cg_tilesum_kernel, tg, dim3(kCgTile), 0, s, w.counts, w.tsum);
    hipLaunchKernelGGL(cg_scan_kernel, tg, dim3(kCgTile), 0, s, w.counts, w.tsum, w.starts);
    hipLaunchKernelGGL(cg_fill_kernel, pg, dim3(256), 0, s, pred, target, (int)N, (int)M, w.starts,
                       w.crank, w.sorted, w.sidx);
    hipLaunchKernelGGL(cg_rowmin_kernel, pg, dim3(256), 0, s, (int)N, (int)M, w.grids, w.starts,
                       w.sorted, w.sidx, min1, arg1, min2, arg2, hybrid ? kCgRingBudget : 0,
                       w.ovf_count, w.ovf_rows);
    if (hybrid) {  // the rows over budget: box-pruned scans
      const int nbs = (int)cdiv(NM, kCgBoxPts);
      hipLaunchKernelGGL(cg_box_kernel, dim3((unsigned)cdiv(nbs, kCgSbBoxes), b, 2), dim3(512), 0, s,
                         (int)N, (int)M, w.sorted, w.boxes, w.sboxes);
      const unsigned lb = (unsigned)std::min<int64_t>(cdiv(NM, 64), kCgListBlocks);
      hipLaunchKernelGGL(cg_list_box_kernel, dim3(lb, b, 2), dim3(256), 0, s, pred, target, (int)N,
                         (int)M, w.grids, w.sorted, w.sidx, w.boxes, w.sboxes, w.ovf_count, w.ovf_rows, min1,
                         arg1, min2, arg2);
    }
    if (out)
      hipLaunchKernelGGL(chamfer_mean_kernel, dim3(b), dim3(1024), 0, s, min1, (int)N, min2, (int)M,
                         out);
    PCST_LAUNCH_CHECK("chamfer_fwd");
    return PCST_OK;
  }
  pack();
  // 2 segments x 1 row per thread (the S x R sweep of round 3: 11 / 41 / 12 / 22 / 14 / 42 slower)
  auto rowmin = [&](const float* P, const float4* Qp, int64_t n, int64_t m, int64_t mp, float* md,
                    int32_t* am) {
    hipLaunchKernelGGL((chamfer_rowmin_kernel<2, 1>), dim3((unsigned)cdiv(n, 256), b), dim3(512), 0, s,
                       P, Qp, (int)n, (int)m, (int)mp, md, am);
  };
  rowmin(pred, Tp, N, M, Mp, min1, arg1);
  rowmin(target, Pp, M, N, Np, min2, arg2);
  if (out)
    hipLaunchKernelGGL(chamfer_mean_kernel, dim3(b), dim3(1024), 0, s, min1, (int)N, min2, (int)M,
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
  // the scatter onto the argmin side from the sorted (destination, row) pairs: segmented sums
  auto seg_gather = [&](const float* D, int ND, const float* S, int NR, const float* go, float* gr) {
    const int nblk = (int)cdiv(NR, kSegE);
    hipLaunchKernelGGL(chamfer_segsum_kernel, dim3((unsigned)nblk, b), dim3(256), 0, s, D, ND, S, NR,
                       w.kA, w.vA, go, 1.0f, gr, nblk, w.part, w.pflag);
    hipLaunchKernelGGL(chamfer_segfix_kernel, dim3((unsigned)cdiv(nblk, 256), b), dim3(256), 0, s, ND,
                       NR, w.kA, 1.0f, gr, nblk, w.part, w.pflag);
  };
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
    seg_gather(target, (int)M, pred, (int)N, grad_out, grad_target);
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
    seg_gather(pred, (int)N, target, (int)M, grad_out, grad_pred);
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
