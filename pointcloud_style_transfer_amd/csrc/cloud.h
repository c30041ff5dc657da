// Per-cloud reductions and scans shared by several kernels (internal linkage).
//  - cloud statistics (min, max, sum, sum of squares per axis) as a two-level reduction:
//    per-block partial records, no contended atomics; consumers fold the partials;
//  - exclusive scan of a long u32 array per segment (tile reduce -> tile-sum scan -> tile
//    scan), all loads coalesced.
#pragma once
#include "common.h"

namespace pcst {
namespace {  // internal linkage: included by several translation units

constexpr int kStatBlocks = 64;  // partial records per cloud

struct StatRec {
  float mn[3], mx[3];
  double s[3], ss[3];
};

// One 256-thread block's partial record (block blk of kStatBlocks) of cloud P: part[blk].
__device__ __forceinline__ void cloud_stats_block(const float* __restrict__ P, int N, int blk,
                                                  StatRec* __restrict__ part) {
  float mn[3] = {3.4e38f, 3.4e38f, 3.4e38f}, mx[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
  double s[3] = {0, 0, 0}, ss[3] = {0, 0, 0};
  // eight of the thread's points per round, all loads in flight before the (in-order) sums
  constexpr int kU = 8, kStride = kStatBlocks * 256;
  for (int n0 = blk * 256 + threadIdx.x; n0 < N; n0 += kU * kStride) {
    float v[kU][3];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int n = n0 + u * kStride;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[u][c] = n < N ? P[n * 3 + c] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (n0 + u * kStride >= N) break;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        mn[c] = fminf(mn[c], v[u][c]);
        mx[c] = fmaxf(mx[c], v[u][c]);
        s[c] += v[u][c];
        ss[c] += (double)v[u][c] * v[u][c];
      }
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      mn[c] = fminf(mn[c], __shfl_xor(mn[c], off));
      mx[c] = fmaxf(mx[c], __shfl_xor(mx[c], off));
      s[c] += __shfl_xor(s[c], off);
      ss[c] += __shfl_xor(ss[c], off);
    }
  }
  __shared__ StatRec w[4];
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    for (int c = 0; c < 3; ++c) {
      w[wid].mn[c] = mn[c]; w[wid].mx[c] = mx[c]; w[wid].s[c] = s[c]; w[wid].ss[c] = ss[c];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    StatRec r = w[0];
    for (int q = 1; q < 4; ++q)
      for (int c = 0; c < 3; ++c) {
        r.mn[c] = fminf(r.mn[c], w[q].mn[c]);
        r.mx[c] = fmaxf(r.mx[c], w[q].mx[c]);
        r.s[c] += w[q].s[c];
        r.ss[c] += w[q].ss[c];
      }
    part[blk] = r;
  }
}

__global__ __launch_bounds__(256) void cloud_stats_partial_kernel(const float* __restrict__ pts,
                                                                  int N, StatRec* __restrict__ part) {
  const int b = blockIdx.y;
  cloud_stats_block(pts + (int64_t)b * N * 3, N, blockIdx.x, part + b * kStatBlocks);
}

// Fold the partial records of cloud b (fixed order: deterministic).
__device__ __forceinline__ StatRec fold_stats(const StatRec* __restrict__ part, int b) {
  StatRec r = part[b * kStatBlocks];
  for (int q = 1; q < kStatBlocks; ++q) {
    const StatRec& o = part[b * kStatBlocks + q];
    for (int c = 0; c < 3; ++c) {
      r.mn[c] = fminf(r.mn[c], o.mn[c]);
      r.mx[c] = fmaxf(r.mx[c], o.mx[c]);
      r.s[c] += o.s[c];
      r.ss[c] += o.ss[c];
    }
  }
  return r;
}

// Same fold by one 64-lane wave (lane q reads partial q, butterfly combine): call from all
// lanes of a wave; every lane returns the result.  (Float min/max are order-free; the float64
// sums are combined in a fixed butterfly order, so the result is deterministic.)
__device__ __forceinline__ StatRec fold_stats_wave(const StatRec* __restrict__ part, int b) {
  static_assert(kStatBlocks == 64, "one partial per lane");
  const int lane = threadIdx.x & 63;
  StatRec r = part[b * kStatBlocks + lane];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      r.mn[c] = fminf(r.mn[c], __shfl_xor(r.mn[c], off));
      r.mx[c] = fmaxf(r.mx[c], __shfl_xor(r.mx[c], off));
      r.s[c] += __shfl_xor(r.s[c], off);
      r.ss[c] += __shfl_xor(r.ss[c], off);
    }
  }
  return r;
}

inline void launch_cloud_stats(const float* pts, int B, int N, StatRec* part, hipStream_t s) {
  hipLaunchKernelGGL(cloud_stats_partial_kernel, dim3(kStatBlocks, B), dim3(256), 0, s, pts, N,
                     part);
}

// ---- exclusive scan of `len` u32 per segment (stride `stride`), in place, optional totals.
constexpr int kScanItems = 16;
constexpr int kScanTile = 256 * kScanItems;  // 4096

__device__ __forceinline__ uint32_t block_excl_scan_256(uint32_t v, uint32_t* sh, uint32_t& total) {
  // sh: 256 + 4 words
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) sh[256 + w] = x;
  __syncthreads();
  uint32_t wofs = 0;
  for (int q = 0; q < w; ++q) wofs += sh[256 + q];
  total = sh[256] + sh[257] + sh[258] + sh[259];
  __syncthreads();
  return wofs + x - v;
}

__global__ __launch_bounds__(256) void scan_tile_sum_kernel(const uint32_t* __restrict__ data,
                                                            int64_t len, int64_t stride,
                                                            uint32_t* __restrict__ tsum, int tiles) {
  const int seg = blockIdx.y, tile = blockIdx.x;
  const uint32_t* D = data + seg * stride;
  const int64_t base = (int64_t)tile * kScanTile;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int64_t i = base + k * 256 + threadIdx.x;
    if (i < len) acc += D[i];
  }
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
  __shared__ uint32_t w[4];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) tsum[(int64_t)seg * tiles + tile] = w[0] + w[1] + w[2] + w[3];
}

// single workgroup per segment: exclusive scan of up to 256*kScanItems tile sums
__global__ __launch_bounds__(256) void scan_tsum_kernel(uint32_t* __restrict__ tsum, int tiles,
                                                        int32_t* __restrict__ total) {
  const int seg = blockIdx.x;
  uint32_t* T = tsum + (int64_t)seg * tiles;
  __shared__ uint32_t sh[260];
  uint32_t carry = 0;
  for (int base = 0; base < tiles; base += 256) {
    const int i = base + threadIdx.x;
    const uint32_t v = i < tiles ? T[i] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan_256(v, sh, tot);
    if (i < tiles) T[i] = carry + ex;
    carry += tot;
  }
  if (total && threadIdx.x == 0) total[seg] = (int32_t)carry;
}

// tile-local scan (items blocked per thread via LDS transpose) + tile offset
__global__ __launch_bounds__(256) void scan_tile_kernel(uint32_t* __restrict__ data, int64_t len,
                                                        int64_t stride,
                                                        const uint32_t* __restrict__ toff, int tiles) {
  const int seg = blockIdx.y, tile = blockIdx.x;
  uint32_t* D = data + seg * stride;
  const int64_t base = (int64_t)tile * kScanTile;
  __shared__ uint32_t buf[kScanTile + kScanTile / 32];
  __shared__ uint32_t sh[260];
  auto pad = [](int i) { return i + (i >> 5); };
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int j = k * 256 + threadIdx.x;
    const int64_t i = base + j;
    buf[pad(j)] = i < len ? D[i] : 0u;
  }
  __syncthreads();
  uint32_t v[kScanItems], s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = buf[pad(threadIdx.x * kScanItems + k)];
    s += v[k];
  }
  uint32_t tot;
  uint32_t run = block_excl_scan_256(s, sh, tot) + toff[(int64_t)seg * tiles + tile];
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    buf[pad(threadIdx.x * kScanItems + k)] = run;
    run += v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int j = k * 256 + threadIdx.x;
    const int64_t i = base + j;
    if (i < len) D[i] = buf[pad(j)];
  }
}

inline size_t scan_tsum_words(int nseg, int64_t len) { return (size_t)nseg * cdiv(len, kScanTile); }

// One workgroup per segment, whole array staged in LDS (len <= kSmallScanMax): coalesced
// load, 16 contiguous entries per thread, block scan, coalesced store.  total[seg] optional.
constexpr int kSmallScanMax = 16384;
__global__ __launch_bounds__(1024) void seg_scan_small_kernel(uint32_t* __restrict__ data, int len,
                                                              int64_t stride,
                                                              int32_t* __restrict__ total) {
  __shared__ uint32_t buf[kSmallScanMax + kSmallScanMax / 32];
  __shared__ uint32_t wsum[16];
  uint32_t* D = data + blockIdx.x * stride;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  auto pad = [](int i) { return i + (i >> 5); };
  for (int i = t; i < kSmallScanMax; i += 1024) buf[pad(i)] = i < len ? D[i] : 0u;
  __syncthreads();
  uint32_t v[16], s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    v[k] = buf[pad(t * 16 + k)];
    s += v[k];
  }
  uint32_t x = s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t run = x - s;
  for (int q = 0; q < w; ++q) run += wsum[q];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    buf[pad(t * 16 + k)] = run;
    run += v[k];
  }
  if (total && t == 1023) total[blockIdx.x] = (int32_t)run;
  __syncthreads();
  for (int i = t; i < len; i += 1024) D[i] = buf[pad(i)];
}

inline void seg_scan_small(uint32_t* data, int nseg, int len, int64_t stride, int32_t* totals,
                           hipStream_t s) {
  hipLaunchKernelGGL(seg_scan_small_kernel, dim3(nseg), dim3(1024), 0, s, data, len, stride, totals);
}

// exclusive scan of data[seg*stride + 0..len) for every segment; totals[seg] if non-null.
inline void seg_scan_long(uint32_t* data, int nseg, int64_t len, int64_t stride, uint32_t* tsum,
                          int32_t* totals, hipStream_t s) {
  const int tiles = (int)cdiv(len, kScanTile);
  hipLaunchKernelGGL(scan_tile_sum_kernel, dim3(tiles, nseg), dim3(256), 0, s, data, len, stride,
                     tsum, tiles);
  hipLaunchKernelGGL(scan_tsum_kernel, dim3(nseg), dim3(256), 0, s, tsum, tiles, totals);
  hipLaunchKernelGGL(scan_tile_kernel, dim3(tiles, nseg), dim3(256), 0, s, data, len, stride, tsum,
                     tiles);
}

}  // namespace
}  // namespace pcst
