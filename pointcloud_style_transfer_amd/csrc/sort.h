// Segmented primitives shared by the voxel downsample, the kNN grid and Chamfer backward:
//  - stable LSD radix sort of (u32 key, u32 value) pairs, 8-bit digits, one segment per
//    point cloud (grid.y), per-segment element counts read from device memory so the
//    data-dependent sizes (unique voxels, pool size) never need a host round trip;
//  - per-segment exclusive scan of small tile tables (one workgroup per segment).
// Tiles are 4096 elements = 4 waves x 16 rounds x 64 lanes; element order inside a tile is
// (wave, round, lane), i.e. the input order, which is what makes the scatter stable.
#pragma once
#include "common.h"
#include "cloud.h"

namespace pcst {
namespace {  // internal linkage: included by several translation units

constexpr int kSortThreads = 256;
constexpr int kSortRounds = 16;
constexpr int kSortTile = kSortThreads * kSortRounds;  // 4096

struct SegCounts {
  const int32_t* dev;  // per-segment count on device, or null
  int32_t fixed;       // used when dev == null
  __device__ __forceinline__ int32_t get(int seg) const { return dev ? dev[seg] : fixed; }
};

// hist[seg][digit][tile] = number of keys of `digit` in the tile.
__global__ __launch_bounds__(kSortThreads) void radix_hist_kernel(
    const uint32_t* __restrict__ keys, int64_t cap, SegCounts counts, int shift, int tiles,
    uint32_t* __restrict__ hist) {
  const int seg = blockIdx.y, tile = blockIdx.x;
  const int n = counts.get(seg);
  const int base = tile * kSortTile;
  __shared__ uint32_t cnt[256];
  cnt[threadIdx.x] = 0;
  __syncthreads();
  if (base < n) {
    const uint32_t* K = keys + seg * cap;
    const int end = min(base + kSortTile, n);
    for (int i = base + threadIdx.x; i < end; i += kSortThreads)
      atomicAdd(&cnt[(K[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[((int64_t)seg * 256 + threadIdx.x) * tiles + tile] = cnt[threadIdx.x];
}

// Stable scatter of one 8-bit digit pass.
__global__ __launch_bounds__(kSortThreads) void radix_scatter_kernel(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin, uint32_t* __restrict__ kout,
    uint32_t* __restrict__ vout, int64_t cap, SegCounts counts, int shift, int tiles,
    const uint32_t* __restrict__ hist) {
  const int seg = blockIdx.y, tile = blockIdx.x;
  const int n = counts.get(seg);
  const int base = tile * kSortTile;
  if (base >= n) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ uint32_t wcnt[4][256];
#pragma unroll
  for (int q = 0; q < 4; ++q) wcnt[q][threadIdx.x] = 0;
  __syncthreads();
  const uint32_t* K = kin + seg * cap;
  const uint32_t* V = vin + seg * cap;
  uint32_t key[kSortRounds], val[kSortRounds];
  uint32_t rank[kSortRounds];
  const unsigned long long lt = lanemask_lt();
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int i = base + w * (kSortRounds * 64) + r * 64 + lane;
    const bool valid = i < n;
    key[r] = valid ? K[i] : 0u;
    val[r] = valid ? V[i] : 0u;
  }
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int i = base + w * (kSortRounds * 64) + r * 64 + lane;
    const bool valid = i < n;
    const uint32_t d = (key[r] >> shift) & 255u;
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const bool b = (d >> bit) & 1u;
      const unsigned long long mb = __ballot(b);
      peers &= b ? mb : ~mb;
    }
    uint32_t before = 0;
    if (valid) before = wcnt[w][d];
    const uint32_t pos = __popcll(peers & lt);
    const bool leader = valid && pos == 0;
    rank[r] = before + pos;
    __builtin_amdgcn_wave_barrier();
    if (leader) wcnt[w][d] = before + (uint32_t)__popcll(peers);
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  {
    const int d = threadIdx.x;
    uint32_t run = hist[((int64_t)seg * 256 + d) * tiles + tile];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t c = wcnt[q][d];
      wcnt[q][d] = run;
      run += c;
    }
  }
  __syncthreads();
  uint32_t* KO = kout + seg * cap;
  uint32_t* VO = vout + seg * cap;
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int i = base + w * (kSortRounds * 64) + r * 64 + lane;
    if (i < n) {
      const uint32_t d = (key[r] >> shift) & 255u;
      const uint32_t p = wcnt[w][d] + rank[r];
      KO[p] = key[r];
      VO[p] = val[r];
    }
  }
}

inline size_t radix_hist_words(int nseg, int64_t cap) {
  return (size_t)nseg * 256 * (size_t)cdiv(cap, kSortTile);
}

// Sort (keys, vals) of every segment by bits [begin_bit, end_bit); end_bit - begin_bit must
// be a multiple of 16 so the result lands back in (keys, vals).  hist: radix_hist_words().
inline int radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* ktmp, uint32_t* vtmp,
                            uint32_t* hist, int nseg, int64_t cap, SegCounts counts, int begin_bit,
                            int end_bit, hipStream_t s) {
  const int tiles = (int)cdiv(cap, kSortTile);
  if (nseg == 0 || tiles == 0) return PCST_OK;
  if (256 * tiles > kSmallScanMax) {
    set_error("radix_sort_pairs: segment capacity %lld exceeds %d", (long long)cap,
              kSmallScanMax / 256 * kSortTile);
    return PCST_EUNSUPPORTED;
  }
  uint32_t *ki = keys, *vi = vals, *ko = ktmp, *vo = vtmp;
  for (int sh = begin_bit; sh < end_bit; sh += 8) {
    hipLaunchKernelGGL(radix_hist_kernel, dim3(tiles, nseg), dim3(kSortThreads), 0, s, ki, cap,
                       counts, sh, tiles, hist);
    // tiles past a segment's count hold zero histograms, so the whole table scans as one
    seg_scan_small(hist, nseg, 256 * tiles, (int64_t)256 * tiles, nullptr, s);
    hipLaunchKernelGGL(radix_scatter_kernel, dim3(tiles, nseg), dim3(kSortThreads), 0, s, ki, vi,
                       ko, vo, cap, counts, sh, tiles, hist);
    uint32_t* t = ki; ki = ko; ko = t;
    t = vi; vi = vo; vo = t;
  }
  PCST_LAUNCH_CHECK("radix_sort_pairs");
  return PCST_OK;
}

}  // namespace
}  // namespace pcst
