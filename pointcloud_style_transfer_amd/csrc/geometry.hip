// PointNet++ geometry kernels for gfx950: square_distance, index_points, farthest-point
// sampling, ball query and the fused SetAbstraction group gather.
// Reference: models/pointnet2_encoder.py (citations per kernel).
// All distance arithmetic uses explicit *_rn intrinsics so the reference's CPU rounding
//  is reproduced bit for bit.
#include "common.h"

namespace pcst {

typedef float fps_f2 __attribute__((ext_vector_type(2)));
typedef int fps_i2 __attribute__((ext_vector_type(2)));


// ------------------------------------------------------------------ square_distance
// pointnet2_encoder.py:8-15.  One thread per (b, s, n) output element, n fastest.
__global__ void square_distance_kernel(const float* __restrict__ src, const float* __restrict__ dst,
                                       int64_t S, int64_t N, int64_t total, float* __restrict__ out) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = e % N;
    const int64_t bs = e / N;
    const int64_t b = bs / S;
    const float* a = src + bs * 3;
    const float* q = dst + (b * N + n) * 3;
    float d = fmul(-2.0f, dot3(a[0], a[1], a[2], q[0], q[1], q[2]));
    d = fadd(d, sqnorm3(a[0], a[1], a[2]));
    d = fadd(d, sqnorm3(q[0], q[1], q[2]));
    out[e] = d;
  }
}

// ------------------------------------------------------------------ index_points
// pointnet2_encoder.py:17-28: gather rows with the index clamped to [0, N-1].
__global__ void index_points_kernel(const float* __restrict__ pts, int64_t N, int64_t C,
                                    const int64_t* __restrict__ idx, int64_t K, int64_t total,
                                    float* __restrict__ out) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = e % C;
    const int64_t bk = e / C;
    const int64_t b = bk / K;
    int64_t g = idx[bk];
    g = g < 0 ? 0 : (g > N - 1 ? N - 1 : g);
    out[e] = pts[(b * N + g) * C + c];
  }
}

// ------------------------------------------------------------------ farthest point sampling
// pointnet2_encoder.py:30-45.  One 512-thread workgroup per cloud; each thread keeps PPT
// points and their running min-distance in registers (point n = tid + k*512), so a whole
// 30000-point cloud is register-resident (60 points x 4 floats per lane).  Per iteration:
// per-thread scan in ascending n with strict '>' (lowest index wins ties, Q3), a 64-lane
// butterfly arg-max, one LDS exchange of the 8 wave winners, one barrier.  The winner's
// coordinates are re-read with a wave-uniform (scalar) load.
constexpr int kFpsThreads = 512;
constexpr int kFpsWaves = kFpsThreads / 64;

__device__ __forceinline__ void argmax_merge(float& v, int& i, float ov, int oi) {
  if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
}

template <int PPT>
__global__ __launch_bounds__(kFpsThreads) void fps_reg_kernel(const float* __restrict__ xyz,
                                                              int N, int npoint,
                                                              const int64_t* __restrict__ start,
                                                              int64_t* __restrict__ out) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const float* P = xyz + (int64_t)b * N * 3;
  float px[PPT], py[PPT], pz[PPT], dist[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int n = tid + k * kFpsThreads;
    if (n < N) {
      px[k] = P[n * 3 + 0]; py[k] = P[n * 3 + 1]; pz[k] = P[n * 3 + 2];
      dist[k] = 1e10f;
    } else {
      px[k] = py[k] = pz[k] = 0.0f;
      dist[k] = -1.0f;  // never the arg-max: real distances are >= 0
    }
  }
  __shared__ float s_val[2][kFpsWaves];
  __shared__ int s_idx[2][kFpsWaves];
  int far = (int)start[b];
  int64_t* o = out + (int64_t)b * npoint;
  for (int it = 0; it < npoint; ++it) {
    far = __builtin_amdgcn_readfirstlane(far);
    if (tid == 0) o[it] = far;
    const float cx = P[far * 3 + 0], cy = P[far * 3 + 1], cz = P[far * 3 + 2];
    // two points per instruction: v_pk_add/mul_f32 perform the same IEEE operations per
    // component ((dx*dx + dy*dy) + dz*dz, nothing fused: this file builds with
    // -ffp-contract=off), so the distances are bit-identical to the scalar form
    const fps_f2 c2x = {cx, cx}, c2y = {cy, cy}, c2z = {cz, cz};
#pragma unroll
    for (int k = 0; k + 1 < PPT; k += 2) {
      const fps_f2 dx = fps_f2{px[k], px[k + 1]} - c2x;
      const fps_f2 dy = fps_f2{py[k], py[k + 1]} - c2y;
      const fps_f2 dz = fps_f2{pz[k], pz[k + 1]} - c2z;
      const fps_f2 d = (dx * dx + dy * dy) + dz * dz;
      dist[k] = d.x < dist[k] ? d.x : dist[k];
      dist[k + 1] = d.y < dist[k + 1] ? d.y : dist[k + 1];
    }
    if (PPT & 1) {
      const int k = PPT - 1;
      const float dx = fsub(px[k], cx), dy = fsub(py[k], cy), dz = fsub(pz[k], cz);
      const float d = fadd(fadd(fmul(dx, dx), fmul(dy, dy)), fmul(dz, dz));
      dist[k] = d < dist[k] ? d : dist[k];
    }
    // arg-max: the value by a max chain, then the lowest k holding it (lowest point index)
    float best = dist[0];
#pragma unroll
    for (int k = 1; k < PPT; ++k) best = fmaxf(best, dist[k]);
    int bestk = PPT - 1;
#pragma unroll
    for (int k = PPT - 2; k >= 0; --k) bestk = dist[k] == best ? k : bestk;
    int bi = tid + bestk * kFpsThreads;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const float ov = __shfl_xor(best, off);
      const int oi = __shfl_xor(bi, off);
      argmax_merge(best, bi, ov, oi);
    }
    const int slot = it & 1;
    if (lane == 0) { s_val[slot][wid] = best; s_idx[slot][wid] = bi; }
    __syncthreads();
    float v = s_val[slot][0];
    int i = s_idx[slot][0];
#pragma unroll
    for (int w = 1; w < kFpsWaves; ++w) argmax_merge(v, i, s_val[slot][w], s_idx[slot][w]);
    far = i;
  }
}

// 1024-thread variant (the default for N <= 30720): 16 waves (4 per SIMD) keep up to 30
// points per lane.  The arg-max is carried as one 64-bit key, (distance bits << 32) | ~n:
// non-negative floats order like their bit patterns, and ~n makes the lowest index win ties
// (Q3).  In-row DPP steps + readlane replace the LDS-crossbar shuffles, and one LDS exchange
// of the 16 wave keys per iteration finishes the reduction.
constexpr int kFps2Threads = 1024;
constexpr int kFps2Waves = kFps2Threads / 64;

__device__ __forceinline__ uint64_t u64max(uint64_t a, uint64_t b) { return a > b ? a : b; }

template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)v, CTRL, 0xf, 0xf, false);
  const uint32_t hi = __builtin_amdgcn_update_dpp(0u, (uint32_t)(v >> 32), CTRL, 0xf, 0xf, false);
  return ((uint64_t)hi << 32) | lo;
}

// max over the 16 lanes of each DPP row; every lane of the row ends with the row maximum
__device__ __forceinline__ uint64_t row_max_u64(uint64_t k) {
  k = u64max(k, dpp_u64<0xB1>(k));   // quad_perm [1,0,3,2]
  k = u64max(k, dpp_u64<0x4E>(k));   // quad_perm [2,3,0,1]
  k = u64max(k, dpp_u64<0x141>(k));  // row_half_mirror
  k = u64max(k, dpp_u64<0x140>(k));  // row_mirror
  return k;
}

__device__ __forceinline__ int wave_max_i32(int v) {  // wave-uniform result
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, false));   // quad_perm [2,3,0,1]
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xf, 0xf, false));  // row_half_mirror
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xf, 0xf, false));  // row_mirror
  return max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t k) {
  k = row_max_u64(k);
  uint64_t m = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)k, r * 16);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(k >> 32), r * 16);
    m = u64max(m, ((uint64_t)hi << 32) | lo);
  }
  return m;
}

template <int PPT>
__global__ __launch_bounds__(kFps2Threads) void fps_key_kernel(const float* __restrict__ xyz,
                                                               int N, int npoint,
                                                               const int64_t* __restrict__ start,
                                                               int64_t* __restrict__ out) {
  // points k and k+1 of a lane live in one register pair (fps_f2), so the packed
  // v_pk_add/mul_f32 distance math needs no operand moves
  constexpr int H = (PPT + 1) / 2;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const float* P = xyz + (int64_t)b * N * 3;
  fps_f2 X[H], Y[H], Z[H];
  fps_i2 D[H];
#pragma unroll
  for (int j = 0; j < H; ++j) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int n = tid + (2 * j + e) * kFps2Threads;
      const bool ok = 2 * j + e < PPT && n < N;
      X[j][e] = ok ? P[n * 3 + 0] : 0.0f;
      Y[j][e] = ok ? P[n * 3 + 1] : 0.0f;
      Z[j][e] = ok ? P[n * 3 + 2] : 0.0f;
      D[j][e] = __float_as_int(ok ? 1e10f : -1.0f);  // -1: never updated, never the arg-max
    }
  }
  __shared__ uint64_t s_key[2][kFps2Waves];
  int far = (int)start[b];
  int64_t* o = out + (int64_t)b * npoint;
  for (int it = 0; it < npoint; ++it) {
    far = __builtin_amdgcn_readfirstlane(far);
    if (tid == 0) o[it] = far;
    const float cx = P[far * 3 + 0], cy = P[far * 3 + 1], cz = P[far * 3 + 2];
    // v_pk_add/mul_f32 perform the same IEEE operations per component ((dx*dx + dy*dy) +
    // dz*dz, nothing fused: this file builds with -ffp-contract=off), so the distances are
    // bit-identical to the scalar form.  The running distances are kept as int bit patterns:
    // every value is -1.0 (a padding slot) or >= 0, and on those signed-int order IS float
    // order, so the strict-< update is one v_min_i32 and the arg-max a v_max_i32 chain (the
    // float min/max would add a canonicalising v_max per operand in IEEE mode).
    const fps_f2 c2x = {cx, cx}, c2y = {cy, cy}, c2z = {cz, cz};
#pragma unroll
    for (int j = 0; j < H; ++j) {
      const fps_f2 dx = X[j] - c2x, dy = Y[j] - c2y, dz = Z[j] - c2z;
      const fps_f2 d = (dx * dx + dy * dy) + dz * dz;
      D[j][0] = min(__float_as_int(d[0]), D[j][0]);
      D[j][1] = min(__float_as_int(d[1]), D[j][1]);
    }
    // arg-max: the value by a max chain, then the lowest k holding it (lowest point index)
    int best = D[0][0];
#pragma unroll
    for (int k = 1; k < 2 * H; ++k) best = max(best, D[k >> 1][k & 1]);
    int bestk = 2 * H - 1;
#pragma unroll
    for (int k = 2 * H - 2; k >= 0; --k) bestk = D[k >> 1][k & 1] == best ? k : bestk;
    const uint32_t n = (uint32_t)(tid + bestk * kFps2Threads);
    const uint32_t bits = best > 0 ? (uint32_t)best : 0u;
    const uint64_t key = wave_max_u64(((uint64_t)bits << 32) | (0xFFFFFFFFu - n));
    const int slot = it & 1;
    if (lane == 0) s_key[slot][wid] = key;
    __syncthreads();
    uint64_t g = lane < kFps2Waves ? s_key[slot][lane] : 0ull;
    g = row_max_u64(g);
    const uint32_t glo = __builtin_amdgcn_readlane((uint32_t)g, 0);
    far = (int)(0xFFFFFFFFu - glo);
  }
}

// Spatially culled FPS (the default for 8192 < N <= 30720).  Same arithmetic, keys and
// result as fps_key_kernel; the points are laid out so that a round can skip most waves.
//   Layout: the cloud is cut into 16 regions, one per wave: contiguous runs of a 14-bit Morton
//   order of the points (5/5/4 bits over the cloud's bounding box), filled greedily up to a
//   wave's 64*R register slots (R = min(PPT, 28): registers hold point pairs, and 15 pairs per
//   lane would not leave the loop its temporaries in 128 VGPRs); the points past 16 full
//   regions (at most 4096) form an overflow set kept in LDS (in the histogram's space), four
//   per lane of the first waves, updated every round.  Inside a
//   region the points keep ascending index order (a stable counting sort by region), so slot s
//   of wave w is lane s % 64, register k = s / 64, and a lane's registers hold ascending
//   indices: the lowest k holding the lane's maximum is still its lowest index (Q3).  perm[]
//   (LDS, 16-bit) maps a slot back to the point index.
//   Culling: a wave whose bounding box is at least its current maximum distance away from the
//   new centroid cannot change any running minimum (fl() is monotone, so the box distance
//   computed with the points' own operation sequence bounds every point's computed distance
//   from below) and keeps last round's key, (distance bits << 32) | ~index.  If the greedy fill
//   leaves more than 4096 points over (a degenerate cloud), the regions are plain index ranges:
//   the same result, little culling.
constexpr int kCullBins = 16384;
constexpr int kCullRegions = kFps2Waves;  // + 1: the overflow set
constexpr int kCullOver = 4096;           // overflow capacity (the histogram's LDS)

__device__ __forceinline__ uint32_t spread3(uint32_t v) {  // 5 bits -> every third bit
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < 5; ++b) r |= ((v >> b) & 1u) << (3 * b);
  return r;
}

__device__ __forceinline__ float wave_minf(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fminf(v, __shfl_xor(v, off));
  return v;
}
__device__ __forceinline__ float wave_maxf(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
  return v;
}
__device__ __forceinline__ float uni(float v) {  // a wave-uniform value into an SGPR
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

template <int PPT>
__global__ __launch_bounds__(kFps2Threads) void fps_cull_kernel(const float* __restrict__ xyz,
                                                                int N, int npoint,
                                                                const int64_t* __restrict__ start,
                                                                int64_t* __restrict__ out) {
  constexpr int R = PPT < 28 ? PPT : 28;  // register slots per lane (an even count)
  constexpr int H = (R + 1) / 2;
  constexpr int W = kFps2Waves;
  constexpr int G = kCullRegions + 1;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const float* P = xyz + (int64_t)b * N * 3;
  __shared__ uint16_t perm[kFps2Threads * PPT];
  __shared__ __attribute__((aligned(16))) uint32_t hist[kCullBins];
  // after the layout is built the histogram's space holds the overflow points: x, y, z, and
  // the running distance bits
  float4* s_over = reinterpret_cast<float4*>(hist);
  static_assert(kCullOver * 16 <= kCullBins * 4, "overflow set must fit the histogram's space");
  __shared__ float s_red[W][6];
  __shared__ int s_rs[G + 1];
  __shared__ int s_cur[G];
  __shared__ int s_cnt[2][W][G];  // [buffer][wave][region]
  __shared__ int s_ok;
  __shared__ uint64_t s_key[2][W];

  // ---- bounding box and Morton bins of the points in index order (n = tid + 1024 k)
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
#pragma unroll 2
  for (int k = 0; k < PPT; ++k) {
    const int n = tid + k * kFps2Threads;
    if (n < N) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float v = P[n * 3 + c];
        mn[c] = fminf(mn[c], v);
        mx[c] = fmaxf(mx[c], v);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    mn[c] = wave_minf(mn[c]);
    mx[c] = wave_maxf(mx[c]);
    if (lane == 0) { s_red[wid][c] = mn[c]; s_red[wid][3 + c] = mx[c]; }
  }
  for (int i = tid; i < kCullBins; i += kFps2Threads) hist[i] = 0;
  __syncthreads();
  float lo[3], sc[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float a = s_red[0][c], z = s_red[0][3 + c];
    for (int w = 1; w < W; ++w) { a = fminf(a, s_red[w][c]); z = fmaxf(z, s_red[w][3 + c]); }
    lo[c] = a;
    const float ext = z - a;
    sc[c] = ext > 0.0f ? (c == 2 ? 16.0f : 32.0f) / ext : 0.0f;
  }
  // 14-bit Morton bin: x and y 5 bits, z 4
  auto bin_of = [&](int n) {
    const uint32_t qx = min((uint32_t)((P[n * 3 + 0] - lo[0]) * sc[0]), 31u);
    const uint32_t qy = min((uint32_t)((P[n * 3 + 1] - lo[1]) * sc[1]), 31u);
    const uint32_t qz = min((uint32_t)((P[n * 3 + 2] - lo[2]) * sc[2]), 15u);
    return (spread3(qx) | (spread3(qy) << 1) | (spread3(qz) << 2)) & (uint32_t)(kCullBins - 1);
  };
#pragma unroll 2
  for (int k = 0; k < PPT; ++k) {
    const int n = tid + k * kFps2Threads;
    if (n < N) atomicAdd(&hist[bin_of(n)], 1u);
  }
  __syncthreads();
  // ---- exclusive scan of the histogram (16 bins per thread)
  {
    uint32_t v[16], sum = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) { v[i] = hist[tid * 16 + i]; sum += v[i]; }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    if (lane == 63) s_cnt[0][0][wid] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int w = 0; w < wid; ++w) base += s_cnt[0][0][w];
    uint32_t run = base + incl - sum;
#pragma unroll
    for (int i = 0; i < 16; ++i) { hist[tid * 16 + i] = run; run += v[i]; }
  }
  __syncthreads();
  // ---- region boundaries (wave 0): region r = bins [e_r, e_{r+1}), greedy up to 64*R points;
  // the overflow set is everything after region 15
  const uint32_t cap = 64u * R;
  if (wid == 0) {
    uint32_t e = 0;  // bin where the current region starts
    for (int r = 0; r < kCullRegions; ++r) {
      const uint32_t s0 = e >= kCullBins ? (uint32_t)N : hist[e];
      // last bin boundary f in [e, kCullBins] with start(f) - s0 <= cap (start(kCullBins) = N)
      uint32_t lo_b = e, hi_b = kCullBins;
      while (hi_b > lo_b) {
        const uint32_t span = hi_b - lo_b;
        const uint32_t f = lo_b + (uint32_t)(((uint64_t)span * (lane + 1) + 63) / 64);
        const uint32_t sf = f >= kCullBins ? (uint32_t)N : hist[f];
        const uint64_t fits = __ballot(sf - s0 <= cap);  // a prefix of the lanes (monotone)
        const int last = fits ? 63 - __builtin_clzll(fits) : -1;
        const uint32_t flast = last < 0 ? lo_b : lo_b + (uint32_t)(((uint64_t)span * (last + 1) + 63) / 64);
        const uint32_t fnext = lo_b + (uint32_t)(((uint64_t)span * (last + 2) + 63) / 64);
        lo_b = flast;
        hi_b = last == 63 ? flast : (fnext > lo_b ? fnext - 1 : lo_b);
      }
      if (lane == 0) s_rs[r] = (int)s0;
      e = lo_b;
    }
    const uint32_t s16 = e >= kCullBins ? (uint32_t)N : hist[e];
    if (lane == 0) {
      const bool ok = (uint32_t)N - s16 <= (uint32_t)kCullOver;
      s_ok = ok;
      s_rs[kCullRegions] = ok ? (int)s16 : (int)min((uint32_t)N, cap * kCullRegions);
      s_rs[G] = N;
      if (!ok)  // plain index ranges
        for (int r = 0; r < kCullRegions; ++r) s_rs[r] = (int)min((uint32_t)N, cap * r);
    }
  }
  if (tid < G) s_cur[tid] = 0;
  __syncthreads();
  const bool morton = s_ok != 0;
  // ---- stable counting sort by region, chunk k = the points tid + 1024 k (ascending index)
#pragma unroll 1
  for (int k = 0; k < PPT; ++k) {
    const int n = tid + k * kFps2Threads;
    int reg = -1;
    if (n < N) {
      if (morton) {
        const uint32_t pos = hist[bin_of(n)];  // region of the bin: its start's region
        reg = 0;
#pragma unroll
        for (int r = 1; r < G; ++r) reg += pos >= (uint32_t)s_rs[r] ? 1 : 0;
      } else {
        reg = min(n / (int)cap, kCullRegions);
      }
    }
    uint64_t mine = 0;
    int cnt_lane = 0;
#pragma unroll
    for (int r = 0; r < G; ++r) {
      const uint64_t m = __ballot(reg == r);
      if (reg == r) mine = m;
      if (lane == r) cnt_lane = __popcll(m);
    }
    const int buf = k & 1;
    if (lane < G) s_cnt[buf][wid][lane] = cnt_lane;
    __syncthreads();
    if (reg >= 0) {
      int pre = s_cur[reg];
      for (int w = 0; w < wid; ++w) pre += s_cnt[buf][w][reg];
      perm[s_rs[reg] + pre + __popcll(mine & lanemask_lt())] = (uint16_t)n;
    }
    __syncthreads();
    if (tid < G) {
      int t = 0;
      for (int w = 0; w < W; ++w) t += s_cnt[buf][w][tid];
      s_cur[tid] += t;
    }
  }
  __syncthreads();
  // ---- overflow points into LDS (slot i: wave i >> 8, lane i & 63, m = (i >> 6) & 3), this
  // wave's region into registers (pairs k, k+1)
  const int o0 = __builtin_amdgcn_readfirstlane(s_rs[kCullRegions]);
  const int nover = N - o0;
  for (int i = tid; i < nover; i += kFps2Threads) {
    const int n = perm[o0 + i];
    s_over[i] = make_float4(P[n * 3 + 0], P[n * 3 + 1], P[n * 3 + 2], 1e10f);
  }
  const int r0 = __builtin_amdgcn_readfirstlane(s_rs[wid]);
  const int r1 = __builtin_amdgcn_readfirstlane(s_rs[wid + 1]);
  fps_f2 X[H], Y[H], Z[H];
  fps_i2 D[H];
#pragma unroll
  for (int j = 0; j < H; ++j) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int p = r0 + (2 * j + e) * 64 + lane;
      const bool ok = 2 * j + e < R && p < r1;
      const int n = ok ? (int)perm[p] : 0;
      X[j][e] = ok ? P[n * 3 + 0] : 0.0f;
      Y[j][e] = ok ? P[n * 3 + 1] : 0.0f;
      Z[j][e] = ok ? P[n * 3 + 2] : 0.0f;
      D[j][e] = __float_as_int(ok ? 1e10f : -1.0f);
    }
  }
  // the wave's bounding box (uniform)
  float bmn[3], bmx[3];
  {
    float a0 = INFINITY, a1 = INFINITY, a2 = INFINITY, z0 = -INFINITY, z1 = -INFINITY, z2 = -INFINITY;
#pragma unroll
    for (int j = 0; j < H; ++j)
#pragma unroll
      for (int e = 0; e < 2; ++e)
        if (D[j][e] >= 0) {
          a0 = fminf(a0, X[j][e]); z0 = fmaxf(z0, X[j][e]);
          a1 = fminf(a1, Y[j][e]); z1 = fmaxf(z1, Y[j][e]);
          a2 = fminf(a2, Z[j][e]); z2 = fmaxf(z2, Z[j][e]);
        }
    bmn[0] = uni(wave_minf(a0)); bmn[1] = uni(wave_minf(a1)); bmn[2] = uni(wave_minf(a2));
    bmx[0] = uni(wave_maxf(z0)); bmx[1] = uni(wave_maxf(z1)); bmx[2] = uni(wave_maxf(z2));
  }
  const bool has_over = wid * 256 < nover;  // this wave carries overflow points (uniform)
  // cached region state: key and maximum distance (-1: no point)
  uint64_t rkey = 0;
  float rmax = r1 > r0 ? 1e10f : -1.0f;
  int far = (int)start[b];
  int64_t* o = out + (int64_t)b * npoint;
  __syncthreads();
  for (int it = 0; it < npoint; ++it) {
    if (tid == 0) o[it] = far;
    const float cx = uni(P[far * 3 + 0]), cy = uni(P[far * 3 + 1]), cz = uni(P[far * 3 + 2]);
    // box distance with the points' own operation sequence (a lower bound of every point's)
    const float ex = cx < bmn[0] ? fsub(bmn[0], cx) : (cx > bmx[0] ? fsub(cx, bmx[0]) : 0.0f);
    const float ey = cy < bmn[1] ? fsub(bmn[1], cy) : (cy > bmx[1] ? fsub(cy, bmx[1]) : 0.0f);
    const float ez = cz < bmn[2] ? fsub(bmn[2], cz) : (cz > bmx[2] ? fsub(cz, bmx[2]) : 0.0f);
    const float lb = fadd(fadd(fmul(ex, ex), fmul(ey, ey)), fmul(ez, ez));
    if (!(lb >= rmax)) {  // wave-uniform
      const fps_f2 c2x = {cx, cx}, c2y = {cy, cy}, c2z = {cz, cz};
#pragma unroll
      for (int j = 0; j < H; ++j) {
        const fps_f2 dx = X[j] - c2x, dy = Y[j] - c2y, dz = Z[j] - c2z;
        const fps_f2 d = (dx * dx + dy * dy) + dz * dz;
        D[j][0] = min(__float_as_int(d[0]), D[j][0]);
        D[j][1] = min(__float_as_int(d[1]), D[j][1]);
      }
      // the wave's maximum distance m (32-bit), then its lowest slot s = 64 k + lane holding m:
      // slots are in ascending point index inside a region, so that is the lowest index (Q3)
      int best = D[0][0];
#pragma unroll
      for (int k = 1; k < 2 * H; ++k) best = max(best, D[k >> 1][k & 1]);
      const int m = wave_max_i32(best);  // >= 0: the region has a point (else it is culled)
      int ks = 2 * H - 1;
      uint64_t lanes = 0;
#pragma unroll
      for (int k = 0; k < 2 * H; ++k) {
        const uint64_t hit = __ballot(D[k >> 1][k & 1] == m);
        if (hit) { ks = k; lanes = hit; break; }
      }
      const uint32_t n = perm[r0 + ks * 64 + (__builtin_ffsll((long long)lanes) - 1)];
      rkey = ((uint64_t)(uint32_t)m << 32) | (0xFFFFFFFFu - n);
      rmax = __int_as_float(m);
    }
    uint64_t wkey = rkey;
    if (has_over) {  // the overflow points of this wave: every round
      uint64_t key = 0;
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int i = wid * 256 + m * 64 + lane;
        if (i < nover) {
          const float4 q = s_over[i];
          const float dx = fsub(q.x, cx), dy = fsub(q.y, cy), dz = fsub(q.z, cz);
          const float d = fadd(fadd(fmul(dx, dx), fmul(dy, dy)), fmul(dz, dz));
          const int dd = min(__float_as_int(d), __float_as_int(q.w));
          s_over[i].w = __int_as_float(dd);
          key = u64max(key, ((uint64_t)(uint32_t)dd << 32) | (0xFFFFFFFFu - (uint32_t)perm[o0 + i]));
        }
      }
      wkey = u64max(wkey, wave_max_u64(key));
    }
    const int slot = it & 1;
    if (lane == 0) s_key[slot][wid] = wkey;
    __syncthreads();
    uint64_t g = lane < W ? s_key[slot][lane] : 0ull;
    g = row_max_u64(g);
    const uint32_t glo = __builtin_amdgcn_readlane((uint32_t)g, 0);
    far = (int)(0xFFFFFFFFu - glo);
  }
}

// Multi-CU FPS (pcst_fps_ws with a workspace, 8192 < N <= 32768, B * K <= kFpsXMaxGroups = 32):
// the same keys and result as fps_key_kernel with the cloud cut over K = ceil(N / 1024)
// work-groups of 512 threads (2 points per lane: a round's distance update is ~30 VALU
// instructions per wave instead of a culled 30-point region's ~250), which exchange their round
// winners through global memory instead of one CU running every point.
//   Round: every lane updates its points and keeps its best key with the point's coordinates; the
//   wave maximum (DPP), one LDS exchange of the 8 wave winners and a barrier give the work-group's
//   winner, which wave 0 publishes to its slot: ONE 64-bit word, (round + 1) << 48 | index << 32 |
//   distance bits, single-copy atomic, so the tag validates the whole word and no fence orders
//   anything.  Wave 0 then polls the cloud's K slots (lane j: slot j, agent-scope relaxed loads
//   that bypass L1); a lane whose slot is ready loads that candidate's coordinates from the
//   (read-only) cloud at once, so they are in flight while the other slots arrive; the maximum key
//   and its coordinates reach the other waves through LDS and a second barrier.  Two slot sets
//   alternate by round parity: a work-group overwrites its parity-p slot (round r + 2) only after
//   it read every slot of round r + 1, each published after ITS work-group's barrier of round r + 1,
//   which all its waves reached only after they were done with round r.  The workspace is zeroed
//   per call by a kernel ahead of it on the stream (tags >= 1).
//   Same-XCD mode: the work-groups first exchange their XCC ids (agent scope, once); if all K share
//   one XCD -- checked, never assumed -- slots are published with plain stores, which keep the line
//   in that L2 where the siblings' L1-bypassing polls hit it; otherwise with agent-scope stores,
//   which write through and drop the line (a fabric round trip per round).  The launch has 8
//   work-groups per working one and only those with blockIdx % 8 == 0 work, which round-robin
//   dispatch puts on one XCD (speed only).
//   Forward progress: a polling work-group needs its K - 1 siblings to run; at most kFpsXMaxGroups
//   work-groups work, far below the device's resident capacity, and everything else on the device
//   is finite, so every sibling gets a CU.  A poll that exceeds max_polls (a broken sibling) marks
//   the work-group dead: it stops publishing and waiting, its siblings give up in turn, and the
//   cloud's samples are written as -1 instead of hanging.
//   Measured (tools/fps_ab.py, B = 1, N = 30000, 512 samples): 1.48 us per round at 2 points per
//   lane (K = 30) and 1.60 at 4 (K = 15), against the culled kernel's 1.96-2.10; polling by every
//   wave (3.0-3.6 with five-word slots carrying the coordinates, 2.1-2.5 with one-word slots) lost
//   to L2 contention on the slot lines, and so did every wave publishing its own winner (no first
//   barrier, wave 0 polling K x 8 words: 2.65).
constexpr int kFpsXThreads = 512;
constexpr int kFpsXWaves = kFpsXThreads / 64;
#ifndef PCST_FPSX_PPT  // experiment builds (csrc/Makefile XDEF)
#define PCST_FPSX_PPT 2
#endif
constexpr int kFpsXPPT = PCST_FPSX_PPT;
constexpr int kFpsXMaxGroups = 32;
constexpr int kFpsXWords = 8;  // 5 tagged words per slot, padded to 64 B

__device__ __forceinline__ void fpsx_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t fpsx_load(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xfu;
}

// the slots zeroed before the FPS launch (a kernel, not hipMemsetAsync: the host then never waits
// here and keeps queueing while the previous call's FPS runs)
__global__ __launch_bounds__(256) void fpsx_zero_kernel(uint64_t* __restrict__ w, int64_t words) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < words; i += (int64_t)gridDim.x * 256)
    w[i] = 0ull;
}

__global__ __launch_bounds__(kFpsXThreads) void fps_multi_kernel(const float* __restrict__ xyz,
                                                                 int N, int npoint,
                                                                 const int64_t* __restrict__ start,
                                                                 int64_t* __restrict__ out,
                                                                 uint64_t* __restrict__ slots,
                                                                 int K, int64_t max_polls) {
  if (blockIdx.x & 7) return;  // (placement only: the working work-groups share an XCD)
  constexpr int H = kFpsXPPT / 2;
  const int gi = blockIdx.x >> 3;
  const int b = gi / K, k = gi - b * K;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const float* P = xyz + (int64_t)b * N * 3;
  const int base = k * (kFpsXThreads * kFpsXPPT);
  fps_f2 X[H], Y[H], Z[H];
  fps_i2 D[H];
#pragma unroll
  for (int j = 0; j < H; ++j) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int n = base + tid + (2 * j + e) * kFpsXThreads;
      const bool ok = n < N;
      X[j][e] = ok ? P[n * 3 + 0] : 0.0f;
      Y[j][e] = ok ? P[n * 3 + 1] : 0.0f;
      Z[j][e] = ok ? P[n * 3 + 2] : 0.0f;
      D[j][e] = __float_as_int(ok ? 1e10f : -1.0f);  // -1: a padding slot, never the arg-max
    }
  }
  __shared__ uint64_t s_key[2][kFpsXWaves];
  __shared__ float4 s_pt[2][kFpsXWaves];
  __shared__ int s_dead;
  __shared__ int s_far[2];
  __shared__ float4 s_c[2];
  if (tid == 0) s_dead = 0;
  __syncthreads();
  uint64_t* S = slots + (int64_t)b * K * 2 * kFpsXWords;  // [parity][k][word]
  int far = (int)start[b];
  float cx = P[far * 3 + 0], cy = P[far * 3 + 1], cz = P[far * 3 + 2];
  int64_t* o = out + (int64_t)b * npoint;
  bool dead = false;
  // Same-XCD mode: the work-groups exchange their XCC ids once (word 5 of the parity-1 slots,
  // tag 0xFFFFFFFF, agent scope; a parity-1 slot is first rewritten in round 1, after every
  // work-group published round 0, i.e. after it read the ids).  If all K share one XCD -- checked,
  // never assumed -- the rounds'
  // slots are published with plain stores, which keep the line in that XCD's L2, where the other
  // work-groups' L1-bypassing (sc1) polls find it; otherwise with agent-scope stores, which drop
  // the line from L2 for readers on other XCDs (a fabric round trip per round).  Every work-group
  // reads the same K ids, so all take the same mode.
  bool local = false;
  if (K > 1) {
    if (tid == 0) fpsx_store(S + (int64_t)(K + k) * kFpsXWords + 5, (0xFFFFFFFFull << 32) | xcc_id());
    uint64_t v = 0;
    for (int64_t poll = 0;; ++poll) {
      if (lane < K) v = fpsx_load(S + (int64_t)(K + lane) * kFpsXWords + 5);
      if (__ballot(lane < K && (v >> 32) != 0xFFFFFFFFull) == 0ull) break;
      if (poll >= max_polls) { dead = true; break; }
    }
    const uint32_t x0 = __builtin_amdgcn_readlane((uint32_t)v, 0);
    local = !dead && __ballot(lane < K && (uint32_t)v != x0) == 0ull;
    if (dead && lane == 0) s_dead = 1;
  }
  for (int it = 0; it < npoint; ++it) {
    if (k == 0 && tid == 0) o[it] = far;
    const fps_f2 c2x = {cx, cx}, c2y = {cy, cy}, c2z = {cz, cz};
    uint64_t lk = 0;  // padding slots keep key 0, below every point's key
    float bx = 0.0f, by = 0.0f, bz = 0.0f;
#pragma unroll
    for (int j = 0; j < H; ++j) {
      // the same IEEE operations as fps_key_kernel ((dx*dx + dy*dy) + dz*dz, nothing fused)
      const fps_f2 dx = X[j] - c2x, dy = Y[j] - c2y, dz = Z[j] - c2z;
      const fps_f2 d = (dx * dx + dy * dy) + dz * dz;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        D[j][e] = min(__float_as_int(d[e]), D[j][e]);
        const uint32_t n = (uint32_t)(base + tid + (2 * j + e) * kFpsXThreads);
        const uint64_t key = D[j][e] >= 0 ? ((uint64_t)(uint32_t)D[j][e] << 32) | (0xFFFFFFFFu - n) : 0ull;
        if (key > lk) { lk = key; bx = X[j][e]; by = Y[j][e]; bz = Z[j][e]; }
      }
    }
    // the wave's winner (key and coordinates), then the work-group's through LDS
    const uint64_t wk = wave_max_u64(lk);
    const uint64_t wl = __ballot(lk == wk);
    const int wlane = __builtin_ffsll((long long)wl) - 1;
    const float wx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bx), wlane));
    const float wy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(by), wlane));
    const float wz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bz), wlane));
    const int slot = it & 1;
    if (lane == 0) {
      s_key[slot][wid] = wk;
      s_pt[slot][wid] = make_float4(wx, wy, wz, 0.0f);
    }
    __syncthreads();
    if (s_dead) dead = true;  // a wave of this work-group gave up in an earlier round
    uint64_t g = lane < kFpsXWaves ? s_key[slot][lane] : 0ull;
    g = row_max_u64(g);
    const uint32_t gk_hi = __builtin_amdgcn_readlane((uint32_t)(g >> 32), 0);  // (readlane's
    const uint32_t gk_lo = __builtin_amdgcn_readlane((uint32_t)g, 0);          // int: no sign-extension)
    const uint64_t gk = ((uint64_t)gk_hi << 32) | gk_lo;
    if (K == 1) {  // the winning wave's coordinates (a full-wave ballot over the LDS keys)
      const int gw = __builtin_ffsll((long long)__ballot(lane < kFpsXWaves && s_key[slot][lane & 7] == gk)) - 1;
      const float4 q = s_pt[slot][gw];
      far = (int)(0xFFFFFFFFu - (uint32_t)gk);
      cx = q.x; cy = q.y; cz = q.z;
      continue;
    }
    uint64_t* mine = S + ((int64_t)slot * K + k) * kFpsXWords;
    // one word per slot: tag (16 bits) | index (16) | distance bits (32)
    const uint64_t tag16 = (uint64_t)(uint32_t)(it + 1) << 48;
    if (wid == 0 && lane == 0 && !dead) {
      const uint64_t w = tag16 | ((uint64_t)(0xFFFFFFFFu - (uint32_t)gk) << 32) | (gk >> 32);
      if (local) *reinterpret_cast<volatile uint64_t*>(mine) = w;
      else fpsx_store(mine, w);
    }
    // wave 0 polls the K slots; a lane whose slot is ready loads that candidate's coordinates at
    // once (read-only cloud), so they are in flight while the other slots arrive; then the
    // winner's index and coordinates go to the other waves through LDS (one more barrier)
    if (wid == 0) {
      const uint64_t* sj = S + ((int64_t)slot * K + (lane < K ? lane : 0)) * kFpsXWords;
      uint64_t w0 = 0;
      bool have = lane >= K;
      float px = 0.0f, py = 0.0f, pz = 0.0f;
      for (int64_t poll = 0;; ++poll) {
        if (!have) {
          w0 = fpsx_load(sj);
          if ((w0 >> 48) == (uint64_t)(uint32_t)(it + 1) || dead) {
            const int j = min((int)((w0 >> 32) & 0xFFFFu), N - 1);
            px = P[j * 3 + 0]; py = P[j * 3 + 1]; pz = P[j * 3 + 2];
            have = true;
          }
        }
        if (__ballot(!have) == 0ull) break;
        if (poll >= max_polls) {
          dead = true;
          if (lane == 0) s_dead = 1;
          break;
        }
      }
      const uint64_t key = lane < K ? ((w0 & 0xFFFFFFFFull) << 32) |
                                          (0xFFFFFFFFu - (uint32_t)((w0 >> 32) & 0xFFFFu))
                                    : 0ull;
      const uint64_t kmax = wave_max_u64(key);
      const int wj = __builtin_ffsll((long long)__ballot(lane < K && key == kmax)) - 1;
      const float ex = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(px), wj));
      const float ey = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(py), wj));
      const float ez = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pz), wj));
      if (lane == 0) {
        s_far[slot] = dead ? -1 : (int)(0xFFFFFFFFu - (uint32_t)kmax);
        s_c[slot] = make_float4(ex, ey, ez, 0.0f);
      }
    }
    __syncthreads();
    far = s_far[slot];
    if (far < 0) dead = true;
    far = dead ? 0 : far;
    const float4 c = s_c[slot];
    cx = c.x; cy = c.y; cz = c.z;
  }
  // a wave whose poll gave up (a sibling that never published): it stopped waiting and its
  // work-group stopped publishing, so every work-group of the cloud gives up in turn; the cloud's
  // samples are then -1 (no hang, no plausible-looking indices)
  __syncthreads();
  if (s_dead && k == 0)
    for (int i = tid; i < npoint; i += kFpsXThreads) o[i] = -1;
}

// Fallback for N > 512*60: running distances in global memory (caller workspace), one
// workgroup per cloud streaming the cloud every iteration.
__global__ __launch_bounds__(1024) void fps_global_kernel(const float* __restrict__ xyz, int N,
                                                          int npoint,
                                                          const int64_t* __restrict__ start,
                                                          float* __restrict__ distbuf,
                                                          int64_t* __restrict__ out) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* P = xyz + (int64_t)b * N * 3;
  float* D = distbuf + (int64_t)b * N;
  for (int n = tid; n < N; n += 1024) D[n] = 1e10f;
  __shared__ float s_val[2][16];
  __shared__ int s_idx[2][16];
  int far = (int)start[b];
  for (int it = 0; it < npoint; ++it) {
    far = __builtin_amdgcn_readfirstlane(far);
    if (tid == 0) out[(int64_t)b * npoint + it] = far;
    const float cx = P[far * 3 + 0], cy = P[far * 3 + 1], cz = P[far * 3 + 2];
    float best = -2.0f;
    int bi = 0;
    for (int n = tid; n < N; n += 1024) {
      const float dx = fsub(P[n * 3 + 0], cx), dy = fsub(P[n * 3 + 1], cy),
                  dz = fsub(P[n * 3 + 2], cz);
      const float d = fadd(fadd(fmul(dx, dx), fmul(dy, dy)), fmul(dz, dz));
      float cur = D[n];
      if (d < cur) { cur = d; D[n] = d; }
      if (cur > best) { best = cur; bi = n; }
    }
    for (int off = 32; off >= 1; off >>= 1) {
      const float ov = __shfl_xor(best, off);
      const int oi = __shfl_xor(bi, off);
      argmax_merge(best, bi, ov, oi);
    }
    const int slot = it & 1;
    if (lane == 0) { s_val[slot][wid] = best; s_idx[slot][wid] = bi; }
    __syncthreads();
    float v = s_val[slot][0];
    int i = s_idx[slot][0];
    for (int w = 1; w < 16; ++w) argmax_merge(v, i, s_val[slot][w], s_idx[slot][w]);
    far = i;
  }
}

// ------------------------------------------------------------------ ball query
// pointnet2_encoder.py:47-59.  One wave per centroid scans the cloud in ascending index
// order, 64 points per step (4 steps in flight), keeps the in-radius points with a ballot +
// prefix popcount (exactly the first `nsample` in index order, as the reference's full sort
// does) and exits as soon as nsample are found.
__global__ __launch_bounds__(256) void ball_query_kernel(float r2, int nsample,
                                                         const float* __restrict__ xyz,
                                                         const float* __restrict__ new_xyz,
                                                         int B, int N, int S,
                                                         int64_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= (int64_t)B * S) return;
  const int b = (int)(q / S);
  const float* a = new_xyz + q * 3;
  const float a0 = a[0], a1 = a[1], a2 = a[2];
  const float na = sqnorm3(a0, a1, a2);
  const float* P = xyz + (int64_t)b * N * 3;
  int64_t* o = out + q * nsample;
  int cnt = 0;
  int first = N;
  for (int base = 0; base < N && cnt < nsample; base += 256) {
    float d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int n = base + u * 64 + lane;
      d[u] = 3.4e38f;
      if (n < N) {
        const float q0 = P[n * 3 + 0], q1 = P[n * 3 + 1], q2 = P[n * 3 + 2];
        float dd = fmul(-2.0f, dot3(a0, a1, a2, q0, q1, q2));
        dd = fadd(dd, na);
        d[u] = fadd(dd, sqnorm3(q0, q1, q2));
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int n = base + u * 64 + lane;
      const bool in = (n < N) && !(d[u] > r2);
      const unsigned long long m = __ballot(in);
      if (m == 0ull) continue;
      if (cnt == 0) first = base + u * 64 + (__ffsll((long long)m) - 1);
      const int slot = cnt + __popcll(m & lanemask_lt());
      if (in && slot < nsample) o[slot] = n;
      cnt += __popcll(m);
      if (cnt >= nsample) break;
    }
  }
  for (int k = (cnt < nsample ? cnt : nsample) + lane; k < nsample; k += 64) o[k] = first;
}

// Split-range variant (the default): one workgroup of kBqWaves waves per centroid; wave w
// scans its contiguous slice of [0, N) in ascending order and keeps the first nsample hits of
// the slice (early exit).  The result -- the first nsample hits of [0, N) -- is the
// concatenation of the slices' lists in slice order, so it is identical to the sequential
// scan.  The cloud is re-read per centroid from L2 (360 KB at N = 30000).
constexpr int kBqWaves = 8;

__global__ __launch_bounds__(kBqWaves * 64) void ball_query_split_kernel(
    float r2, int nsample, const float* __restrict__ xyz, const float* __restrict__ new_xyz,
    int N, int S, int64_t* __restrict__ out) {
  extern __shared__ int bq_smem[];
  int* s_cnt = bq_smem;              // [kBqWaves]
  int* s_list = bq_smem + kBqWaves;  // [kBqWaves][nsample]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t q = blockIdx.x;
  const int b = (int)(q / S);
  const float a0 = new_xyz[q * 3 + 0], a1 = new_xyz[q * 3 + 1], a2 = new_xyz[q * 3 + 2];
  const float na = sqnorm3(a0, a1, a2);
  const float* P = xyz + (int64_t)b * N * 3;
  const int per = (int)((((int64_t)N + kBqWaves - 1) / kBqWaves + 63) / 64 * 64);
  const int lo = w * per, hi = min(N, lo + per);
  int* my = s_list + w * nsample;
  int cnt = 0;
  for (int base = lo; base < hi && cnt < nsample; base += 256) {
    float d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int n = base + u * 64 + lane;
      d[u] = 3.4e38f;
      if (n < hi) {
        const float q0 = P[n * 3 + 0], q1 = P[n * 3 + 1], q2 = P[n * 3 + 2];
        float dd = fmul(-2.0f, dot3(a0, a1, a2, q0, q1, q2));
        dd = fadd(dd, na);
        d[u] = fadd(dd, sqnorm3(q0, q1, q2));
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int n = base + u * 64 + lane;
      const bool in = (n < hi) && !(d[u] > r2);
      const unsigned long long m = __ballot(in);
      if (m == 0ull) continue;
      const int slot = cnt + __popcll(m & lanemask_lt());
      if (in && slot < nsample) my[slot] = n;
      cnt += __popcll(m);
      if (cnt >= nsample) break;
    }
  }
  if (lane == 0) s_cnt[w] = min(cnt, nsample);
  __syncthreads();
  int64_t* o = out + q * nsample;
  int total = 0, first = N;
  for (int v = 0; v < kBqWaves; ++v) {
    if (first == N && s_cnt[v] > 0) first = s_list[v * nsample];
    total += s_cnt[v];
  }
  for (int k = threadIdx.x; k < nsample; k += kBqWaves * 64) {
    int val = first;
    if (k < total) {
      int v = 0, pre = 0;
      while (k >= pre + s_cnt[v]) pre += s_cnt[v++];
      val = s_list[v * nsample + (k - pre)];
    }
    o[k] = val;
  }
}

// ------------------------------------------------------------------ group gather
// pointnet2_encoder.py:92-99: new_xyz = index_points(xyz, fps_idx); grouped =
// cat(index_points(xyz, gidx) - new_xyz, index_points(feats, gidx)).
__global__ void new_xyz_kernel(const float* __restrict__ xyz, int64_t N,
                               const int64_t* __restrict__ fps_idx, int64_t S, int64_t total,
                               float* __restrict__ new_xyz) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = e % 3, bs = e / 3, b = bs / S;
    int64_t g = fps_idx[bs];
    g = g < 0 ? 0 : (g > N - 1 ? N - 1 : g);
    new_xyz[e] = xyz[(b * N + g) * 3 + c];
  }
}

__global__ void group_gather_kernel(const float* __restrict__ xyz, const float* __restrict__ feats,
                                    int64_t N, int64_t C, const float* __restrict__ new_xyz,
                                    const int64_t* __restrict__ gidx, int64_t S, int64_t ns,
                                    int64_t total, float* __restrict__ grouped) {
  const int64_t W = 3 + C;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = e % W, r = e / W;  // r = (b*S + s)*ns + k
    const int64_t bs = r / ns, b = bs / S;
    int64_t g = gidx[r];
    g = g < 0 ? 0 : (g > N - 1 ? N - 1 : g);
    float v;
    if (c < 3) v = fsub(xyz[(b * N + g) * 3 + c], new_xyz[bs * 3 + c]);
    else v = feats[(b * N + g) * C + (c - 3)];
    grouped[e] = v;
  }
}

static int grid_for(int64_t total, int threads = 256) {
  int64_t g = cdiv(total, threads);
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace pcst

using namespace pcst;

extern "C" int pcst_square_distance(const float* src, const float* dst, int64_t B, int64_t S,
                                    int64_t N, float* out, void* stream) {
  PCST_CHECK_ARG(B >= 0 && S >= 0 && N >= 0, "square_distance: bad shape");
  const int64_t total = B * S * N;
  if (total == 0) return PCST_OK;
  PCST_CHECK_ARG(src && dst && out, "square_distance: null pointer");
  hipLaunchKernelGGL(square_distance_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream),
                     src, dst, S, N, total, out);
  PCST_LAUNCH_CHECK("square_distance");
  return PCST_OK;
}

extern "C" int pcst_index_points(const float* points, int64_t B, int64_t N, int64_t C,
                                 const int64_t* idx, int64_t K, float* out, void* stream) {
  PCST_CHECK_ARG(B >= 0 && N > 0 && C > 0 && K >= 0, "index_points: bad shape");
  const int64_t total = B * K * C;
  if (total == 0) return PCST_OK;
  PCST_CHECK_ARG(points && idx && out, "index_points: null pointer");
  hipLaunchKernelGGL(index_points_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream),
                     points, N, C, idx, K, total, out);
  PCST_LAUNCH_CHECK("index_points");
  return PCST_OK;
}

template <int PPT>
static void launch_fps(const float* xyz, int B, int N, int npoint, const int64_t* start,
                       int64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(fps_reg_kernel<PPT>, dim3(B), dim3(kFpsThreads), 0, s, xyz, N, npoint, start,
                     out);
}

template <int PPT>
static void launch_fps2(const float* xyz, int B, int N, int npoint, const int64_t* start,
                        int64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(fps_key_kernel<PPT>, dim3(B), dim3(kFps2Threads), 0, s, xyz, N, npoint, start,
                     out);
}

template <int PPT>
static void launch_fps_cull(const float* xyz, int B, int N, int npoint, const int64_t* start,
                            int64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(fps_cull_kernel<PPT>, dim3(B), dim3(kFps2Threads), 0, s, xyz, N, npoint, start,
                     out);
}

// the multi-CU kernel's work-groups per cloud, or 0 where it does not apply
static int64_t fps_multi_groups(int64_t B, int64_t N) {
  const int64_t K = cdiv(N, (int64_t)kFpsXThreads * kFpsXPPT);
  return (N > 8192 && K <= 32 && B * K <= kFpsXMaxGroups) ? K : 0;
}

extern "C" int pcst_fps_workspace_size(int64_t B, int64_t N, size_t* bytes) {
  PCST_CHECK_ARG(B >= 0 && N >= 0 && bytes, "fps_workspace_size: bad args");
  // the larger of the multi-CU slots and the streaming fallback's distances (a call with
  // npoint >= 65536 -- more than the slots' 16-bit round tag -- takes the fallback)
  const int64_t K = fps_multi_groups(B, N);
  const size_t slots = K > 0 ? (size_t)(B * K * 2 * kFpsXWords) * sizeof(uint64_t) : 0;
  const size_t dists = (N > (int64_t)kFpsThreads * 60) ? (size_t)(B * N) * sizeof(float) : 0;
  *bytes = slots > dists ? slots : dists;
  return PCST_OK;
}

extern "C" int pcst_fps_ws(const float* xyz, int64_t B, int64_t N, int64_t npoint,
                           const int64_t* start_idx, int64_t* out_idx, void* workspace,
                           void* stream) {
  PCST_CHECK_ARG(B >= 0 && N > 0 && npoint >= 0 && N < (1ll << 31), "fps: bad shape");
  if (B == 0 || npoint == 0) return PCST_OK;
  PCST_CHECK_ARG(xyz && start_idx && out_idx, "fps: null pointer");
  hipStream_t s = as_stream(stream);
  const int b = (int)B, n = (int)N, np = (int)npoint;
  const int64_t K = fps_multi_groups(B, N);
  if (K > 0 && workspace != nullptr && npoint < 65536) {  // the cloud over K work-groups (one XCD), slots zeroed
    const int64_t words = B * K * 2 * kFpsXWords;
    hipLaunchKernelGGL(fpsx_zero_kernel, dim3((unsigned)cdiv(words, 256)), dim3(256), 0, s,
                       static_cast<uint64_t*>(workspace), words);
    hipLaunchKernelGGL(fps_multi_kernel, dim3((unsigned)(B * K * 8)), dim3(kFpsXThreads), 0, s, xyz, n,
                       np, start_idx, out_idx, static_cast<uint64_t*>(workspace), (int)K,
                       (int64_t)kSignalPolls);
    PCST_LAUNCH_CHECK("fps");
    return PCST_OK;
  }
  const int64_t ppt2 = cdiv(N, kFps2Threads);
  if (ppt2 > 8 && ppt2 <= 30) {
    if (ppt2 <= 16) launch_fps_cull<16>(xyz, b, n, np, start_idx, out_idx, s);
    else if (ppt2 <= 24) launch_fps_cull<24>(xyz, b, n, np, start_idx, out_idx, s);
    else launch_fps_cull<30>(xyz, b, n, np, start_idx, out_idx, s);
    PCST_LAUNCH_CHECK("fps");
    return PCST_OK;
  }
  if (ppt2 <= 30) {
    if (ppt2 <= 1) launch_fps2<1>(xyz, b, n, np, start_idx, out_idx, s);
    else if (ppt2 <= 2) launch_fps2<2>(xyz, b, n, np, start_idx, out_idx, s);
    else if (ppt2 <= 4) launch_fps2<4>(xyz, b, n, np, start_idx, out_idx, s);
    else if (ppt2 <= 8) launch_fps2<8>(xyz, b, n, np, start_idx, out_idx, s);
    else if (ppt2 <= 16) launch_fps2<16>(xyz, b, n, np, start_idx, out_idx, s);
    else if (ppt2 <= 24) launch_fps2<24>(xyz, b, n, np, start_idx, out_idx, s);
    else launch_fps2<30>(xyz, b, n, np, start_idx, out_idx, s);
    PCST_LAUNCH_CHECK("fps");
    return PCST_OK;
  }
  const int64_t ppt = cdiv(N, kFpsThreads);
  if (ppt <= 1) launch_fps<1>(xyz, b, n, np, start_idx, out_idx, s);
  else if (ppt <= 2) launch_fps<2>(xyz, b, n, np, start_idx, out_idx, s);
  else if (ppt <= 4) launch_fps<4>(xyz, b, n, np, start_idx, out_idx, s);
  else if (ppt <= 8) launch_fps<8>(xyz, b, n, np, start_idx, out_idx, s);
  else if (ppt <= 16) launch_fps<16>(xyz, b, n, np, start_idx, out_idx, s);
  else if (ppt <= 24) launch_fps<24>(xyz, b, n, np, start_idx, out_idx, s);
  else if (ppt <= 32) launch_fps<32>(xyz, b, n, np, start_idx, out_idx, s);
  else if (ppt <= 40) launch_fps<40>(xyz, b, n, np, start_idx, out_idx, s);
  else if (ppt <= 48) launch_fps<48>(xyz, b, n, np, start_idx, out_idx, s);
  else if (ppt <= 60) launch_fps<60>(xyz, b, n, np, start_idx, out_idx, s);
  else {
    PCST_CHECK_ARG(workspace != nullptr, "fps: N > 30720 needs a workspace of B*N floats");
    hipLaunchKernelGGL(fps_global_kernel, dim3(b), dim3(1024), 0, s, xyz, n, np, start_idx,
                       static_cast<float*>(workspace), out_idx);
  }
  PCST_LAUNCH_CHECK("fps");
  return PCST_OK;
}

extern "C" int pcst_fps(const float* xyz, int64_t B, int64_t N, int64_t npoint,
                        const int64_t* start_idx, int64_t* out_idx, void* stream) {
  PCST_CHECK_ARG(N <= (int64_t)kFpsThreads * 60, "fps: N > 30720 needs pcst_fps_ws");
  return pcst_fps_ws(xyz, B, N, npoint, start_idx, out_idx, nullptr, stream);
}

extern "C" int pcst_ball_query(double radius, int64_t nsample, const float* xyz,
                               const float* new_xyz, int64_t B, int64_t N, int64_t S,
                               int64_t* out_idx, void* stream) {
  PCST_CHECK_ARG(B >= 0 && N > 0 && S >= 0 && nsample > 0 && N < (1ll << 31),
                 "ball_query: bad shape");
  if (B * S == 0) return PCST_OK;
  PCST_CHECK_ARG(xyz && new_xyz && out_idx, "ball_query: null pointer");
  const float r2 = (float)(radius * radius);  // python float r**2, then cast to fp32 (Q4)
  const int64_t waves = B * S;
  const size_t lds = (size_t)kBqWaves * (1 + nsample) * sizeof(int);
  if (lds <= 64 * 1024) {
    hipLaunchKernelGGL(ball_query_split_kernel, dim3((unsigned)(B * S)), dim3(kBqWaves * 64), lds,
                       as_stream(stream), r2, (int)nsample, xyz, new_xyz, (int)N, (int)S, out_idx);
  } else {
    hipLaunchKernelGGL(ball_query_kernel, dim3((unsigned)cdiv(waves, 4)), dim3(256), 0,
                       as_stream(stream), r2, (int)nsample, xyz, new_xyz, (int)B, (int)N, (int)S,
                       out_idx);
  }
  PCST_LAUNCH_CHECK("ball_query");
  return PCST_OK;
}

extern "C" int pcst_group_gather(const float* xyz, const float* feats, int64_t B, int64_t N,
                                 int64_t C, const int64_t* fps_idx, const int64_t* group_idx,
                                 int64_t S, int64_t ns, float* new_xyz, float* grouped,
                                 void* stream) {
  PCST_CHECK_ARG(B >= 0 && N > 0 && C >= 0 && S >= 0 && ns > 0, "group_gather: bad shape");
  PCST_CHECK_ARG(C == 0 || feats != nullptr, "group_gather: feats required when C > 0");
  if (B * S == 0) return PCST_OK;
  hipStream_t s = as_stream(stream);
  const int64_t t1 = B * S * 3;
  hipLaunchKernelGGL(new_xyz_kernel, dim3(grid_for(t1)), dim3(256), 0, s, xyz, N, fps_idx, S, t1,
                     new_xyz);
  const int64_t t2 = B * S * ns * (3 + C);
  hipLaunchKernelGGL(group_gather_kernel, dim3(grid_for(t2)), dim3(256), 0, s, xyz, feats, N, C,
                     new_xyz, group_idx, S, ns, t2, grouped);
  PCST_LAUNCH_CHECK("group_gather");
  return PCST_OK;
}
