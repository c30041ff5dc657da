// Voxel-hash downsample of HierarchicalProcessor._voxel_grid_downsample_torch
// (models/diffusion_model.py:69-122), all clouds of a batch at once, entirely on the device
// (no host round trip for the data-dependent unique-voxel count U or pool size P).
//
// Pipeline (one segment per cloud, grid.y = cloud):
//   minmax -> voxel size + int32 wrap-around hash -> stable LSD radix sort (hash, index)
//   -> unique voxels (head flags, tile scan) -> per-voxel index sum/count (wave segmented
//   reduction + int64 atomics, exact and order independent) -> representative
//   trunc(f32(sum)/f32(count)) in ascending signed-hash order (Q5/Q6) -> pool of
//   non-representative indices in ascending order (tile compaction) -> selection:
//     U > T : reps[perm[:T]]          U < T : reps ++ pool[perm[:T-U]]      U == T : reps
//   with perm either replayed (parity) or drawn on the device: Philox-style 32-bit keys
//   per candidate + the same radix sort = torch.randperm's random-key-sort construction.
#include "common.h"
#include "knn_rows.h"
#include "sort.h"
#include "cloud.h"

namespace pcst {

struct VoxelWS {
  StatRec* mm;           // [B][kStatBlocks] partial min/max records
  uint32_t *kA, *vA, *kB, *vB;  // [B][N]
  uint32_t* hist;        // radix hist
  uint32_t* tileh;       // [B][tiles]
  int32_t* U;            // [B]
  int32_t* P;            // [B]
  int32_t* cand;         // [B]
  unsigned long long* sum;  // [B][N]
  uint32_t* cnt;         // [B][N]
  int64_t* reps;         // [B][N]
  uint32_t* isrep;       // [B][N]
  int32_t* pool;         // [B][N]
  int32_t* err;          // [1]
  float4* vp;            // [B] min xyz + voxel size
  size_t bytes;
};

static VoxelWS carve_voxel(void* base, int64_t B, int64_t N) {
  Carver c(base);
  VoxelWS w;
  const size_t BN = (size_t)(B * N);
  const int64_t tiles = cdiv(N, kSortTile);
  w.mm = c.take<StatRec>(B * kStatBlocks);
  w.kA = c.take<uint32_t>(BN);
  w.vA = c.take<uint32_t>(BN);
  w.kB = c.take<uint32_t>(BN);
  w.vB = c.take<uint32_t>(BN);
  w.hist = c.take<uint32_t>(radix_hist_words((int)B, N));
  w.tileh = c.take<uint32_t>(B * tiles);
  w.U = c.take<int32_t>(B);
  w.P = c.take<int32_t>(B);
  w.cand = c.take<int32_t>(B);
  w.err = c.take<int32_t>(4);
  w.vp = c.take<float4>(B);
  // zeroed every call: sum, cnt, isrep are contiguous so one memset covers them
  w.sum = c.take<unsigned long long>(BN);
  w.cnt = c.take<uint32_t>(BN);
  w.isrep = c.take<uint32_t>(BN);
  w.reps = c.take<int64_t>(BN);
  w.pool = c.take<int32_t>(BN);
  w.bytes = c.bytes();
  return w;
}

// voxel_size = (prod(range)/target)^(1/3) * 1.2 with the reference's fp32/fp64 steps
// (diffusion_model.py:82-87): range < 1e-6 -> 1; prod = (r0*r1)*r2 in fp32; pow of the 0-d
// fp32 tensor is evaluated in double (verified bit-exact), then * 1.2f; < 1e-6 -> 1e-3.
__device__ __forceinline__ float voxel_size(const StatRec& M, int64_t target) {
  float r[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    r[c] = fsub(M.mx[c], M.mn[c]);
    if (r[c] < 1e-6f) r[c] = 1.0f;
  }
  const float prod = fmul(fmul(r[0], r[1]), r[2]);
  const float q = __fdiv_rn(prod, (float)target);
  float vs = (float)pow((double)q, 1.0 / 3.0);
  vs = fmul(vs, 1.2f);
  if (vs < 1e-6f) vs = 1e-3f;
  return vs;
}

// per cloud: fold the stat partials once -> (min x, min y, min z, voxel size)
__global__ __launch_bounds__(64) void vox_params_kernel(const StatRec* __restrict__ mm, int B,
                                                        int64_t target, float4* __restrict__ vp) {
  const int b = blockIdx.x;  // one wave per cloud
  const StatRec M = fold_stats_wave(mm, b);
  if (threadIdx.x == 0) vp[b] = make_float4(M.mn[0], M.mn[1], M.mn[2], voxel_size(M, target));
}

__device__ __forceinline__ int32_t wrap_mul(int32_t a, uint32_t m) {
  return (int32_t)((uint32_t)a * m);
}

// v = int32(floor((p - min) / vs)); h = (vx*73856093)^(vy*19349663)^(vz*83492791) (int32 wrap,
// Q5).  Sort key = h ^ 0x80000000 so unsigned order == torch.unique's signed order.
__global__ __launch_bounds__(256) void vox_hash_kernel(const float* __restrict__ pts, int N,
                                                       const float4* __restrict__ vp,
                                                       uint32_t* __restrict__ keys,
                                                       uint32_t* __restrict__ vals) {
  const int b = blockIdx.y;
  const float4 v4 = vp[b];
  const float vs = v4.w;
  const float m0 = v4.x, m1 = v4.y, m2 = v4.z;
  const float* P = pts + (int64_t)b * N * 3;
  for (int n = blockIdx.x * 256 + threadIdx.x; n < N; n += gridDim.x * 256) {
    const int32_t vx = (int32_t)floorf(__fdiv_rn(fsub(P[n * 3 + 0], m0), vs));
    const int32_t vy = (int32_t)floorf(__fdiv_rn(fsub(P[n * 3 + 1], m1), vs));
    const int32_t vz = (int32_t)floorf(__fdiv_rn(fsub(P[n * 3 + 2], m2), vs));
    const int32_t h = wrap_mul(vx, 73856093u) ^ wrap_mul(vy, 19349663u) ^ wrap_mul(vz, 83492791u);
    keys[(int64_t)b * N + n] = (uint32_t)h ^ 0x80000000u;
    vals[(int64_t)b * N + n] = (uint32_t)n;
  }
}

// Tile element i for (wave w, round r, lane l): base + w*1024 + r*64 + l (input order).
__device__ __forceinline__ int tile_elem(int base, int w, int r, int lane) {
  return base + w * (kSortRounds * 64) + r * 64 + lane;
}

// Count voxel heads (first element of each run of equal sorted keys) per tile.
__global__ __launch_bounds__(256) void vox_head_count_kernel(const uint32_t* __restrict__ keys,
                                                             int N, int tiles,
                                                             uint32_t* __restrict__ tileh) {
  const int b = blockIdx.y, tile = blockIdx.x;
  const int base = tile * kSortTile;
  const uint32_t* K = keys + (int64_t)b * N;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t c = 0;
  for (int r = 0; r < kSortRounds; ++r) {
    const int i = tile_elem(base, w, r, lane);
    const bool head = i < N && (i == 0 || K[i] != K[i - 1]);
    c += __popcll(__ballot(head));
  }
  __shared__ uint32_t s[4];
  if (lane == 0) s[w] = c;
  __syncthreads();
  if (threadIdx.x == 0) tileh[(int64_t)b * tiles + tile] = s[0] + s[1] + s[2] + s[3];
}

// Per-voxel sum of point indices and count: segment id = (#heads in [0, i]) - 1; a wave
// segmented scan leaves one int64 atomic per voxel run per 64 elements.
__global__ __launch_bounds__(256) void vox_segsum_kernel(const uint32_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ vals, int N,
                                                         int tiles,
                                                         const uint32_t* __restrict__ tileoff,
                                                         unsigned long long* __restrict__ sum,
                                                         uint32_t* __restrict__ cnt) {
  const int b = blockIdx.y, tile = blockIdx.x;
  const int base = tile * kSortTile;
  if (base >= N) return;
  const uint32_t* K = keys + (int64_t)b * N;
  const uint32_t* V = vals + (int64_t)b * N;
  unsigned long long* S = sum + (int64_t)b * N;
  uint32_t* C = cnt + (int64_t)b * N;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long lt = lanemask_lt();
  unsigned long long heads[kSortRounds];
  uint32_t wc = 0;
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int i = tile_elem(base, w, r, lane);
    heads[r] = __ballot(i < N && (i == 0 || K[i] != K[i - 1]));
    wc += __popcll(heads[r]);
  }
  __shared__ uint32_t s[4];
  if (lane == 0) s[w] = wc;
  __syncthreads();
  int run = (int)tileoff[(int64_t)b * tiles + tile];
  for (int q = 0; q < w; ++q) run += (int)s[q];
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int i = tile_elem(base, w, r, lane);
    const bool valid = i < N;
    const int seg = run + (int)__popcll(heads[r] & (lt | (1ull << lane))) - 1;
    run += (int)__popcll(heads[r]);
    unsigned long long v = valid ? (unsigned long long)V[i] : 0ull;
    uint32_t c = valid ? 1u : 0u;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned long long ov = __shfl_up(v, off);
      const uint32_t oc = __shfl_up(c, off);
      const int os = __shfl_up(seg, off);
      if (lane >= off && os == seg) { v += ov; c += oc; }
    }
    const int nseg = __shfl_down(seg, 1);
    const bool last = valid && (lane == 63 || nseg != seg || i + 1 >= N);
    if (last) {
      atomicAdd(&S[seg], v);
      atomicAdd(&C[seg], c);
    }
  }
}

// rep_k = trunc(f32(sum_k) / f32(count_k))  (int64 / int64 true division -> float32, Q6).
__global__ void vox_reps_kernel(const unsigned long long* __restrict__ sum,
                                const uint32_t* __restrict__ cnt, const int32_t* __restrict__ U,
                                int N, int64_t* __restrict__ reps, uint32_t* __restrict__ isrep) {
  const int b = blockIdx.y;
  const int u = U[b];
  for (int k = blockIdx.x * 256 + threadIdx.x; k < u; k += gridDim.x * 256) {
    const float fs = (float)(long long)sum[(int64_t)b * N + k];
    const float fc = (float)cnt[(int64_t)b * N + k];
    const int64_t r = (int64_t)__fdiv_rn(fs, fc);
    reps[(int64_t)b * N + k] = r;
    isrep[(int64_t)b * N + r] = 1u;
  }
}

// Pool = ascending indices n with !isrep[n] (diffusion_model.py:105-108).
__global__ __launch_bounds__(256) void vox_pool_count_kernel(const uint32_t* __restrict__ isrep,
                                                             int N, int tiles,
                                                             uint32_t* __restrict__ tileh) {
  const int b = blockIdx.y, tile = blockIdx.x;
  const int base = tile * kSortTile;
  const uint32_t* F = isrep + (int64_t)b * N;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t c = 0;
  for (int r = 0; r < kSortRounds; ++r) {
    const int i = tile_elem(base, w, r, lane);
    c += __popcll(__ballot(i < N && F[i] == 0u));
  }
  __shared__ uint32_t s[4];
  if (lane == 0) s[w] = c;
  __syncthreads();
  if (threadIdx.x == 0) tileh[(int64_t)b * tiles + tile] = s[0] + s[1] + s[2] + s[3];
}

__global__ __launch_bounds__(256) void vox_pool_write_kernel(const uint32_t* __restrict__ isrep,
                                                             int N, int tiles,
                                                             const uint32_t* __restrict__ tileoff,
                                                             int32_t* __restrict__ pool) {
  const int b = blockIdx.y, tile = blockIdx.x;
  const int base = tile * kSortTile;
  if (base >= N) return;
  const uint32_t* F = isrep + (int64_t)b * N;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long lt = lanemask_lt();
  unsigned long long m[kSortRounds];
  uint32_t wc = 0;
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int i = tile_elem(base, w, r, lane);
    m[r] = __ballot(i < N && F[i] == 0u);
    wc += __popcll(m[r]);
  }
  __shared__ uint32_t s[4];
  if (lane == 0) s[w] = wc;
  __syncthreads();
  uint32_t run = tileoff[(int64_t)b * tiles + tile];
  for (int q = 0; q < w; ++q) run += s[q];
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int i = tile_elem(base, w, r, lane);
    if ((m[r] >> lane) & 1ull) pool[(int64_t)b * N + run + __popcll(m[r] & lt)] = i;
    run += __popcll(m[r]);
  }
}

__global__ void vox_cand_kernel(const int32_t* U, const int32_t* P, int B, int64_t target,
                                int32_t* cand) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int u = U[b];
  cand[b] = u > target ? u : (u < target ? P[b] : 0);
}

// splitmix64 finaliser: counter-based random keys (seed, cloud, candidate).
__device__ __forceinline__ uint32_t rand_key(uint64_t seed, int b, int i) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * ((uint64_t)b * 0x100000001ull + (uint64_t)i + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)((z ^ (z >> 31)) >> 32);
}

__global__ void vox_randkey_kernel(const int32_t* __restrict__ cand, int N, uint64_t seed,
                                   uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const int b = blockIdx.y;
  const int n = cand[b];
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    keys[(int64_t)b * N + i] = rand_key(seed, b, i);
    vals[(int64_t)b * N + i] = (uint32_t)i;
  }
}

// Final selection + gather of the kept points (diffusion_model.py:99-119).
// perm source: replayed int64 perms (perm + perm_off[b], perm_len[b]) or device-drawn (dperm).
__global__ void vox_select_kernel(const float* __restrict__ pts, int N, int64_t T,
                                  const int32_t* __restrict__ U, const int32_t* __restrict__ P,
                                  const int64_t* __restrict__ reps, const int32_t* __restrict__ pool,
                                  const int64_t* __restrict__ perm, const int64_t* __restrict__ perm_off,
                                  const int64_t* __restrict__ perm_len,
                                  const uint32_t* __restrict__ dperm, int32_t* __restrict__ err,
                                  int64_t* __restrict__ out_idx, float* __restrict__ out_pts) {
  const int b = blockIdx.y;
  const int u = U[b], p = P[b];
  const int64_t* R = reps + (int64_t)b * N;
  for (int64_t j = blockIdx.x * 256 + threadIdx.x; j < T; j += gridDim.x * 256) {
    int64_t r;
    int64_t pj = -1;  // position drawn from the permutation
    if (u == T) {
      r = R[j];
    } else if (u > T) {
      pj = j;
    } else {
      if (j < u) r = R[j];
      else pj = j - u;
    }
    if (pj >= 0) {
      int64_t k;
      if (perm) {
        const int64_t need = u > T ? u : p;
        if (perm_len[b] != need && threadIdx.x == 0) atomicOr(err, 1);
        k = perm[perm_off[b] + pj];
        if (k < 0 || k >= need) { atomicOr(err, 2); k = 0; }
      } else {
        k = dperm[(int64_t)b * N + pj];
      }
      r = u > T ? R[k] : (int64_t)pool[(int64_t)b * N + k];
    }
    out_idx[(int64_t)b * T + j] = r;
    const float* src = pts + ((int64_t)b * N + r) * 3;
    float* dst = out_pts + ((int64_t)b * T + j) * 3;
    dst[0] = src[0]; dst[1] = src[1]; dst[2] = src[2];
  }
}

// ============================================================================================
// Performance path (device-drawn subset).  The sorts of the replay path are replaced by:
//   open-addressing voxel table (int64 index sums / counts by integer atomics: exact)
//   -> representatives (same values as the sorted path, arbitrary list order)
//   -> random subset of the candidates (reps if U > T, pool if U < T) = the `need` smallest
//      counter-based random keys (key of a rep = f(seed, voxel hash), of a pool point =
//      f(seed, index): independent of list order, hence deterministic), found by a 12-bit
//      radix select plus an exact sort of the boundary bin;
//   -> every kept point is MARKED (a per-row count over the point index: a representative
//      index two voxels share is kept twice, as the reference keeps it) and the emit kernel
//      writes the row in ascending point-index order by a tile prefix over the counts.
// The kept multiset is fixed by the seed, and so is the row order: the result does not
// depend on the arrival order of any atomic (the style encoder's FPS start and ball query
// read positions in this list, so the order matters there).
// Radix-select bins of the 32-bit subset keys (bin = key >> shift).  The kept set is the `need`
// smallest (key, id) whatever the bin width.  Up to 4M points a row uses 1024 bins (shift 22;
// round 4, was 4096): 4x fewer global histogram adds, ~candidates / 1024 boundary-bin ties per
// row for emit to rank; larger clouds keep 4096 (the tie list holds kTieCap).
constexpr int kSelBins = 4096;  // histogram stride per row (the most bins)
static int vox_sel_shift(int64_t N) { return N <= (4ll << 20) ? 22 : 20; }
constexpr int kTieCap = 8192;
constexpr int kVoxChunk = 1024;           // points aggregated per workgroup in LDS (512 / 2048: DESIGN §6a)
constexpr int kVoxLds = 2 * kVoxChunk;    // LDS table slots (load factor <= 1/2)
constexpr int kVoxRepsBlocks = 128;       // workgroups per cloud over the voxel list / dense cells

// Copies.  guided_sample_loop downsamples the CFG batch cat([x] * 2) (diffusion_model.py:244-247):
// identical clouds.  With copies = k the input is the B distinct clouds and the output has the
// k*B rows of cat([x] * k) (row = c*B + b of cloud b = row % B): the voxel table and the
// representatives are built once per cloud, only the random subset is drawn per row, with
// the row's own keys -- the kept SET of every row equals the one the concatenated call draws
// from the same seed.
constexpr int kPrepMaxBlocks = 1024;  // min/max partials of pcst_cfg_ddim_voxel_prep per cloud
struct VoxelFastWS {
  StatRec* mm;            // [B][kStatBlocks]
  float* pmm;             // [B][kPrepMaxBlocks][6]  min xyz, max xyz partials (prepped calls)
  int32_t* sel;           // [R][4]: bin*, rem, need, U>T flag  (R = copies * B rows)
  int64_t* reps;          // [B][N]
  uint32_t* rhash;        // [B][N]
  int32_t* vlist;         // [B][N]    occupied table slots in arrival order (cnt4[b][0] of them)
  int32_t* vdim;          // [B][4]    the voxel box dims (dx, dy, dz) and 1 if the dense grid is used
  unsigned long long* ties;  // [R][kTieCap] (key<<32 | id)
  // zeroed every call (one memset): counters, histograms, tables, rep flags
  int32_t* cnt4;          // [R][4]: U (of cloud r, rows r < B), selected, ties, err
  uint32_t* phist;        // [R][kSelBins] the pool-key histogram of every point made ahead by
                          // pcst_cfg_ddim_voxel_prep (pool calls), outside the zeroed state:
                          // emit zeroes it after its readers (reps, select) are done
  uint32_t* hist;         // [R][kSelBins] pool keys (U < T): every point's, less the reps'
  uint32_t* hist2;        // [R][kSelBins] representative keys (U > T)
  unsigned long long* tkey;  // [B][H]  0 = empty, else (1<<32)|hash
  unsigned long long* tsum;  // [B][H]
  uint32_t* tcnt;         // [B][H]
  uint32_t* isrep;        // [B][N]
  uint32_t* kcnt;         // [R][N]    times point n is kept in row r
  uint32_t* ktile;        // [R][tiles] per-tile sums of kcnt (kEmitTile indices per tile)
  int64_t H, tiles;
  size_t bytes;
};

#ifndef PCST_EMIT_TILE  // experiment builds override (csrc/Makefile XDEF)
#define PCST_EMIT_TILE 1024
#endif
constexpr int kEmitTile = PCST_EMIT_TILE;  // 256 threads x 4 indices
constexpr int kMarkTiles = 1024;  // tiles counted in LDS by the marking kernels

static int64_t vox_table_size(int64_t N) {
  int64_t h = 1024;
  while (h < 2 * N) h <<= 1;
  return h;
}

static VoxelFastWS carve_voxel_fast(void* base, int64_t B, int64_t N, int64_t copies = 1) {
  Carver c(base);
  VoxelFastWS w;
  const int64_t R = B * copies;
  w.H = vox_table_size(N);
  w.mm = c.take<StatRec>(B * kStatBlocks);
  w.pmm = c.take<float>(B * kPrepMaxBlocks * 6);
  w.sel = c.take<int32_t>(R * 4);
  w.reps = c.take<int64_t>(B * N);
  w.rhash = c.take<uint32_t>(B * N);
  w.vlist = c.take<int32_t>(B * N);
  w.vdim = c.take<int32_t>(B * 4);
  w.phist = c.take<uint32_t>(R * kSelBins);
  w.ties = c.take<unsigned long long>(R * kTieCap);
  w.cnt4 = c.take<int32_t>(R * 4);
  w.hist = c.take<uint32_t>(R * kSelBins);
  w.hist2 = c.take<uint32_t>(R * kSelBins);
  w.tkey = c.take<unsigned long long>(B * w.H);
  w.tsum = c.take<unsigned long long>(B * w.H);
  w.tcnt = c.take<uint32_t>(B * w.H);
  w.isrep = c.take<uint32_t>(B * N);
  w.tiles = cdiv(N, kEmitTile);
  w.kcnt = c.take<uint32_t>(R * N);
  w.ktile = c.take<uint32_t>(R * w.tiles);
  w.bytes = c.bytes();
  return w;
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

// Cloud statistics (blocks [0, kStatBlocks) of row y) and, in the other blocks, the zeroing of
// the counters / histograms / tables / rep flags of this call (instead of a separate memset).
constexpr int kVoxZeroBlocks = 128;
constexpr int kPoolBlocks = 16;  // pool-histogram work-groups per row in the prep kernel
__global__ __launch_bounds__(256) void voxf_stats_zero_kernel(const float* __restrict__ pts, int N,
                                                              StatRec* __restrict__ part,
                                                              uint4* __restrict__ zero,
                                                              int64_t zero_words) {
  const int b = blockIdx.y;
  if (blockIdx.x < kStatBlocks) {
    cloud_stats_block(pts + (int64_t)b * N * 3, N, blockIdx.x, part + b * kStatBlocks);
    return;
  }
  const int64_t stride = (int64_t)kVoxZeroBlocks * gridDim.y * 256;
  const int64_t z0 = ((int64_t)b * kVoxZeroBlocks + (blockIdx.x - kStatBlocks)) * 256 + threadIdx.x;
  for (int64_t i = z0; i < zero_words; i += stride) zero[i] = make_uint4(0u, 0u, 0u, 0u);
}

// min / max partials [b][kPrepMaxBlocks][6] of cloud b folded by one wave (s, ss left 0: the
// voxel parameters do not use them)
__device__ __forceinline__ StatRec fold_minmax_wave(const float* __restrict__ pmm, int b, int n) {
  StatRec r;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    r.mn[c] = 3.4e38f;
    r.mx[c] = -3.4e38f;
    r.s[c] = r.ss[c] = 0.0;
  }
  // eight records per lane per round, all loads in flight together (a serial loop here waited
  // out one L2 miss per record: the partials were just written on other XCDs)
  constexpr int kU = 8;
  for (int q0 = threadIdx.x & 63; q0 < n; q0 += kU * 64) {
    float v[kU][6];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int q = q0 + u * 64;
      const float* src = pmm + ((int64_t)b * kPrepMaxBlocks + (q < n ? q : q0)) * 6;
#pragma unroll
      for (int c = 0; c < 6; ++c) v[u][c] = src[c];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        r.mn[c] = fminf(r.mn[c], v[u][c]);
        r.mx[c] = fmaxf(r.mx[c], v[u][3 + c]);
      }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      r.mn[c] = fminf(r.mn[c], __shfl_xor(r.mn[c], off));
      r.mx[c] = fmaxf(r.mx[c], __shfl_xor(r.mx[c], off));
    }
  return r;
}

static int vox_prep_blocks(int64_t N) { return (int)std::min<int64_t>(cdiv(N, 256), kPrepMaxBlocks); }

// pcst_cfg_ddim_voxel_prep: the CFG + DDIM update of C clouds (eps [2C,N,3]: rows c and C + c,
// the elementwise update of sampler.hip's cfg_ddim_kernel through cfg_ddim_value), x_out and
// x_cat [2C,N,3] written, fused with what the next downsample of x_out would launch first: the
// min / max partials of the new points (blocks [0, nprep) of cloud y) and the zeroing of the
// voxel workspace's per-call state (the other blocks).  One launch fewer per sampling step.
__global__ __launch_bounds__(256) void voxf_cfg_prep_kernel(
    const float* __restrict__ x, const float* __restrict__ eps, const float* __restrict__ src,
    int64_t C, int N, float scale, float c1, float c2, float c3, float c4,
    float* __restrict__ x_out, float* __restrict__ x_cat, float* __restrict__ pmm, int nprep,
    uint4* __restrict__ zero, int64_t zero_words, uint32_t* __restrict__ phist, uint64_t pool_seed,
    int copies, int sshift, int vec4) {
  const int c = blockIdx.y;
  if ((int)blockIdx.x >= nprep + kVoxZeroBlocks) {
    // the next downsample's pool-key histogram (every point of this cloud, each copy's row):
    // it depends on (seed, row, index) only, so it is made here instead of in the insert
    const int q = (int)blockIdx.x - nprep - kVoxZeroBlocks;
    const int cp = q / kPoolBlocks, part = q % kPoolBlocks;
    const int row = cp * (int)C + c;
    const int nbins = 1 << (32 - sshift);
    __shared__ uint32_t lh[1024];
    for (int i = threadIdx.x; i < nbins; i += 256) lh[i] = 0u;
    __syncthreads();
    const int per = (N + kPoolBlocks - 1) / kPoolBlocks;
    const int n0 = part * per, n1 = min(n0 + per, N);
    for (int n = n0 + threadIdx.x; n < n1; n += 256)
      atomicAdd(&lh[rand_key(pool_seed, row + 0x10000, n) >> sshift], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < nbins; i += 256)
      if (lh[i]) atomicAdd(&phist[(int64_t)row * kSelBins + i], lh[i]);
    (void)copies;
    return;
  }
  if ((int)blockIdx.x < nprep) {
    float mn[3] = {3.4e38f, 3.4e38f, 3.4e38f}, mx[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
    const int64_t half = C * (int64_t)N * 3;
    // N % 4 == 0 (and 16-B aligned bases, the host's check): four points = three float4 per
    // array and thread, the same elementwise values (cfg_ddim_value) and order-free min / max
    // folds, so the same bits as the per-point loop below; a third of the memory instructions
    // (32 clouds: 138 us at ~2.3 TB/s with the per-point loop)
    const bool quads = vec4 && (N & 3) == 0;
    for (int q = blockIdx.x * 256 + threadIdx.x; quads && q < (N >> 2); q += nprep * 256) {
      const int64_t e0 = ((int64_t)c * N + 4 * (int64_t)q) * 3;  // 12 floats, 16-B aligned
      float xa[12], ca[12], ua[12], sa[12] = {};
      auto ld = [](const float* p, float* d) {
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const float4 v = reinterpret_cast<const float4*>(p)[u];
          d[4 * u + 0] = v.x; d[4 * u + 1] = v.y; d[4 * u + 2] = v.z; d[4 * u + 3] = v.w;
        }
      };
      ld(x + e0, xa);
      ld(eps + e0, ca);
      ld(eps + half + e0, ua);
      if (src) ld(src + e0, sa);
      float o[12];
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        const int j = k % 3;
        o[k] = cfg_ddim_value(xa[k], ca[k], &ua[k], src ? &sa[k] : nullptr, scale, c1, c2, c3, c4);
        mn[j] = fminf(mn[j], o[k]);
        mx[j] = fmaxf(mx[j], o[k]);
      }
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const float4 v = make_float4(o[4 * u + 0], o[4 * u + 1], o[4 * u + 2], o[4 * u + 3]);
        reinterpret_cast<float4*>(x_out + e0)[u] = v;
        reinterpret_cast<float4*>(x_cat + e0)[u] = v;
        reinterpret_cast<float4*>(x_cat + half + e0)[u] = v;
      }
    }
    for (int n = blockIdx.x * 256 + threadIdx.x; !quads && n < N; n += nprep * 256) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int64_t e = ((int64_t)c * N + n) * 3 + j;
        const float xn = cfg_ddim_value(x[e], eps[e], eps + half + e, src ? src + e : nullptr,
                                        scale, c1, c2, c3, c4);
        x_out[e] = xn;
        x_cat[e] = xn;
        x_cat[half + e] = xn;
        mn[j] = fminf(mn[j], xn);
        mx[j] = fmaxf(mx[j], xn);
      }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        mn[j] = fminf(mn[j], __shfl_xor(mn[j], off));
        mx[j] = fmaxf(mx[j], __shfl_xor(mx[j], off));
      }
    __shared__ float w[4][6];
    const int wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
      for (int j = 0; j < 3; ++j) { w[wid][j] = mn[j]; w[wid][3 + j] = mx[j]; }
    __syncthreads();
    if (threadIdx.x < 6) {
      float v = w[0][threadIdx.x];
      for (int q = 1; q < 4; ++q)
        v = threadIdx.x < 3 ? fminf(v, w[q][threadIdx.x]) : fmaxf(v, w[q][threadIdx.x]);
      pmm[((int64_t)c * kPrepMaxBlocks + blockIdx.x) * 6 + threadIdx.x] = v;
    }
    return;
  }
  const int64_t stride = (int64_t)kVoxZeroBlocks * gridDim.y * 256;
  const int64_t z0 = ((int64_t)c * kVoxZeroBlocks + (blockIdx.x - nprep)) * 256 + threadIdx.x;
  for (int64_t i = z0; i < zero_words; i += stride) zero[i] = make_uint4(0u, 0u, 0u, 0u);
}

// Dense voxel grid.  The reference groups points by the int32 xor-hash of their voxel coordinates
// (torch.unique on voxel_hash, diffusion_model.py:89-92), so two voxels whose hashes collide are
// ONE group.  Inside a box of voxel coordinates in which no two voxels share a hash, a group is
// exactly a voxel, and the per-group (index sum, count) can be accumulated by plain atomic adds
// into a dense array indexed by the voxel's position in the box -- no hash table, no probing, no
// returning atomics.  PCST_DENSE_BOXES lists boxes [0,X) x [0,Y) x [0,Z) checked collision-free
// (tools/voxel_cert.py; tests/test_host.py re-checks every entry with numpy); a cloud whose voxel
// box (dx, dy, dz) = floor((max - min) / vs) + 1 lies inside one of them, with dx dy dz <= the
// table size H, takes the dense path, any other the hash table (same groups, same bits).  The
// bench's clouds: noise 26 x 28 x 26, lidar-like 48 x 52 x 8.
// (A table in the kernel's code: a __constant__ array would be a writable host-side symbol.)
#define PCST_DENSE_BOXES                                                                       \
  {56, 56, 56}, {1, 306, 306}, {265, 1, 265}, {313, 313, 1}, {2, 306, 306}, {265, 2, 265},      \
      {305, 305, 2}, {4, 234, 234}, {175, 4, 175}, {196, 196, 4}, {8, 116, 116}, {175, 8, 175}, \
      {190, 190, 8}, {16, 116, 116}, {128, 16, 128}, {117, 117, 16}, {32, 101, 101},            \
      {56, 32, 56}, {90, 90, 32}
__device__ __forceinline__ bool dense_box_ok(int dx, int dy, int dz) {
  constexpr int kBoxes[][3] = {PCST_DENSE_BOXES};
  bool ok = false;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(kBoxes) / sizeof(kBoxes[0])); ++i)
    ok = ok || (dx <= kBoxes[i][0] && dy <= kBoxes[i][1] && dz <= kBoxes[i][2]);
  return ok;
}

// The cloud's voxel box dims (every point's coordinate lies in [0, d): rounding is monotone) and
// whether the dense grid takes it.
__device__ __forceinline__ int4 voxel_box(const StatRec& M, float4 v4, int64_t H, int pack) {
  float q[3];
  q[0] = floorf(__fdiv_rn(fsub(M.mx[0], v4.x), v4.w));
  q[1] = floorf(__fdiv_rn(fsub(M.mx[1], v4.y), v4.w));
  q[2] = floorf(__fdiv_rn(fsub(M.mx[2], v4.z), v4.w));
  if (!(q[0] < 4096.0f && q[1] < 4096.0f && q[2] < 4096.0f)) return make_int4(0, 0, 0, 0);
  const int dx = (int)q[0] + 1, dy = (int)q[1] + 1, dz = (int)q[2] + 1;
  int dense = 0;
#ifdef PCST_VOX_NO_DENSE  // experiment builds only (csrc/Makefile XDEF): the hash table always
  pack = 0;
#endif
  if (pack && (int64_t)dx * dy * dz <= H && dense_box_ok(dx, dy, dz)) dense = 1;
  return make_int4(dx, dy, dz, dense);
}

// The dense grid's accumulators are spread over replicas (point n adds to replica n % R, the
// reps launch sums them): the densest voxels of a noise cloud hold ~300 points, whose 64-bit adds
// to ONE address serialise at the memory-side atomic unit (insert 15.9 us with one replica on a
// squashed noise cloud, tools/voxel_probe.py).  R = the largest power of two <= 8 with R cells
// in the table.
#ifndef PCST_DENSE_REPLICAS  // experiment builds override (csrc/Makefile XDEF)
#define PCST_DENSE_REPLICAS 8
#endif
constexpr int kDenseReplicas = PCST_DENSE_REPLICAS;
__device__ __forceinline__ int dense_replicas(int cells, int64_t H) {
  int r = kDenseReplicas;
  while (r > 1 && (int64_t)r * cells > H) r >>= 1;
  return r;
}

__device__ __forceinline__ uint32_t voxel_hash(int32_t vx, int32_t vy, int32_t vz) {
  return (uint32_t)(wrap_mul(vx, 73856093u) ^ wrap_mul(vy, 19349663u) ^ wrap_mul(vz, 83492791u));
}

// Voxel table insert; the first wave also folds the cloud's min/max partials into the voxel
// parameters (min xyz, voxel size) and the voxel box for its workgroup (work-group 0 records the
// box for the reps launch).  Dense box (voxel_box): one 64-bit add of (index << 20 | 1) per point
// into the dense grid (the table's sum array, zeroed per call), nothing returned.  Otherwise:
// each workgroup first aggregates its kVoxChunk points in an LDS table (LDS atomics), then
// publishes one global (sum, count) per distinct voxel hash: dense voxels see at most one global
// atomic per workgroup instead of one per point.
__global__ __launch_bounds__(256) void voxf_insert_kernel(const float* __restrict__ pts, int N,
                                                          const StatRec* __restrict__ mm,
                                                          int64_t T, int64_t H,
                                                          unsigned long long* __restrict__ tkey,
                                                          unsigned long long* __restrict__ tsum,
                                                          uint32_t* __restrict__ tcnt, int B,
                                                          int copies, uint64_t seed_v,
                                                          const uint64_t* __restrict__ seed_p,
                                                          uint32_t* __restrict__ hist,
                                                          int32_t* __restrict__ cnt4,
                                                          int32_t* __restrict__ vlist, int pack,
                                                          int sshift, const float* __restrict__ pmm,
                                                          int npm, int pool_made,
                                                          uint32_t* __restrict__ sflag, uint32_t svalue,
                                                          int32_t* __restrict__ vdim) {
  // the start signal: every launch ahead of this one on its stream has completed (the points are
  // final), published for another stream (pcst_voxel_downsample_copies_prepped's start_flag)
  if (sflag && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    __hip_atomic_store(sflag, svalue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int nbins = 1 << (32 - sshift);
  const int b = blockIdx.y;
  const float* P = pts + (int64_t)b * N * 3;
  unsigned long long* K = tkey + b * H;
  __shared__ unsigned long long lkey[kVoxLds];
  __shared__ unsigned long long lsum[kVoxLds];
  __shared__ uint32_t lcnt[kVoxLds];
  __shared__ float4 vps;
  __shared__ int4 vbox;
  if (threadIdx.x < 64) {
    // the voxel parameters use only min / max (order-free folds): from the stats partials, or
    // from pcst_cfg_ddim_voxel_prep's min / max partials on a prepped call
    const StatRec M = pmm ? fold_minmax_wave(pmm, b, npm) : fold_stats_wave(mm, b);
    if (threadIdx.x == 0) {
      const float4 v = make_float4(M.mn[0], M.mn[1], M.mn[2], voxel_size(M, T));
      const int4 box = voxel_box(M, v, H, pack);
      vps = v;
      vbox = box;
      if (blockIdx.x == 0) *reinterpret_cast<int4*>(vdim + b * 4) = box;
    }
  }
  __syncthreads();
  const float4 v4 = vps;
  const int4 box = vbox;
  const int n0 = blockIdx.x * kVoxChunk, n1 = min(n0 + kVoxChunk, N);
  if (box.w) {  // the dense grid: cell = vx + dx (vy + dy vz), replica n % kDenseReplicas
    const int cells = box.x * box.y * box.z;
    const int reps = dense_replicas(cells, H);
    unsigned long long* D = tsum + b * H;
    for (int n = n0 + threadIdx.x; n < n1; n += 256) {
      const int32_t vx = (int32_t)floorf(__fdiv_rn(fsub(P[n * 3 + 0], v4.x), v4.w));
      const int32_t vy = (int32_t)floorf(__fdiv_rn(fsub(P[n * 3 + 1], v4.y), v4.w));
      const int32_t vz = (int32_t)floorf(__fdiv_rn(fsub(P[n * 3 + 2], v4.z), v4.w));
      atomicAdd(&D[(n & (reps - 1)) * cells + vx + box.x * (vy + box.y * vz)],
                ((unsigned long long)n << 20) | 1ull);
    }
  } else {
    for (int i = threadIdx.x; i < kVoxLds; i += 256) { lkey[i] = 0ull; lsum[i] = 0ull; lcnt[i] = 0u; }
    __syncthreads();
    for (int n = n0 + threadIdx.x; n < n1; n += 256) {
      const int32_t vx = (int32_t)floorf(__fdiv_rn(fsub(P[n * 3 + 0], v4.x), v4.w));
      const int32_t vy = (int32_t)floorf(__fdiv_rn(fsub(P[n * 3 + 1], v4.y), v4.w));
      const int32_t vz = (int32_t)floorf(__fdiv_rn(fsub(P[n * 3 + 2], v4.z), v4.w));
      const uint32_t h = voxel_hash(vx, vy, vz);
      const unsigned long long kw = (1ull << 32) | h;
      int slot = (int)(mix32(h) & (kVoxLds - 1));
      for (;;) {  // <= kVoxChunk keys in kVoxLds = 2 kVoxChunk slots: always terminates
        const unsigned long long old = atomicCAS(&lkey[slot], 0ull, kw);
        if (old == 0ull || old == kw) break;
        slot = (slot + 1) & (kVoxLds - 1);
      }
      atomicAdd(&lsum[slot], (unsigned long long)n);
      atomicAdd(&lcnt[slot], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kVoxLds; i += 256) {
      const unsigned long long kw = lkey[i];
      if (!kw) continue;
      int64_t slot = mix32((uint32_t)kw) & (H - 1);
      for (;;) {
        const unsigned long long old = atomicCAS(&K[slot], 0ull, kw);
        if (old == 0ull) {  // a new voxel: list its slot (U = the list length, U <= N)
          vlist[(int64_t)b * N + atomicAdd(&cnt4[b * 4 + 0], 1)] = (int32_t)slot;
          break;
        }
        if (old == kw) break;
        slot = (slot + 1) & (H - 1);
      }
      if (pack) {  // N < 2^20: (index sum << 20) | count in one 64-bit add (sum < 2^40)
        atomicAdd(&tsum[b * H + slot], (lsum[i] << 20) | (unsigned long long)lcnt[i]);
      } else {
        atomicAdd(&tsum[b * H + slot], lsum[i]);
        atomicAdd(&tcnt[b * H + slot], lcnt[i]);
      }
    }
  }
  // The pool-key histogram of every row of this cloud over EVERY point of the chunk (a pool
  // key depends on (seed, row, index) only); voxf_reps_kernel takes the representatives' keys
  // back out, leaving the histogram of the pool (the U < T candidates) without a launch of its
  // own.  The LDS table above is reused as the (at most 4096) bins (kVoxLds * 8 B >= 16 KiB).
  static_assert(kVoxLds * 2 >= 1024, "LDS table too small for the key histogram");
  uint32_t* lh = reinterpret_cast<uint32_t*>(lkey);
  const uint64_t seed = seed_p ? *seed_p : seed_v;
  for (int c = 0; c < (pool_made ? 0 : copies); ++c) {  // (a pool call: the prep made it)
    const int row = c * B + b;
    __syncthreads();
    for (int i = threadIdx.x; i < nbins; i += 256) lh[i] = 0u;
    __syncthreads();
    for (int n = n0 + threadIdx.x; n < n1; n += 256)
      atomicAdd(&lh[rand_key(seed, row + 0x10000, n) >> sshift], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < nbins; i += 256)
      if (lh[i]) atomicAdd(&hist[(int64_t)row * kSelBins + i], lh[i]);
  }
}

// occupied slot -> representative trunc(f32(sum)/f32(count)) (Q6); list order = arrival order
// (only the SET matters downstream: rows are emitted in point-index order).
// One listed voxel (voxf_insert_kernel's slot list) -> representative trunc(f32(sum)/f32(count))
// (Q6) at its list position (arrival order: only the SET matters downstream, rows are emitted in
// point-index order).  Each representative also updates both selection histograms of every row
// of its cloud: its voxel's key into hist2 (the U > T candidates), and its index's pool key out of
// hist (once per distinct index: the first voxel to flag the index does it).
__device__ __forceinline__ void voxf_rep_out(int64_t r, uint32_t h, int k, int b, int N, int B,
                                             int copies, uint64_t seed, int64_t* __restrict__ reps,
                                             uint32_t* __restrict__ rhash, uint32_t* __restrict__ isrep,
                                             uint32_t* __restrict__ hist, uint32_t* __restrict__ hist2,
                                             int sshift) {
  reps[(int64_t)b * N + k] = r;
  rhash[(int64_t)b * N + k] = h;
  const bool first = atomicExch(&isrep[(int64_t)b * N + r], 1u) == 0u;
  for (int c = 0; c < copies; ++c) {
    const int row = c * B + b;
    atomicAdd(&hist2[(int64_t)row * kSelBins + (rand_key(seed, row, (int)(h & 0x7fffffff)) >> sshift)], 1u);
    if (first) atomicSub(&hist[(int64_t)row * kSelBins + (rand_key(seed, row + 0x10000, (int)r) >> sshift)], 1u);
  }
}

// Dense grid (vdim[b].w): one thread per cell of the voxel box (its replicas summed), an
// occupied cell -> its representative, its voxel hash (recomputed from the cell's coordinates)
// and a list position taken by one atomic per wave (cnt4[b][0] counts the listed voxels: U).
__global__ __launch_bounds__(256) void voxf_reps_kernel(
    const unsigned long long* __restrict__ tkey, const unsigned long long* __restrict__ tsum,
    const uint32_t* __restrict__ tcnt, int64_t H, int N, int32_t* __restrict__ cnt4,
    const int32_t* __restrict__ vlist, int pack, int64_t* __restrict__ reps,
    uint32_t* __restrict__ rhash, uint32_t* __restrict__ isrep, int B, int copies, uint64_t seed_v,
    const uint64_t* __restrict__ seed_p, uint32_t* __restrict__ hist, uint32_t* __restrict__ hist2,
    int sshift, const int32_t* __restrict__ vdim) {
  const int b = blockIdx.y;
  const uint64_t seed = seed_p ? *seed_p : seed_v;
  const int4 box = *reinterpret_cast<const int4*>(vdim + b * 4);
  if (box.w) {
    const int cells = box.x * box.y * box.z;
    const int lane = threadIdx.x & 63;
    // whole waves per round (the list position is taken per wave)
    const int nrep = dense_replicas(cells, H);
    for (int c0 = (blockIdx.x * 256 + threadIdx.x) & ~63; c0 < cells; c0 += gridDim.x * 256) {
      const int c = c0 + lane;
      unsigned long long v = 0ull;
      if (c < cells)
        for (int k = 0; k < nrep; ++k) v += tsum[b * H + (int64_t)k * cells + c];
      const uint64_t occ = __ballot(v != 0ull);
      if (!occ) continue;
      int base = 0;
      if (lane == 0) base = atomicAdd(&cnt4[b * 4 + 0], (int)__popcll(occ));
      base = __shfl(base, 0);
      if (v == 0ull) continue;
      const float fs = (float)(long long)(v >> 20);
      const float fc = (float)(uint32_t)(v & 0xFFFFFull);
      const int64_t r = (int64_t)__fdiv_rn(fs, fc);
      const int32_t vx = c % box.x, vy = (c / box.x) % box.y, vz = c / (box.x * box.y);
      const int k = base + (int)__popcll(occ & lanemask_lt());
      voxf_rep_out(r, voxel_hash(vx, vy, vz), k, b, N, B, copies, seed, reps, rhash, isrep, hist,
                   hist2, sshift);
    }
    return;
  }
  const int U = cnt4[b * 4 + 0];
  for (int k = blockIdx.x * 256 + threadIdx.x; k < U; k += gridDim.x * 256) {
    const int64_t s = vlist[(int64_t)b * N + k];
    const unsigned long long kw = tkey[b * H + s];
    const unsigned long long v = tsum[b * H + s];
    const float fs = (float)(long long)(pack ? (v >> 20) : v);
    const float fc = (float)(pack ? (uint32_t)(v & 0xFFFFFull) : tcnt[b * H + s]);
    const int64_t r = (int64_t)__fdiv_rn(fs, fc);
    voxf_rep_out(r, (uint32_t)kw, k, b, N, B, copies, seed, reps, rhash, isrep, hist, hist2, sshift);
  }
}

// candidate e of row `row` (cloud cl): (key, id); returns false if e is not a candidate.  Keys
// follow the row, the candidate arrays the cloud.
__device__ __forceinline__ bool voxf_cand(int row, int cl, int e, int N, int U, int64_t T,
                                          uint64_t seed, const uint32_t* __restrict__ rhash,
                                          const uint32_t* __restrict__ isrep, uint32_t& key,
                                          uint32_t& id) {
  if (U > T) {
    if (e >= U) return false;
    id = (uint32_t)e;
    key = rand_key(seed, row, (int)(rhash[(int64_t)cl * N + e] & 0x7fffffff));
    return true;
  }
  if (U == T || e >= N || isrep[(int64_t)cl * N + e]) return false;
  id = (uint32_t)e;
  key = rand_key(seed, row + 0x10000, e);
  return true;
}

// kept candidate -> one more keep of its point index in this row (index n = the rep's index if
// U > T, else the pool index itself); tile sums in LDS (lt) when the tile is < kMarkTiles
__device__ __forceinline__ void voxf_mark(int row, int N, int64_t n, uint32_t* __restrict__ kcnt,
                                          uint32_t* __restrict__ ktile, int64_t tiles,
                                          uint32_t* lt) {
  atomicAdd(&kcnt[(int64_t)row * N + n], 1u);
  const int64_t tl = n / kEmitTile;
  if (tl < kMarkTiles) atomicAdd(&lt[tl], 1u);
  else atomicAdd(&ktile[row * tiles + tl], 1u);
}

__device__ __forceinline__ void voxf_flush_tiles(int row, int64_t tiles, const uint32_t* lt,
                                                 uint32_t* __restrict__ ktile) {
  __syncthreads();
  const int nt = (int)(tiles < kMarkTiles ? tiles : kMarkTiles);
  for (int i = threadIdx.x; i < nt; i += blockDim.x)
    if (lt[i]) atomicAdd(&ktile[row * tiles + i], lt[i]);
}

// Every workgroup first finds the row's boundary bin b* (the bin holding the need-th smallest
// key) from the histogram; workgroup 0 records it for the emit kernel's tie ranking.  Then, over one
// contiguous candidate range per workgroup: U <= T keeps every representative; keys below b*
// are kept, keys in b* go to the tie list (its order is irrelevant: the emit kernel ranks).
__global__ __launch_bounds__(256) void voxf_select_kernel(
    int N, int64_t T, int B, uint64_t seed_v, const uint64_t* __restrict__ seed_p,
    const uint32_t* __restrict__ hist, const uint32_t* __restrict__ hist2,
    int32_t* __restrict__ sel, int32_t* __restrict__ cnt4,
    const uint32_t* __restrict__ rhash, const uint32_t* __restrict__ isrep,
    const int64_t* __restrict__ reps, unsigned long long* __restrict__ ties,
    uint32_t* __restrict__ kcnt, uint32_t* __restrict__ ktile, int64_t tiles, int sshift) {
  const uint64_t seed = seed_p ? *seed_p : seed_v;
  const int row = blockIdx.y, cl = row % B;
  const int U = cnt4[cl * 4];
  const int need = U > T ? (int)T : (U < T ? (int)(T - U) : 0);
  __shared__ uint32_t sh[260];
  __shared__ uint32_t lt[kMarkTiles];
  __shared__ int s_bstar, s_rem;
  for (int i = threadIdx.x; i < kMarkTiles; i += 256) lt[i] = 0u;
  {
    constexpr int per = kSelBins / 256;
    const int nbins = 1 << (32 - sshift);  // bins past nbins read as empty
    uint32_t v[per], s = 0;
    const uint32_t* hs = (U > T ? hist2 : hist) + (int64_t)row * kSelBins;
#pragma unroll
    for (int k = 0; k < per; ++k) {
      v[k] = threadIdx.x * per + k < nbins ? hs[threadIdx.x * per + k] : 0u;
      s += v[k];
    }
    if (threadIdx.x == 0) { s_bstar = -1; s_rem = 0; }
    uint32_t tot;
    uint32_t run = block_excl_scan_256(s, sh, tot);
#pragma unroll
    for (int k = 0; k < per; ++k) {
      if (need > 0 && run < (uint32_t)need && run + v[k] >= (uint32_t)need) {
        s_bstar = threadIdx.x * per + k;
        s_rem = need - (int)run;
      }
      run += v[k];
    }
    __syncthreads();
  }
  const int bstar = s_bstar;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    sel[row * 4 + 0] = bstar;
    sel[row * 4 + 1] = s_rem;
    sel[row * 4 + 2] = need;
    sel[row * 4 + 3] = U > T ? 1 : 0;
  }
  const int chunk = (N + gridDim.x - 1) / gridDim.x;
  const int e0 = blockIdx.x * chunk, e1 = min(e0 + chunk, N);
  const int64_t* R = reps + (int64_t)cl * N;
  if (U <= T) {  // every representative entry is kept (a shared index twice)
    for (int e = e0 + threadIdx.x; e < min(e1, U); e += 256)
      voxf_mark(row, N, R[e], kcnt, ktile, tiles, lt);
  }
  if (bstar >= 0) {
    for (int e = e0 + threadIdx.x; e < e1; e += 256) {
      uint32_t key, id;
      if (!voxf_cand(row, cl, e, N, U, T, seed, rhash, isrep, key, id)) continue;
      const int bin = (int)(key >> sshift);
      if (bin < bstar) {
        voxf_mark(row, N, U > T ? R[id] : (int64_t)id, kcnt, ktile, tiles, lt);
      } else if (bin == bstar) {
        const int pti = atomicAdd(&cnt4[row * 4 + 2], 1);
        if (pti < kTieCap) ties[(int64_t)row * kTieCap + pti] = ((unsigned long long)key << 32) | id;
        else atomicOr(&cnt4[row * 4 + 3], 1);
      }
    }
  }
  voxf_flush_tiles(row, tiles, lt, ktile);
}

// Row emit in ascending point-index order: tile j's offset is the sum of the earlier tiles'
// keep counts; inside the tile a block scan places each index kcnt[n] times (index + point).
// The boundary bin's ties (select's list, one per row) are ranked exactly by (key, id) here, by
// every workgroup of the row (the list holds about candidates / 4096 entries), instead of by a
// launch of their own: the kept ties in this tile add to its counts, those in earlier tiles to
// its offset.  The 16 points of a thread are loaded before any store, so their latencies overlap.
constexpr int kTieLds = 2048;  // ties ranked from LDS up to this many (else from L2)
__global__ __launch_bounds__(256) void voxf_emit_kernel(const float* __restrict__ pts, int N,
                                                        int64_t T, int B,
                                                        const uint32_t* __restrict__ kcnt,
                                                        const uint32_t* __restrict__ ktile,
                                                        int64_t tiles, int32_t* __restrict__ cnt4,
                                                        const int32_t* __restrict__ sel,
                                                        const unsigned long long* __restrict__ ties,
                                                        const int64_t* __restrict__ reps,
                                                        int64_t* __restrict__ out_idx,
                                                        float* __restrict__ out_pts,
                                                        uint32_t* __restrict__ phist,
                                                        const RowsPlace rp,
                                                        const uint32_t* __restrict__ wflag,
                                                        uint32_t wvalue, int32_t* __restrict__ werr,
                                                        int64_t max_polls) {
  constexpr int kPer = kEmitTile / 256;
  const int row = blockIdx.y, cl = row % B;
  const int64_t tile = blockIdx.x;
  if (tile == 0)  // the row's pool histogram is read (reps, select) before this launch: clear it
    for (int i = threadIdx.x; i < kSelBins; i += 256) phist[(int64_t)row * kSelBins + i] = 0u;
  __shared__ uint32_t sh[260];
  __shared__ uint32_t add[kEmitTile];
  __shared__ unsigned long long tl[kTieLds];
  const int64_t n0 = tile * kEmitTile + threadIdx.x * kPer;
  const uint32_t* C = kcnt + (int64_t)row * N;
  const float* P = pts + (int64_t)cl * N * 3;
  uint32_t c[kPer];
  float q[kPer * 3];
#pragma unroll
  for (int k = 0; k < kPer; ++k) c[k] = n0 + k < N ? C[n0 + k] : 0u;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t n = n0 + k < N ? n0 + k : N - 1;
    q[3 * k] = P[n * 3]; q[3 * k + 1] = P[n * 3 + 1]; q[3 * k + 2] = P[n * 3 + 2];
  }
  // the boundary bin: keep the `rem` smallest (key, id) of the row's tie list
  for (int i = threadIdx.x; i < kEmitTile; i += 256) add[i] = 0u;
  const int bstar = sel[row * 4 + 0];
  uint32_t tie_before = 0;
  if (bstar >= 0) {
    const int rem = sel[row * 4 + 1];
    const int U = cnt4[(row % B) * 4];
    const int nt = min(cnt4[row * 4 + 2], kTieCap);
    const unsigned long long* Tb = ties + (int64_t)row * kTieCap;
    const bool in_lds = nt <= kTieLds;
    if (in_lds)
      for (int i = threadIdx.x; i < nt; i += 256) tl[i] = Tb[i];
    __syncthreads();
    for (int i = threadIdx.x; i < nt; i += 256) {
      const unsigned long long v = in_lds ? tl[i] : Tb[i];
      int rank = 0;
      if (in_lds)
        for (int k = 0; k < nt; ++k) rank += tl[k] < v;
      else
        for (int k = 0; k < nt; ++k) rank += Tb[k] < v;
      if (rank < rem) {
        const uint32_t id = (uint32_t)v;
        const int64_t n = U > T ? reps[(int64_t)cl * N + id] : (int64_t)id;
        const int64_t tn = n / kEmitTile;
        if (tn < tile) ++tie_before;
        else if (tn == tile) atomicAdd(&add[n - tile * kEmitTile], 1u);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPer; ++k) c[k] += add[threadIdx.x * kPer + k];
  uint32_t before = tie_before;
  for (int64_t i = threadIdx.x; i < tile; i += 256) before += ktile[row * tiles + i];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) s += c[k];
  uint32_t tot0, tot;
  block_excl_scan_256(before, sh, tot0);  // tot0 = everything kept in the earlier tiles
  int64_t pos = (int64_t)tot0 + block_excl_scan_256(s, sh, tot);
  int64_t p0[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    p0[k] = pos;
    for (uint32_t r = 0; r < c[k]; ++r, ++pos) {
      if (pos >= T) { atomicOr(&cnt4[row * 4 + 3], 2); break; }
      out_idx[row * T + pos] = n0 + k;
      float* d = out_pts + (row * T + pos) * 3;
      d[0] = q[3 * k]; d[1] = q[3 * k + 1]; d[2] = q[3 * k + 2];
    }
  }
  // Phase B of the step's kNN rows layout (rp.refs given; knn_rows.h): every kept copy j of point
  // n is placed as the query's ref j of this row, once phase A (the side stream's binning of the
  // same points) has published its flag -- the wait comes after this launch's own output, and a
  // work-group whose wait gives up places nothing and sets *werr (the query then reads nothing).
  if (rp.refs && (!wflag || block_wait_flag(wflag, wvalue, werr, max_polls))) {
#pragma unroll
    for (int k = 0; k < kPer; ++k)
      for (uint32_t r = 0; r < c[k] && p0[k] + r < T; ++r) {
        const float pt[3] = {q[3 * k], q[3 * k + 1], q[3 * k + 2]};
        rows_place(rp, row, n0 + k, p0[k] + r, pt);
      }
  }
}

// stats (+ zeroing), insert (+ voxel parameters, every point's pool-key histogram), reps (+ the
// representatives' keys into / out of the histograms), select (+ boundary bin, marks, tie list),
// emit (+ tie ranking; rows in point-index order): 5 launches.
static size_t vox_zero_bytes(const VoxelFastWS& w, int64_t rows) {
  return (size_t)((char*)(w.ktile + rows * w.tiles) - (char*)w.cnt4);
}

// place (optional): phase B of the kNN rows layout fused into the emit (knn_rows.h RowsPlace of
// the rows workspace, with its phase-A flag wait).
struct EmitPlace {
  const KnnRowsWS* kw = nullptr;  // the rows workspace (rp's arrays)
  RowsPlace rp{};
  const uint32_t* wflag = nullptr;
  uint32_t wvalue = 0;
  int32_t* werr = nullptr;
  int64_t max_polls = 0;
};

static int voxel_fast(const float* pts, int64_t B, int64_t N, int64_t copies, int64_t T,
                      void* workspace, uint64_t seed, const uint64_t* seed_p, int64_t* out_idx,
                      float* out_pts, hipStream_t s, bool prepped = false, bool pool = false,
                      uint32_t* sflag = nullptr, uint32_t svalue = 0,
                      const EmitPlace& place = EmitPlace()) {
  VoxelFastWS w = carve_voxel_fast(workspace, B, N, copies);
  const int b = (int)B, n = (int)N, rows = (int)(B * copies);
  if (!prepped)  // (a prepped call: pcst_cfg_ddim_voxel_prep made the partials and zeroed)
    hipLaunchKernelGGL(voxf_stats_zero_kernel, dim3(kStatBlocks + kVoxZeroBlocks, b), dim3(256), 0,
                       s, pts, n, w.mm, reinterpret_cast<uint4*>(w.cnt4),
                       (int64_t)cdiv(vox_zero_bytes(w, rows), 16));
  const int cp = (int)copies;
  const int pack = N < (1 << 20) ? 1 : 0;
  const int sshift = vox_sel_shift(N);
  PCST_CHECK_ARG((1 << (32 - sshift)) <= 2 * kVoxLds, "voxel_downsample: cloud too large for this build");
  hipLaunchKernelGGL(voxf_insert_kernel, dim3((unsigned)cdiv(N, kVoxChunk), b), dim3(256), 0, s,
                     pts, n, w.mm, T, w.H, w.tkey, w.tsum, w.tcnt, b, cp, seed, seed_p, w.hist, w.cnt4,
                     w.vlist, pack, sshift, prepped ? w.pmm : nullptr, vox_prep_blocks(N), pool ? 1 : 0,
                     sflag, svalue, w.vdim);
  uint32_t* hist = pool ? w.phist : w.hist;  // the pool histogram: made ahead, or by the insert
  hipLaunchKernelGGL(voxf_reps_kernel, dim3((unsigned)std::min<int64_t>(cdiv(N, 256), kVoxRepsBlocks), b),
                     dim3(256), 0, s, w.tkey, w.tsum, w.tcnt, w.H, n, w.cnt4, w.vlist, pack, w.reps,
                     w.rhash, w.isrep, b, cp, seed, seed_p, hist, w.hist2, sshift, w.vdim);
  hipLaunchKernelGGL(voxf_select_kernel, dim3(128, rows), dim3(256), 0, s, n, T, b, seed, seed_p,
                     hist, w.hist2, w.sel, w.cnt4, w.rhash, w.isrep, w.reps, w.ties, w.kcnt,
                     w.ktile, w.tiles, sshift);
  // the placement inside the emit only while its work-groups fit one per CU (each may wait for
  // phase A, which needs CUs to finish); otherwise phase B's own, capped launch after it
  const bool fuse = place.rp.refs != nullptr && (int64_t)w.tiles * rows <= device_cus();
  const EmitPlace none;
  const EmitPlace& ep = fuse ? place : none;
  hipLaunchKernelGGL(voxf_emit_kernel, dim3((unsigned)w.tiles, rows), dim3(256), 0, s, pts, n, T,
                     b, w.kcnt, w.ktile, w.tiles, w.cnt4, w.sel, w.ties, w.reps, out_idx, out_pts,
                     w.phist, ep.rp, ep.wflag, ep.wvalue, ep.werr,
                     ep.max_polls > 0 ? ep.max_polls : (int64_t)kSignalPolls);
  if (place.rp.refs != nullptr && !fuse)
    rows_place_launch(*place.kw, pts, out_idx, N, T, place.wflag, place.wvalue, place.werr, place.max_polls, s);
  PCST_LAUNCH_CHECK("voxel_downsample");
  return PCST_OK;
}

}  // namespace pcst

using namespace pcst;

extern "C" int pcst_voxel_workspace_size(int64_t B, int64_t N, size_t* bytes) {
  PCST_CHECK_ARG(B >= 0 && N >= 0 && bytes, "voxel_workspace_size: bad args");
  *bytes = std::max(carve_voxel(nullptr, B, N).bytes, carve_voxel_fast(nullptr, B, N).bytes);
  return PCST_OK;
}

extern "C" int pcst_voxel_copies_workspace_size(int64_t B, int64_t N, int64_t copies,
                                                size_t* bytes) {
  PCST_CHECK_ARG(B >= 0 && N >= 0 && copies >= 1 && bytes, "voxel_copies_workspace_size: bad args");
  *bytes = carve_voxel_fast(nullptr, B, N, copies).bytes;
  return PCST_OK;
}

static int voxel_grid(int64_t N) { return (int)std::min<int64_t>(cdiv(N, 256), 1024); }

extern "C" int pcst_voxel_stats(const float* pts, int64_t B, int64_t N, int64_t target,
                                void* workspace, int32_t* counts_out, void* stream) {
  PCST_CHECK_ARG(B > 0 && N > target && target > 0 && N < (1ll << 30), "voxel_stats: bad shape");
  PCST_CHECK_ARG(pts && workspace, "voxel_stats: null pointer");
  hipStream_t s = as_stream(stream);
  VoxelWS w = carve_voxel(workspace, B, N);
  const int tiles = (int)cdiv(N, kSortTile);
  const int b = (int)B, n = (int)N;
  const size_t zero_bytes = (size_t)((char*)w.reps - (char*)w.sum);
  PCST_HIP(hipMemsetAsync(w.sum, 0, zero_bytes, s), "voxel_stats: memset");
  PCST_HIP(hipMemsetAsync(w.err, 0, 16, s), "voxel_stats: memset");
  launch_cloud_stats(pts, b, n, w.mm, s);
  hipLaunchKernelGGL(vox_params_kernel, dim3((unsigned)B), dim3(64), 0, s, w.mm, b,
                     target, w.vp);
  hipLaunchKernelGGL(vox_hash_kernel, dim3(voxel_grid(N), b), dim3(256), 0, s, pts, n, w.vp,
                     w.kA, w.vA);
  SegCounts all{nullptr, n};
  int rc = radix_sort_pairs(w.kA, w.vA, w.kB, w.vB, w.hist, b, N, all, 0, 32, s);
  if (rc) return rc;
  hipLaunchKernelGGL(vox_head_count_kernel, dim3(tiles, b), dim3(256), 0, s, w.kA, n, tiles,
                     w.tileh);
  seg_scan_small(w.tileh, b, tiles, tiles, w.U, s);
  hipLaunchKernelGGL(vox_segsum_kernel, dim3(tiles, b), dim3(256), 0, s, w.kA, w.vA, n, tiles,
                     w.tileh, w.sum, w.cnt);
  hipLaunchKernelGGL(vox_reps_kernel, dim3(voxel_grid(N), b), dim3(256), 0, s, w.sum, w.cnt, w.U,
                     n, w.reps, w.isrep);
  hipLaunchKernelGGL(vox_pool_count_kernel, dim3(tiles, b), dim3(256), 0, s, w.isrep, n, tiles,
                     w.tileh);
  seg_scan_small(w.tileh, b, tiles, tiles, w.P, s);
  hipLaunchKernelGGL(vox_pool_write_kernel, dim3(tiles, b), dim3(256), 0, s, w.isrep, n, tiles,
                     w.tileh, w.pool);
  hipLaunchKernelGGL(vox_cand_kernel, dim3(cdiv(B, 256)), dim3(256), 0, s, w.U, w.P, b, target,
                     w.cand);
  if (counts_out) {
    PCST_HIP(hipMemcpyAsync(counts_out, w.U, sizeof(int32_t) * B, hipMemcpyDeviceToDevice, s),
             "voxel_stats: copy U");
    PCST_HIP(hipMemcpyAsync(counts_out + B, w.P, sizeof(int32_t) * B, hipMemcpyDeviceToDevice, s),
             "voxel_stats: copy P");
  }
  PCST_LAUNCH_CHECK("voxel_stats");
  return PCST_OK;
}

extern "C" int pcst_voxel_select(const float* pts, int64_t B, int64_t N, int64_t target,
                                 void* workspace, const int64_t* perm, const int64_t* perm_off,
                                 const int64_t* perm_len, uint64_t seed, int64_t* out_idx,
                                 float* out_pts, void* stream) {
  PCST_CHECK_ARG(B > 0 && N > target && target > 0, "voxel_select: bad shape");
  PCST_CHECK_ARG(pts && workspace && out_idx && out_pts, "voxel_select: null pointer");
  PCST_CHECK_ARG(!perm || (perm_off && perm_len), "voxel_select: perm needs perm_off/perm_len");
  hipStream_t s = as_stream(stream);
  VoxelWS w = carve_voxel(workspace, B, N);
  const int b = (int)B, n = (int)N;
  if (!perm) {
    hipLaunchKernelGGL(vox_randkey_kernel, dim3(voxel_grid(N), b), dim3(256), 0, s, w.cand, n,
                       seed, w.kA, w.vA);
    SegCounts cc{w.cand, 0};
    int rc = radix_sort_pairs(w.kA, w.vA, w.kB, w.vB, w.hist, b, N, cc, 0, 32, s);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(vox_select_kernel, dim3((unsigned)std::min<int64_t>(cdiv(target, 256), 1024), b),
                     dim3(256), 0, s, pts, n, target, w.U, w.P, w.reps, w.pool, perm, perm_off,
                     perm_len, w.vA, w.err, out_idx, out_pts);
  PCST_LAUNCH_CHECK("voxel_select");
  return PCST_OK;
}

extern "C" int pcst_voxel_error(void* workspace, int64_t B, int64_t N, int32_t* err_out,
                                void* stream) {
  VoxelWS w = carve_voxel(workspace, B, N);
  PCST_HIP(hipMemcpyAsync(err_out, w.err, sizeof(int32_t), hipMemcpyDeviceToDevice,
                          as_stream(stream)), "voxel_error");
  return PCST_OK;
}

extern "C" int pcst_voxel_downsample(const float* pts, int64_t B, int64_t N, int64_t target,
                                     void* workspace, uint64_t seed, int64_t* out_idx,
                                     float* out_pts, void* stream) {
  PCST_CHECK_ARG(B > 0 && N > target && target > 0 && N < (1ll << 30), "voxel_downsample: bad shape");
  PCST_CHECK_ARG(pts && workspace && out_idx && out_pts, "voxel_downsample: null pointer");
  return voxel_fast(pts, B, N, 1, target, workspace, seed, nullptr, out_idx, out_pts,
                    as_stream(stream));
}

extern "C" int pcst_voxel_downsample_copies(const float* pts, int64_t B, int64_t N, int64_t copies,
                                            int64_t target, void* workspace, uint64_t seed,
                                            int64_t* out_idx, float* out_pts, void* stream) {
  PCST_CHECK_ARG(B > 0 && copies >= 1 && B * copies < (1 << 15) && N > target && target > 0 &&
                     N < (1ll << 30),
                 "voxel_downsample_copies: bad shape");
  PCST_CHECK_ARG(pts && workspace && out_idx && out_pts, "voxel_downsample_copies: null pointer");
  return voxel_fast(pts, B, N, copies, target, workspace, seed, nullptr, out_idx, out_pts,
                    as_stream(stream));
}

extern "C" int pcst_voxel_downsample_copies_prepped(const float* pts, int64_t B, int64_t N,
                                                    int64_t copies, int64_t target, void* workspace,
                                                    uint64_t seed, int pool, int64_t* out_idx,
                                                    float* out_pts, uint32_t* start_flag,
                                                    uint32_t start_value, void* stream) {
  PCST_CHECK_ARG(B > 0 && copies >= 1 && B * copies < (1 << 15) && N > target && target > 0 &&
                     N < (1ll << 30),
                 "voxel_downsample_copies_prepped: bad shape");
  PCST_CHECK_ARG(pts && workspace && out_idx && out_pts, "voxel_downsample_copies_prepped: null pointer");
  return voxel_fast(pts, B, N, copies, target, workspace, seed, nullptr, out_idx, out_pts,
                    as_stream(stream), true, pool != 0, start_flag, start_value);
}

extern "C" int pcst_voxel_downsample_rows(const float* pts, int64_t B, int64_t N, int64_t copies,
                                          int64_t target, void* workspace, uint64_t seed,
                                          int prepped, int pool, int64_t* out_idx, float* out_pts,
                                          uint32_t* start_flag, uint32_t start_value,
                                          void* knn_workspace, const uint32_t* wait_flag,
                                          uint32_t wait_value, int32_t* wait_err, int64_t max_polls,
                                          void* stream) {
  PCST_CHECK_ARG(B > 0 && copies >= 1 && B * copies < (1 << 15) && N > target && target > 0 &&
                     N < (1ll << 30) && target < (1ll << 27),
                 "voxel_downsample_rows: bad shape");
  PCST_CHECK_ARG(pts && workspace && out_idx && out_pts && knn_workspace,
                 "voxel_downsample_rows: null pointer");
  PCST_CHECK_ARG(prepped || (!pool && !start_flag), "voxel_downsample_rows: pool / start need prepped");
  const KnnRowsWS kw = carve_knn_rows(knn_workspace, B, copies, N, target);
  EmitPlace place;
  place.kw = &kw;
  place.rp = rows_place_args(kw, N, target);
  place.wflag = wait_flag;
  place.wvalue = wait_value;
  place.werr = wait_err;
  place.max_polls = max_polls;
  return voxel_fast(pts, B, N, copies, target, workspace, seed, nullptr, out_idx, out_pts,
                    as_stream(stream), prepped != 0, pool != 0, start_flag, start_value, place);
}

extern "C" int pcst_cfg_ddim_voxel_prep(const float* x, const float* eps, const float* source,
                                        int64_t C, int64_t N, float guidance_scale,
                                        float sqrt_1m_at, float sqrt_at_eps, float sqrt_aprev,
                                        float sqrt_1m_aprev, float* x_out, float* x_cat,
                                        void* vox_workspace, int64_t copies, uint64_t pool_seed,
                                        int pool, void* stream) {
  PCST_CHECK_ARG(C > 0 && N > 0 && copies >= 1 && C * copies < (1 << 15) && N < (1ll << 30),
                 "cfg_ddim_voxel_prep: bad shape");
  PCST_CHECK_ARG(x && eps && x_out && x_cat && vox_workspace, "cfg_ddim_voxel_prep: null pointer");
  VoxelFastWS w = carve_voxel_fast(vox_workspace, C, N, copies);
  const int nprep = vox_prep_blocks(N);
  const int sshift = vox_sel_shift(N);
  PCST_CHECK_ARG(!pool || (1 << (32 - sshift)) <= 1024, "cfg_ddim_voxel_prep: pool histogram needs N <= 4M");
  const unsigned npool = pool ? (unsigned)(kPoolBlocks * copies) : 0u;
  // the kernel's four-point path: every base 16-B aligned (then so is every cloud's and the
  // uncond half's start when N % 4 == 0)
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
#ifdef PCST_PREP_NO_VEC4  // experiment builds only (csrc/Makefile XDEF): the per-point loop
  const int vec4 = 0;
  (void)al16;
#else
  const int vec4 = (N % 4 == 0 && al16(x) && al16(eps) && al16(x_out) && al16(x_cat) &&
                    (!source || al16(source))) ? 1 : 0;
#endif
  hipLaunchKernelGGL(voxf_cfg_prep_kernel, dim3(nprep + kVoxZeroBlocks + npool, (unsigned)C), dim3(256),
                     0, as_stream(stream), x, eps, source, C, (int)N, guidance_scale, sqrt_1m_at,
                     sqrt_at_eps, sqrt_aprev, sqrt_1m_aprev, x_out, x_cat, w.pmm, nprep,
                     reinterpret_cast<uint4*>(w.cnt4),
                     (int64_t)cdiv(vox_zero_bytes(w, C * copies), 16), w.phist, pool_seed,
                     (int)copies, sshift, vec4);
  PCST_LAUNCH_CHECK("cfg_ddim_voxel_prep");
  return PCST_OK;
}

extern "C" int pcst_voxel_downsample_copies_dseed(const float* pts, int64_t B, int64_t N,
                                                  int64_t copies, int64_t target, void* workspace,
                                                  const uint64_t* seed_dev, int64_t* out_idx,
                                                  float* out_pts, void* stream) {
  PCST_CHECK_ARG(B > 0 && copies >= 1 && B * copies < (1 << 15) && N > target && target > 0 &&
                     N < (1ll << 30),
                 "voxel_downsample_copies_dseed: bad shape");
  PCST_CHECK_ARG(pts && workspace && seed_dev && out_idx && out_pts,
                 "voxel_downsample_copies_dseed: null pointer");
  return voxel_fast(pts, B, N, copies, target, workspace, 0, seed_dev, out_idx, out_pts,
                    as_stream(stream));
}

