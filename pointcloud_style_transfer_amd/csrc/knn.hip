// kNN-3 inverse-distance upsampling of HierarchicalProcessor.upsample_knn
// (models/diffusion_model.py:127-153), on the device instead of the reference's
// device->host->sklearn KD-tree->device round trip.
//
//   result[idx[j]] = coarse[j]                  (last j wins for repeated indices, as numpy)
//   other rows n:  3 nearest refs orig[idx[j]] by float64 rdist ((dx^2+dy^2)+dz^2) (the
//                  KD-tree's euclidean rdist on float64-converted coordinates), ascending,
//                  exact ties -> lower j; w = 1/(sqrt(rdist)+1e-8), w /= ((w0+w1)+w2),
//                  value = ((v0*w0 + v1*w1) + v2*w2) in float64, rounded to float32.
//
// Grid.  A uniform grid whose cell size follows the cloud's PEAK density (about kRefsPerCell
// refs per cell where the cloud is densest).  Cells are numbered brick-major: 4x4x4-cell
// bricks in row-major order, Morton order inside a brick, so consecutive cell ids form a
// compact box and a brick's refs are one contiguous range.  Refs and the unknown rows
// (queries) are counting-sorted by cell.
//
// Query pass (wave-cooperative).  One wave per chunk of <= 64 queries of one brick (the scan
// kernel cuts the chunks).  Two passes, the second over refs the first did not visit:
//   1. the cells of the chunk's cell bounding box grown by one cell;
//   2. for lanes not yet settled that hold 3 refs: the cells of the union of their balls (the
//      current 3rd distance bounds the true one, so a lane's ball holds its answer).
// A lane is settled once its 3rd-best distance is below the distance to the unscanned region.
// The refs of a pass are gathered into the wave's LDS window (x, y, z, j arrays) by LDS-DMA
// (global_load_lds, a per-lane source address: a balanced copy, each lane finds the cell of its
// slot by a binary search over the lanes' offsets) and every lane screens every staged ref: the fp32 three
// smallest distances are kept branch-free, then only refs within (1 + 2e-6) of the fp32 3rd
// best are ranked in exact float64.  Pass 2 runs under a staging budget (a wave's time is
// bounded); lanes still open after it (sparse neighbourhoods: in the bench trajectory ~0.05 %
// of the queries, which a wave-wide staging pass would serve at the cost of the kernel's tail)
// go to the outlier list: one wave per outlier query searches shells of bricks around it
// (knn_outlier_brick_kernel).
//
// Chunk scheduling (round 6).  A chunk's time is a chain of dependent loads and one or two
// staged windows (8-45 us, median ~19), and there are more chunk-waves than wave slots (6670 vs
// 4096 at the bench's two CFG rows).  With one wave per chunk a wave slot is freed only when its
// whole work-group retires, so the launch was two rounds of the slowest chunk of four.  Now the
// query grid is the resident one (4 work-groups per CU) and every wave is persistent: its first
// chunk is static (its wave index), the next ones come from a work counter of its CFG row, sharded
// over eight counters (work-group m of a row takes from counter m % 8, i.e. all its users sit on
// one XCD under round-robin placement), so a wave that finishes early takes the next chunk
// instead of idling and no counter sees more than an eighth of the dequeues (one word saturates
// at ~88 dequeues per us: MI355X_MICROARCH.md, dequeue).  The scan lists the wide chunks (runs of
// two or more occupied octants: the long ones) first, so the static first chunks are the long
// ones and the counters hand out the short ones.  The counters live in the build's zeroed
// state; the outlier launch zeroes them again for the next query on the same workspace.
//
// Launches: memset, pre (cloud stats + known rows), count (grid params, per-cell counts with
// each element's rank in its cell, per-tile sums, known-row copies), scan (single pass: tile
// offsets from the per-tile sums; the chunk list), fill (no atomics: start + rank), query,
// outlier.
#include "common.h"
#include "cloud.h"
#include "knn_rows.h"

namespace pcst {

constexpr double kRefsPerCell = 6.0;     // refs per cell at the cloud's peak density
constexpr int kCandCap = 512;            // LDS candidates per wave
constexpr int kBallCells = 512;          // largest cell box one lane's ball may ask for
constexpr int kBallUnion = 1024;         // largest union box of a ball pass
constexpr uint32_t kBallBudget = 2048;   // refs the ball pass may stage
constexpr int kPreKnownBlocks = 64;      // known-row scatter blocks per cloud in the pre kernel
constexpr int kCountPerBlock = 1024;     // elements per count-kernel block (4 per thread)
constexpr int kOvlLds = 256;             // overflow refs staged in LDS per query work-group
constexpr int kOutlierBrickBlocks = 256; // outlier workgroups per cloud (brick search, 4 queries)
constexpr int kBrickBatch = 4;           // bricks per brick-copy work item of the rows query
#ifndef PCST_KNN_WIDE_VOL                // experiment builds override (csrc/Makefile XDEF)
#define PCST_KNN_WIDE_VOL 80
#endif
constexpr int kWideBoxVol = PCST_KNN_WIDE_VOL;  // a chunk whose one-ring box holds this many cells
                                                // or more stages two rings in pass 1
constexpr int kQueryBlocksPerCU = 4;     // resident query work-groups per CU (waves_per_eu 4, 38 KiB LDS)


struct KnnWS {
  StatRec* stats;    // [B][kStatBlocks]
  float* gp;         // [B][8]: origin xyz, cell size, inv size, dims xyz (int bits)
  float4* refs;      // [B][M]   (x, y, z, j) cell-sorted
  int32_t* qorder;   // [B][N]   query row index in cell order
  int2* crank;       // [B][M+N] (cell, rank in cell); cell -1 for known rows
  uint2* chunks;     // [B][maxch] query ranges [q0, q1) of <= 64 queries inside one brick
  int32_t* olist;    // [B][N]   outlier query rows
  float* obound;     // [B][N]   their kk-th best squared distance so far (rounded up; inf: none)
  // zeroed every call (contiguous):
  int32_t* err;
  int32_t* qctr;     // [B][8][kCtrStride] the query's work counters (chunk scheduling), one per line
  int32_t* nchunk;   // [nchunk_stride(B)] chunks, then [B] u64 wide (list front) << 32 | narrow (back)
  int32_t* ocount;   // [B]
  uint32_t* known;   // [B][N]  (j+1 of the last coarse row writing n, 0 = query)
  uint64_t* tsum;    // [B][T]  per-tile sums of the packed counts
  uint64_t* cnt;     // [B][T*kKnnTile] packed counts (refs | queries << 32) -> starts
  int64_t Cmax, T, Cpad, maxch;
  size_t bytes;
};

static KnnWS carve_knn(void* base, int64_t B, int64_t N, int64_t M) {
  Carver c(base);
  KnnWS w;
  w.Cmax = knn_cells(M);
  w.T = cdiv(w.Cmax + 1, kKnnTile);
  w.Cpad = w.T * kKnnTile;
  w.maxch = cdiv(N, 64) + 8 * (w.Cmax / 64) + 1;  // <= ceil(q/64) + 8 chunks per brick
  w.stats = c.take<StatRec>(B * kStatBlocks);
  w.gp = c.take<float>(B * 8);
  w.refs = c.take<float4>(B * M);
  w.qorder = c.take<int32_t>(B * N);
  w.crank = c.take<int2>(B * (M + N));
  w.chunks = c.take<uint2>(B * w.maxch);
  w.olist = c.take<int32_t>(B * N);
  w.obound = c.take<float>(B * N);
  w.err = c.take<int32_t>(4);
  w.qctr = c.take<int32_t>(B * kQueryShards * kCtrStride);
  w.nchunk = c.take<int32_t>(3 * nchunk_stride(B));
  w.ocount = c.take<int32_t>(B);
  w.known = c.take<uint32_t>(B * N);
  w.tsum = c.take<uint64_t>(B * w.T);
  w.cnt = c.take<uint64_t>(B * w.Cpad);
  w.bytes = c.bytes();
  return w;
}

struct Grid {
  float o[3], s, inv;
  int d[3], bx, by;
  __device__ void load(const float* G) {
    o[0] = G[0]; o[1] = G[1]; o[2] = G[2];
    s = G[3]; inv = G[4];
    d[0] = __float_as_int(G[5]); d[1] = __float_as_int(G[6]); d[2] = __float_as_int(G[7]);
    bx = (d[0] + 3) >> 2;
    by = (d[1] + 3) >> 2;
    // A point's computed cell floor((p - o) * inv) can differ from its exact cell when p lies
    // within this distance of a cell face: fp32 rounding of p - o and of the product (|p - o| <=
    // (d + 1) s, 2^-24 relative each) and inv = fl(1/s) against s (2^-24 each side) give at most
    // ~(d + 1) * 2.4e-7 cells.  Every lower bound of a distance to unscanned cells subtracts it.
    slack = (double)s * (3e-7 * (double)(max(d[0], max(d[1], d[2])) + 1) + 1e-5);
  }
  double slack;
};

__device__ __forceinline__ int cell_coord(float p, float o, float inv, int d) {
  int c = (int)floorf((p - o) * inv);
  return c < 0 ? 0 : (c >= d ? d - 1 : c);
}

// brick-major cell id: bricks row-major, Morton (x0 y0 z0 x1 y1 z1) inside the brick
__device__ __forceinline__ int cell_id(int x, int y, int z, const Grid& g) {
  const int m = (x & 1) | ((y & 1) << 1) | ((z & 1) << 2) | ((x & 2) << 2) | ((y & 2) << 3) |
                ((z & 2) << 4);
  return ((((z >> 2) * g.by + (y >> 2)) * g.bx + (x >> 2)) << 6) + m;
}

__device__ __forceinline__ int cell_of(const float* p, const Grid& g) {
  return cell_id(cell_coord(p[0], g.o[0], g.inv, g.d[0]), cell_coord(p[1], g.o[1], g.inv, g.d[1]),
                 cell_coord(p[2], g.o[2], g.inv, g.d[2]), g);
}

// Cell size from the peak density of a Gaussian with the cloud's per-axis spread:
// rho_max = M / ((2 pi)^1.5 sx sy sz); s^3 = kRefsPerCell / rho_max.  Grown until the bricked
// bounding box holds at most Cmax cells (and at most 2048 per axis).  Called by one whole
// wave; lane 0 writes G.
__device__ void knn_grid_params(const StatRec* __restrict__ stats, int b, int64_t N, int64_t M,
                                int64_t Cmax, float* G) {
  const StatRec r = fold_stats_wave(stats, b);
  if ((threadIdx.x & 63) != 0) return;
  double ext[3], sig[3];
  for (int c = 0; c < 3; ++c) {
    ext[c] = (double)r.mx[c] - (double)r.mn[c];
    if (!(ext[c] > 1e-9)) ext[c] = 1e-9;
    const double mean = r.s[c] / (double)N;
    const double var = r.ss[c] / (double)N - mean * mean;
    sig[c] = sqrt(fmax(var, 0.0));
    sig[c] = fmax(sig[c], 1e-3 * ext[c]);
  }
  const double rho = (double)M / (15.7496099457 * sig[0] * sig[1] * sig[2]);
  double s = cbrt(kRefsPerCell / rho);
  int d[3];
  for (int it = 0; it < 400; ++it) {
    int64_t tot = 64;
    for (int c = 0; c < 3; ++c) {
      d[c] = (int)fmin(2048.0, fmax(1.0, ceil(ext[c] / s)));
      tot *= (d[c] + 3) >> 2;
    }
    if (tot <= Cmax) break;
    s *= 1.1;
  }
  G[0] = r.mn[0]; G[1] = r.mn[1]; G[2] = r.mn[2];
  G[3] = (float)s;
  G[4] = (float)(1.0 / s);
  G[5] = __int_as_float(d[0]); G[6] = __int_as_float(d[1]); G[7] = __int_as_float(d[2]);
}

// blocks [0, kStatBlocks): cloud statistics; the rest: known[n] = max j+1 with idx[j] == n.
// zero (rows layout, M = 0): blocks [kStatBlocks, grid) zero zero_words 16-byte words instead of
// a memset launch (the per-build state; the kernels that read it are later launches).
constexpr int kPreZeroBlocks = 128;
__global__ __launch_bounds__(256) void knn_pre_kernel(const float* __restrict__ orig,
                                                      const int64_t* __restrict__ idx, int N,
                                                      int64_t M, StatRec* __restrict__ stats,
                                                      uint32_t* __restrict__ known,
                                                      int32_t* __restrict__ err,
                                                      uint4* __restrict__ zero = nullptr,
                                                      int64_t zero_words = 0) {
  const int b = blockIdx.y;
  if (zero) {
    if ((int)blockIdx.x >= kStatBlocks) {
      const int64_t stride = (int64_t)kPreZeroBlocks * gridDim.y * 256;
      for (int64_t i = ((int64_t)b * kPreZeroBlocks + (blockIdx.x - kStatBlocks)) * 256 + threadIdx.x;
           i < zero_words; i += stride)
        zero[i] = make_uint4(0u, 0u, 0u, 0u);
      return;
    }
    cloud_stats_block(orig + (int64_t)b * N * 3, N, blockIdx.x, stats + b * kStatBlocks);
    return;
  }
  // any grid size (a capped side-stream build has few workgroups): the stats partials and the
  // known rows are strided over the workgroups
  for (int sb = blockIdx.x; sb < kStatBlocks; sb += gridDim.x) {
    cloud_stats_block(orig + (int64_t)b * N * 3, N, sb, stats + b * kStatBlocks);
    __syncthreads();  // the block helper's LDS is reused by the next partial
  }
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < M; j += (int64_t)gridDim.x * 256) {
    const int64_t n = idx[b * M + j];
    if (n < 0 || n >= N) { atomicOr(err, 1); continue; }
    atomicMax(&known[b * (int64_t)N + n], (uint32_t)(j + 1));
  }
}

// Per element e of [refs j < M | rows n = e - M]: its cell and its rank in the cell (the old
// value of the cell's packed counter), per-tile sums via an LDS histogram.  Known rows are not
// counted (known == nullptr: every row is, the rows layout's phase A with M = 0).  The grid is
// sized for Mgrid refs.  Each thread handles 4 elements with their atomics in flight together.
__global__ __launch_bounds__(256) void knn_count_kernel(
    const float* __restrict__ orig, const int64_t* __restrict__ idx,
    const StatRec* __restrict__ stats, const uint32_t* __restrict__ known, int64_t N, int64_t M,
    int64_t Mgrid, int64_t Cmax, int64_t T, int64_t Cpad, float* __restrict__ gp, uint64_t* __restrict__ cnt,
    uint64_t* __restrict__ tsum, int2* __restrict__ crank) {
  constexpr int U = kCountPerBlock / 256;
  const int b = blockIdx.y;
  __shared__ float Gs[8];
  __shared__ unsigned long long th[kKnnMaxTiles];
  // element blocks of kCountPerBlock strided over the workgroups (a capped side-stream build has
  // few); the first block's coordinates are loaded before the grid parameters are folded, so
  // their latency overlaps
  const int64_t nblk = (M + N + kCountPerBlock - 1) / kCountPerBlock;
  float px[U], py[U], pz[U];
  bool need[U];
  unsigned long long inc[U], old[U];
  auto load = [&](int64_t blk) {
    const int64_t e0 = blk * kCountPerBlock + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = e0 + u * 256;
      need[u] = false;
      inc[u] = 0ull;
      px[u] = py[u] = pz[u] = 0.0f;
      if (e < M) {
        int64_t n = idx[b * M + e];
        n = n < 0 ? 0 : (n >= N ? N - 1 : n);
        const float* p = orig + (b * N + n) * 3;
        px[u] = p[0]; py[u] = p[1]; pz[u] = p[2];
        need[u] = true;
        inc[u] = 1ull;
      } else if (e < M + N) {
        const int64_t n = e - M;
        const uint32_t kn = known ? known[b * N + n] : 0u;  // (rows layout: every row)
        if (!kn) {  // known rows take the coarse value in the outlier pass (after the MLP)
          const float* p = orig + (b * N + n) * 3;
          px[u] = p[0]; py[u] = p[1]; pz[u] = p[2];
          need[u] = true;
          inc[u] = 1ull << 32;
        }
      }
    }
  };
  load(blockIdx.x);
  if (threadIdx.x < 64) knn_grid_params(stats, b, N, Mgrid, Cmax, Gs);
  for (int t = threadIdx.x; t < T; t += 256) th[t] = 0ull;
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x < 8) gp[b * 8 + threadIdx.x] = Gs[threadIdx.x];
  Grid g;
  g.load(Gs);
  uint64_t* Cn = cnt + b * Cpad;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    if (blk != blockIdx.x) load(blk);
    const int64_t e0 = blk * kCountPerBlock + threadIdx.x;
    int cell[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float p[3] = {px[u], py[u], pz[u]};
      cell[u] = need[u] ? cell_of(p, g) : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      old[u] = cell[u] >= 0 ? atomicAdd((unsigned long long*)&Cn[cell[u]], inc[u]) : 0ull;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = e0 + u * 256;
      if (e >= M + N) continue;
      int2 cr = make_int2(-1, 0);
      if (cell[u] >= 0) {
        atomicAdd(&th[cell[u] / kKnnTile], inc[u]);
        cr = make_int2(cell[u], (int)(uint32_t)(e < M ? old[u] : old[u] >> 32));
      }
      crank[b * (M + N) + e] = cr;
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += 256)
    if (th[t]) atomicAdd((unsigned long long*)&tsum[b * T + t], th[t]);
}

__device__ __forceinline__ uint64_t block_excl_scan_256_u64(uint64_t v, unsigned long long* sh,
                                                            uint64_t& total) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint64_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint64_t wofs = 0;
  for (int q = 0; q < w; ++q) wofs += sh[q];
  total = sh[0] + sh[1] + sh[2] + sh[3];
  return wofs + x - v;
}

// Exclusive scan of the packed counts in place (the tile offset is the sum of the earlier
// tiles' sums: at most kKnnMaxTiles words, read by the whole block), then the tile's 64
// bricks are cut into chunks of <= 64 queries (by octant, below) appended to the cloud's chunk
// list (order free: chunks are independent).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void knn_scan_kernel(uint64_t* __restrict__ cnt,
                                                       const uint64_t* __restrict__ tsum,
                                                       int64_t T, int64_t Cpad,
                                                       uint2* __restrict__ chunks, int64_t maxch,
                                                       int32_t* __restrict__ nchunk) {
  const int b = blockIdx.y;
  __shared__ unsigned long long buf[kKnnTile + kKnnTile / 32];
  __shared__ unsigned long long sh[8];
  auto pad = [](int i) { return i + (i >> 5); };
  // tiles strided over the workgroups (a capped side-stream build has few)
  for (int tile = blockIdx.x; tile < (int)T; tile += gridDim.x) {
    __syncthreads();  // the previous tile's buf / sh readers are done
    uint64_t* D = cnt + b * Cpad + (int64_t)tile * kKnnTile;
    uint64_t pre = 0;
    for (int t = threadIdx.x; t < tile; t += 256) pre += tsum[b * T + t];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) pre += __shfl_xor(pre, off);
    if ((threadIdx.x & 63) == 0) sh[4 + (threadIdx.x >> 6)] = pre;
#pragma unroll
    for (int k = 0; k < 16; ++k) buf[pad(k * 256 + threadIdx.x)] = D[k * 256 + threadIdx.x];
    __syncthreads();
    const uint64_t base = sh[4] + sh[5] + sh[6] + sh[7];
    uint64_t v[16], s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      v[k] = buf[pad(threadIdx.x * 16 + k)];
      s += v[k];
    }
    uint64_t tot;
    uint64_t run = block_excl_scan_256_u64(s, sh, tot) + base;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      buf[pad(threadIdx.x * 16 + k)] = run;
      run += v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) D[k * 256 + threadIdx.x] = buf[pad(k * 256 + threadIdx.x)];
    if (threadIdx.x < 64) {
      // brick t's queries by octant (2x2x2 cells: Morton cells [8o, 8o + 8)).  A chunk is a run of
      // whole consecutive octants holding <= 64 queries, or a balanced part of one octant that
      // holds more, so a dense chunk's cell box stays within 2x2x2 cells (the query pass stages
      // the box grown by one cell: at most 4x4x4).
      const int t = threadIdx.x;
      uint32_t qo[9];
#pragma unroll
      for (int o = 0; o < 8; ++o) qo[o] = (uint32_t)(buf[pad(t * 64 + 8 * o)] >> 32);
      qo[8] = (uint32_t)((t < 63 ? buf[pad(t * 64 + 64)] : base + tot) >> 32);
      // walk the octants; emit(a, b, wide) is called for every chunk [a, b) in order, wide for a
      // run of two or more occupied octants (a sparse region: the query stages two rings and runs
      // its ball pass for almost every such chunk -- the long chunks)
      auto walk = [&](auto&& emit) {
        uint32_t cs = qo[0];  // start of the open run of octants
        int ro = 0;           // occupied octants in the run
#pragma unroll
        for (int o = 0; o < 8; ++o) {
          const uint32_t a = qo[o], n = qo[o + 1] - a;
          if (n > 64) {
            if (a > cs) emit(cs, a, ro > 1);
            const uint32_t k = (n + 63) / 64;
            for (uint32_t i = 0; i < k; ++i)
              emit(a + (uint32_t)((uint64_t)n * i / k), a + (uint32_t)((uint64_t)n * (i + 1) / k), false);
            cs = a + n;
            ro = 0;
          } else if (a + n - cs > 64) {
            emit(cs, a, ro > 1);
            cs = a;
            ro = n > 0 ? 1 : 0;
          } else {
            ro += n > 0 ? 1 : 0;
          }
        }
        if (qo[8] > cs) emit(cs, qo[8], ro > 1);
      };
      // the cloud's list holds the wide chunks from the front and the others from the back, so
      // the query's waves take the long chunks first (their first, static chunks) and the
      // second round is short ones
      uint32_t nw = 0, nn = 0;
      walk([&](uint32_t, uint32_t, bool wide) {  // (branch-free: a selected ++ put both in scratch)
        nw += wide ? 1u : 0u;
        nn += wide ? 0u : 1u;
      });
      uint32_t offw = nw, offn = nn;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t yw = __shfl_up(offw, o), yn = __shfl_up(offn, o);
        if (t >= o) {
          offw += yw;
          offn += yn;
        }
      }
      const uint32_t allw = __shfl(offw, 63), alln = __shfl(offn, 63);
      offw -= nw;
      offn -= nn;
      uint32_t atw = 0, atn = 0;
      if (t == 0 && allw + alln) {  // both lists' bases from one returning atomic (wide << 32 | narrow)
        unsigned long long* packed = reinterpret_cast<unsigned long long*>(nchunk + nchunk_stride(gridDim.y));
        const unsigned long long old = atomicAdd(packed + b, ((unsigned long long)allw << 32) | alln);
        atw = (uint32_t)(old >> 32);
        atn = (uint32_t)old;
        __hip_atomic_fetch_add(&nchunk[b], (int32_t)(allw + alln), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      atw = __shfl(atw, 0) + offw;
      atn = __shfl(atn, 0) + offn;
      uint2* Ch = chunks + b * maxch;
      walk([&](uint32_t a, uint32_t e, bool wide) {
        if (wide) Ch[atw++] = make_uint2(a, e);
        else Ch[maxch - 1 - (atn++)] = make_uint2(a, e);
      });
    }
  }  // tile
}

__global__ __launch_bounds__(256) void knn_fill_kernel(const float* __restrict__ orig,
                                                       const int64_t* __restrict__ idx, int64_t N,
                                                       int64_t M, int64_t Cpad,
                                                       const uint64_t* __restrict__ start,
                                                       const int2* __restrict__ crank,
                                                       float4* __restrict__ refs,
                                                       int32_t* __restrict__ qorder) {
  const int b = blockIdx.y;
  const uint64_t* S = start + b * Cpad;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < M + N; e += gridDim.x * 256) {
    const int2 cr = crank[b * (M + N) + e];
    if (cr.x < 0) continue;
    if (e < M) {
      int64_t n = idx[b * M + e];
      n = n < 0 ? 0 : (n >= N ? N - 1 : n);
      const float* p = orig + (b * N + n) * 3;
      const uint32_t pos = (uint32_t)S[cr.x] + (uint32_t)cr.y;
      refs[b * M + pos] = make_float4(p[0], p[1], p[2], __int_as_float((int)e));
    } else {
      const uint32_t pos = (uint32_t)(S[cr.x] >> 32) + (uint32_t)cr.y;
      qorder[b * N + pos] = (int32_t)(e - M);
    }
  }
}

// Rows layout fill: row n of cloud b at its cell-order position, as (x, y, z, n), so the query
// reads a chunk's rows with one load (no index -> position chain).
__global__ __launch_bounds__(256) void knn_rows_fill_kernel(const float* __restrict__ x, int64_t N,
                                                            int64_t Cpad, const uint64_t* __restrict__ start,
                                                            const int2* __restrict__ crank,
                                                            float4* __restrict__ xs) {
  const int b = blockIdx.y;
  const uint64_t* S = start + b * Cpad;
  for (int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x; n < N; n += gridDim.x * 256) {
    const int2 cr = crank[b * N + n];
    const float* p = x + (b * N + n) * 3;
    xs[b * N + (uint32_t)(S[cr.x] >> 32) + (uint32_t)cr.y] = make_float4(p[0], p[1], p[2], __int_as_float((int)n));
  }
}

// ---- Rows layout (the sampling loop's step: pcst_knn3_rows_build / _refs / _query) ----
// Phase A needs the clouds' positions only, so the loop runs it beside the voxel downsample
// (before the coarse indices exist): every row of cloud cl is binned (statistics, grid, per-cell
// row counts with each row's rank, the scan -- row starts and the chunk list over ALL rows --
// and the fill: rows in cell order), shared by the `copies` CFG rows b = c * C + cl of the cloud.
// Phase B (after the downsample), ONE launch: ref j of row b marks its point n known (atomicMax:
// the last j wins, as the reference's index assignment), takes a rank in n's cell (atomicAdd) and
// is stored at slot start(cell) + rank: a cell's refs are the front of the cell's own row range.
// The outlier pass scans whole bricks, so it reads a second copy in which each brick's refs are
// one run at the front of the brick's row range: the query's waves build it once they run out of
// chunks (the query's tail, where waves otherwise idle behind the last long chunks; the outlier
// launch is its only reader).  Distinct refs always fit (a cell has one row per distinct ref);
// refs repeating an index (the downsample's representatives may share one: ~200 of 30000 per row
// in the bench) fit while their cell has rows to spare, and the rest go to the row's overflow
// list, which the query and the outlier pass offer wherever their scanned box holds them.
// (Round 5 packed a brick's refs into one run with a cell-scan launch between a rank and a place
// launch: three launches on the step's critical path instead of one.)  The query skips known rows
// (copying their coarse value instead).  The grid is the compact layout's (the same statistics
// and ref count), so both layouts give the same bits.
// A flag for work on another stream: every launch ahead of this one on its stream has completed.
__global__ void knn_flag_kernel(uint32_t* flag, uint32_t value) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Phase B as its own launch (rows_place per ref; pcst_knn3_rows_refs).  The sampling step runs it
// inside the voxel emit instead (voxel.hip, the same rows_place).
// wflag (optional): the side stream's phase-A flag; every work-group waits until it holds wvalue
// (the consumer side of the guide's hand-off: one relaxed poll loop, one agent-scope acquire, a
// barrier), so no wait launch sits in front of this one; a work-group whose wait gives up sets
// *werr and writes nothing at all -- no mark, rank, slot or overflow entry (the workspace may hold
// anything then: an earlier build's state or, fresh, uninitialised memory) -- and the query and
// outlier launches, handed werr as their refs_err, leave the workspace alone and write eps = 0.
// The coarse indices are loaded before the wait (they do not depend on phase A).
__global__ __launch_bounds__(256) void knn_rows_place_kernel(
    const float* __restrict__ x, const int64_t* __restrict__ idx, const RowsPlace rp,
    int32_t* __restrict__ err, const uint32_t* __restrict__ wflag, uint32_t wvalue,
    int32_t* __restrict__ werr, int64_t max_polls) {
  const int b = blockIdx.y;
  const int64_t N = rp.N, M = rp.M, cl = b % rp.C;
  const int64_t j0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int64_t n0 = j0 < M ? idx[b * M + j0] : 0;
  if (wflag && !block_wait_flag(wflag, wvalue, werr, max_polls)) return;
  for (int64_t j = j0; j < M; j += (int64_t)gridDim.x * 256) {
    const int64_t n = j == j0 ? n0 : idx[b * M + j];
    if (n < 0 || n >= N) {
      atomicOr(err, 1);
      continue;
    }
    rows_place(rp, b, n, j, x + (cl * N + n) * 3);
  }
}

struct Top3 {
  // named fields, not arrays: a runtime index would put an array in scratch
  double d0, d1, d2;
  int j0, j1, j2;
  __device__ void init() {
    d0 = d1 = d2 = INFINITY;
    j0 = j1 = j2 = 0x7fffffff;
  }
  // kk-th best (kk in 1..3; a compile-time constant at every call site)
  __device__ __forceinline__ double last(int kk) const {
    return kk >= 3 ? d2 : (kk == 2 ? d1 : d0);
  }
  __device__ __forceinline__ void push(double dd, int jj) {
    // lexicographic (distance, j): deterministic whatever the visiting order (a ref is never
    // offered twice; the j guard would keep a repeat harmless)
    if (dd > d2 || (dd == d2 && jj >= j2)) return;
    if (jj == j0 || jj == j1) return;
    if (dd < d1 || (dd == d1 && jj < j1)) {
      d2 = d1; j2 = j1;
      if (dd < d0 || (dd == d0 && jj < j0)) {
        d1 = d0; j1 = j0;
        d0 = dd; j0 = jj;
      } else {
        d1 = dd; j1 = jj;
      }
    } else {
      d2 = dd; j2 = jj;
    }
  }
};

// IDW of the reference (float64, sequential sums), rounded to float32.  A row that found no ref
// at all (only after a timed-out wait left the workspace unplaced: every CFG row has M >= 1 refs)
// writes 0 instead of reading a value at an invalid index.
__device__ __forceinline__ void idw_write(const Top3& t, int kk, const float* __restrict__ V,
                                          float* __restrict__ O) {
  if (t.j0 == 0x7fffffff || (kk > 1 && t.j1 == 0x7fffffff) || (kk > 2 && t.j2 == 0x7fffffff)) {
    O[0] = O[1] = O[2] = 0.0f;
    return;
  }
  const double w0 = __ddiv_rn(1.0, dadd(__dsqrt_rn(t.d0), 1e-8));
  const double w1 = kk > 1 ? __ddiv_rn(1.0, dadd(__dsqrt_rn(t.d1), 1e-8)) : 0.0;
  const double w2 = kk > 2 ? __ddiv_rn(1.0, dadd(__dsqrt_rn(t.d2), 1e-8)) : 0.0;
  double wsum = w0;
  if (kk > 1) wsum = dadd(wsum, w1);
  if (kk > 2) wsum = dadd(wsum, w2);
  const double u0 = __ddiv_rn(w0, wsum), u1 = __ddiv_rn(w1, wsum), u2 = __ddiv_rn(w2, wsum);
  const float* v0 = V + (int64_t)t.j0 * 3;
  const float* v1 = V + (int64_t)(kk > 1 ? t.j1 : t.j0) * 3;
  const float* v2 = V + (int64_t)(kk > 2 ? t.j2 : t.j0) * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double acc = dmul((double)v0[c], u0);
    if (kk > 1) acc = dadd(acc, dmul((double)v1[c], u1));
    if (kk > 2) acc = dadd(acc, dmul((double)v2[c], u2));
    O[c] = (float)acc;
  }
}

__device__ __forceinline__ float dist32(float fx, float fy, float fz, float4 r) {
  const float ex = fx - r.x, ey = fy - r.y, ez = fz - r.z;
  return fmaf(ez, ez, fmaf(ey, ey, ex * ex));
}

typedef float f2 __attribute__((ext_vector_type(2)));

// dist32 on two refs at once (the same IEEE operations per component: v_pk_add/mul/fma_f32)
__device__ __forceinline__ f2 dist2(f2 qx, f2 qy, f2 qz, f2 X, f2 Y, f2 Z) {
  const f2 ex = qx - X, ey = qy - Y, ez = qz - Z;
  return __builtin_elementwise_fma(ez, ez, __builtin_elementwise_fma(ey, ey, ex * ex));
}

// A wave's LDS window of staged refs as four arrays (x, y, z, j), 16-byte aligned
struct Win {
  float* x;
  float* y;
  float* z;
  int* j;
};

// fp32 distances of refs i..i+3 of the window (i a multiple of 4): 16-byte LDS reads of each
// coordinate array, packed (v_pk_*) arithmetic, two refs per instruction
__device__ __forceinline__ void dist4(const Win& W, int i, f2 qx, f2 qy, f2 qz, f2& d01, f2& d23) {
  const float4 X = *reinterpret_cast<const float4*>(W.x + i);
  const float4 Y = *reinterpret_cast<const float4*>(W.y + i);
  const float4 Z = *reinterpret_cast<const float4*>(W.z + i);
  d01 = dist2(qx, qy, qz, f2{X.x, X.y}, f2{Y.x, Y.y}, f2{Z.x, Z.y});
  d23 = dist2(qx, qy, qz, f2{X.z, X.w}, f2{Y.z, Y.w}, f2{Z.z, Z.w});
}
__device__ __forceinline__ float dist1(const Win& W, int i, float ax, float ay, float az) {
  return dist32(ax, ay, az, make_float4(W.x[i], W.y[i], W.z[i], 0.0f));
}

// One query: an fp32 screen and the exact (float64) top-3.
//   consider(): one candidate at a time: screen against the exact 3rd best.
//   window():   a staged window of candidates in one pass of slot-keyed fp32 distances (below),
//               then float64 ranks of the few candidates that can be in the top 3.  The window
//               is four coordinate arrays so the pass uses packed fp32 math.  Every member of the
//               exact top-3 survives its window's screen: its fp32 distance is within
//               (1 + 3e-7)^2 of its float64 one, and the fp32 kk-th best bounds the float64 one
//               the same way (a ref must never reach the window twice: a repeat would shrink it).
struct Query {
  float fx, fy, fz;
  double qx, qy, qz;
  Top3 t;
  float thr;            // exact-path screen (from the float64 3rd best)
  __device__ void init(float x, float y, float z) {
    fx = x; fy = y; fz = z;
    qx = x; qy = y; qz = z;
    t.init();
    thr = INFINITY;
  }
  __device__ __forceinline__ void exact(float4 ref) {
    const double ux = dsub(qx, (double)ref.x), uy = dsub(qy, (double)ref.y),
                 uz = dsub(qz, (double)ref.z);
    t.push(dadd(dadd(dmul(ux, ux), dmul(uy, uy)), dmul(uz, uz)), __float_as_int(ref.w));
  }
  __device__ __forceinline__ void consider(float4 ref, int kk) {
    if (dist32(fx, fy, fz, ref) > thr) return;
    exact(ref);
    if (t.last(kk) != INFINITY) thr = (float)(t.last(kk) * (1.0 + 2e-6)) + 1e-30f;
  }
  // Slot-keyed window (one pass over the staged refs): each fp32 distance with its low 9
  // mantissa bits replaced by the ref's window slot (< kCandCap = 512) is a key whose order is
  // the distances' order up to 2^-14 relative; the four smallest keys are kept branch-free
  // (min / med3, on the keys as non-negative floats).  Ranked exactly: the three smallest keys'
  // refs (all three whatever kk: extra candidates are harmless).  Screen sc = min(upper(kk-th
  // key) (1 + 2e-6), thr) bounds every exact top-kk member's
  // fp32 distance (at least kk refs lie at or below the kk-th key's upper end), and every ref
  // within sc that is not among the three ranked has a key >= the fourth, so lanes whose fourth
  // key's lower end lies within sc (near-ties: ~1e-3 of the lanes) re-screen the window the
  // two-pass way.  The exact top-3 is order-independent and repeats are rejected, so the result
  // is the bit-identical one of the two-pass window.
  // The keys are compared as unsigned integers: for the non-negative distances their bit patterns
  // order as the floats do, and integer min / med3 need no NaN canonicalisation (the float forms
  // cost the screen a v_max per key under IEEE mode); the key itself is one v_and_or_b32.
  static __device__ __forceinline__ uint32_t slot_key(float d, uint32_t mask, uint32_t slot) {
    uint32_t k;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(k) : "v"(__float_as_uint(d)), "v"(mask), "s"(slot));
    return k;
  }
  static __device__ __forceinline__ uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
  }
  static __device__ __forceinline__ float key_lo(float k) { return __uint_as_float(__float_as_uint(k) & ~511u); }
  static __device__ __forceinline__ float key_hi(float k) {
    return k == INFINITY ? INFINITY : __uint_as_float(__float_as_uint(k) | 511u);
  }
  __device__ __forceinline__ void window(const Win& W, int fill, int kk) {
    const float ax = fx, ay = fy, az = fz;  // by value: keeps the query out of private memory
    const f2 qx = {ax, ax}, qy = {ay, ay}, qz = {az, az};
    const uint32_t inf = __float_as_uint(INFINITY);
    uint32_t u0 = inf, u1 = inf, u2 = inf, u3 = inf;
    uint32_t hi_mask = ~511u;
    asm volatile("" : "+v"(hi_mask));  // a VGPR operand of v_and_or_b32 (no literal in VOP3)
    auto put = [&](float d, int slot) {
      const uint32_t key = slot_key(d, hi_mask, (uint32_t)slot);
      const uint32_t n0 = min(u0, key);
      const uint32_t n1 = med3u(u0, u1, key);
      const uint32_t n2 = med3u(u1, u2, key);
      const uint32_t n3 = med3u(u2, u3, key);
      u0 = n0; u1 = n1; u2 = n2; u3 = n3;
    };
    int i = 0;
    for (; i + 4 <= fill; i += 4) {
      f2 d01, d23;
      dist4(W, i, qx, qy, qz, d01, d23);
      put(d01.x, i);
      put(d01.y, i + 1);
      put(d23.x, i + 2);
      put(d23.y, i + 3);
    }
    for (; i < fill; ++i) put(dist1(W, i, ax, ay, az), i);
    const float k0 = __uint_as_float(u0), k1 = __uint_as_float(u1), k2 = __uint_as_float(u2),
                k3 = __uint_as_float(u3);
    const float ck = kk >= 3 ? k2 : (kk == 2 ? k1 : k0);
    const float sc = fminf(key_hi(ck) * 1.000002f + 1e-30f, thr);
    const bool again = k3 != INFINITY && key_lo(k3) <= sc;
    auto rank = [&](float k) {
      if (k == INFINITY) return;
      const int s = (int)(__float_as_uint(k) & 511u);
      exact(make_float4(W.x[s], W.y[s], W.z[s], __int_as_float(W.j[s])));
    };
    rank(k0);
    rank(k1);
    rank(k2);
    if (__any(again)) rescreen(W, fill, again ? sc : -1.0f);
    if (t.last(kk) != INFINITY) thr = fminf(thr, (float)(t.last(kk) * (1.0 + 2e-6)) + 1e-30f);
  }
  // the two-pass window's second pass for the lanes that need it (sc < 0: none)
  __device__ __forceinline__ void rescreen(const Win& W, int fill, float sc) {
    const float ax = fx, ay = fy, az = fz;
    const f2 qx = {ax, ax}, qy = {ay, ay}, qz = {az, az};
    for (int b0 = 0; b0 < fill; b0 += 64) {
      const int nb = min(64, fill - b0);
      uint64_t m = 0;
      int u = 0;
      for (; u + 4 <= nb; u += 4) {
        f2 d01, d23;
        dist4(W, b0 + u, qx, qy, qz, d01, d23);
        m |= ((uint64_t)(d01.x <= sc) | ((uint64_t)(d01.y <= sc) << 1) |
              ((uint64_t)(d23.x <= sc) << 2) | ((uint64_t)(d23.y <= sc) << 3)) << u;
      }
      for (; u < nb; ++u) m |= (uint64_t)(dist1(W, b0 + u, ax, ay, az) <= sc) << u;
      while (m) {
        const int k = b0 + __builtin_ctzll(m);
        m &= m - 1;
        exact(make_float4(W.x[k], W.y[k], W.z[k], __int_as_float(W.j[k])));
      }
    }
  }
};

// LDS reads/writes of this wave done (before the window is overwritten or read)
__device__ __forceinline__ void lds_order() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// the window's LDS-DMA gathers landed (global_load_lds retires through vmcnt)
__device__ __forceinline__ void dma_landed() {
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
}

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = min(v, __shfl_xor(v, off));
  return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = max(v, __shfl_xor(v, off));
  return v;
}

struct Box {
  int x0, x1, y0, y1, z0, z1;
  __device__ bool has(int x, int y, int z) const {
    return x >= x0 && x <= x1 && y >= y0 && y <= y1 && z >= z0 && z <= z1;
  }
  __device__ int volume() const { return (x1 - x0 + 1) * (y1 - y0 + 1) * (z1 - z0 + 1); }
};

// Wave-cooperative scan of the refs of every cell of box `bx` that is not in `prev`: each lane
// takes one cell per round (its ref range is contiguous; the next round's ranges are loaded
// while this round's refs are staged), the round's refs are gathered into the wave's LDS
// window by LDS-DMA (each lane finds the cell of its slot by a binary search over the lanes'
// offsets) and every lane screens every staged ref.
// Returns false (abandoned: the open lanes then go to the outlier pass, never to another
// pass) once more than `budget` refs would be staged; otherwise charges them to `budget`.
// The staging loop over `vol` units; unit(li, lo, hi) gives the packed start words bounding
// unit li's contiguous ref range (lo == hi: nothing to scan).
template <class Unit>
__device__ __forceinline__ bool scan_units(int vol, const Unit& unit, const float4* __restrict__ R,
                                           const Win& W, Query& me, int kk, uint32_t& budget) {
  const int lane = threadIdx.x & 63;
  uint64_t nlo, nhi;
  unit(lane, nlo, nhi);
  int fill = 0;
  uint32_t staged = 0;
  for (int c0 = 0; c0 < vol; c0 += 64) {
    const uint32_t a = (uint32_t)nlo, cnt = (uint32_t)nhi - a;
    if (c0 + 64 < vol) unit(c0 + 64 + lane, nlo, nhi);
    uint32_t off = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(off, o);
      if (lane >= o) off += y;
    }
    const uint32_t tot = __shfl(off, 63);
    off -= cnt;
    staged += tot;
    if (staged > budget) return false;
    for (uint32_t w0 = 0; w0 < tot;) {
      const uint32_t len = min(tot - w0, (uint32_t)(kCandCap - fill));
      for (uint32_t t0 = 0; t0 < len; t0 += 64) {  // wave-uniform: every lane shuffles
        const uint32_t t = t0 + lane, v = w0 + t;
        int l = 0;  // last lane whose offset <= v (it owns slot v: zero-count lanes never do)
#pragma unroll
        for (int st = 32; st >= 1; st >>= 1)
          if (__shfl(off, l + st) <= v) l += st;
        const uint32_t src = __shfl(a, l) + (v - __shfl(off, l));
        // LDS destination = wave-uniform base + 4 * lane: slot fill + t0 + lane of each array
        if (t < len) {
          const float* g = reinterpret_cast<const float*>(R + src);
          __builtin_amdgcn_global_load_lds(g + 0, (__attribute__((address_space(3))) void*)(W.x + fill + t0), 4, 0, 0);
          __builtin_amdgcn_global_load_lds(g + 1, (__attribute__((address_space(3))) void*)(W.y + fill + t0), 4, 0, 0);
          __builtin_amdgcn_global_load_lds(g + 2, (__attribute__((address_space(3))) void*)(W.z + fill + t0), 4, 0, 0);
          __builtin_amdgcn_global_load_lds(g + 3, (__attribute__((address_space(3))) void*)(W.j + fill + t0), 4, 0, 0);
        }
      }
      fill += (int)len;
      w0 += len;
      if (fill == kCandCap) {
        dma_landed();
        me.window(W, fill, kk);
        lds_order();
        fill = 0;
      }
    }
  }
  dma_landed();
  me.window(W, fill, kk);
  lds_order();
  budget -= staged;
  return true;
}

// One query per wave: the units' refs are split over the lanes (slot v of the round's
// concatenated ranges goes to lane v % 64, found by the same binary search over the lanes'
// offsets), loaded straight into registers four slots at a time and offered to the lane's own
// top-3 (Query::consider: fp32 screen against the lane's exact 3rd best, then float64).
template <class Unit>
__device__ __forceinline__ void scan_units_1q(int vol, const Unit& unit, const float4* __restrict__ R,
                                              Query& me, int kk, uint32_t& staged) {
  const int lane = threadIdx.x & 63;
  uint64_t nlo, nhi;
  unit(lane, nlo, nhi);
  for (int c0 = 0; c0 < vol; c0 += 64) {
    const uint32_t a = (uint32_t)nlo, cnt = (uint32_t)nhi - a;
    if (c0 + 64 < vol) unit(c0 + 64 + lane, nlo, nhi);
    uint32_t off = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(off, o);
      if (lane >= o) off += y;
    }
    const uint32_t tot = __shfl(off, 63);
    off -= cnt;
    staged += tot;
    for (uint32_t t0 = 0; t0 < tot; t0 += 256) {
      float4 r[4];
      bool ok[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t v = t0 + 64 * k + lane;
        int l = 0;  // last lane whose offset <= v
#pragma unroll
        for (int st = 32; st >= 1; st >>= 1)
          if (__shfl(off, l + st) <= v) l += st;
        const uint32_t src = __shfl(a, l) + (v - __shfl(off, l));
        ok[k] = v < tot;
        if (ok[k]) r[k] = R[src];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)  // (j < 0: an empty slot of the rows layout's brick range)
        if (ok[k] && __float_as_int(r[k].w) >= 0) me.consider(r[k], kk);
    }
  }
}

// rng(u0, lo, hi): the ref range [lo, hi) of cell u0 (in the low 32 bits of each word)
template <class Rng>
__device__ __forceinline__ bool scan_box(const Box& bx, const Box& prev, const Grid& g, const Rng& rng,
                                         const float4* __restrict__ R, const Win& W, Query& me,
                                         int kk, uint32_t& budget) {
  const int nx = bx.x1 - bx.x0 + 1, ny = bx.y1 - bx.y0 + 1;
  const int vol = bx.volume();
  const float rnx = 1.0f / nx, rnxy = 1.0f / (nx * ny);  // exact quotients for li < 2^20
  // ref range of cell li (empty if outside bx or inside prev)
  auto unit = [&](int li, uint64_t& lo, uint64_t& hi) {
    lo = hi = 0;
    if (li < vol) {
      const int qz = (int)(((float)li + 0.5f) * rnxy), rz = li - qz * nx * ny;
      const int qy = (int)(((float)rz + 0.5f) * rnx), qx = rz - qy * nx;
      const int x = bx.x0 + qx, y = bx.y0 + qy, z = bx.z0 + qz;
      if (!prev.has(x, y, z)) rng(cell_id(x, y, z, g), lo, hi);
    }
  };
  return scan_units(vol, unit, R, W, me, kk, budget);
}

// Distance from q to the region outside the box of cells [x0,x1]x[y0,y1]x[z0,z1] (faces on
// the grid boundary excluded: nothing lies beyond them), less the cell-rounding slack.
__device__ __forceinline__ double outside_bound(const Query& me, const Box& c, const Grid& g) {
  const double ox = g.o[0], oy = g.o[1], oz = g.o[2], s = g.s;
  double bound = INFINITY;
  if (c.x0 > 0) bound = fmin(bound, me.qx - (ox + c.x0 * s));
  if (c.x1 + 1 < g.d[0]) bound = fmin(bound, (ox + (c.x1 + 1) * s) - me.qx);
  if (c.y0 > 0) bound = fmin(bound, me.qy - (oy + c.y0 * s));
  if (c.y1 + 1 < g.d[1]) bound = fmin(bound, (oy + (c.y1 + 1) * s) - me.qy);
  if (c.z0 > 0) bound = fmin(bound, me.qz - (oz + c.z0 * s));
  if (c.z1 + 1 < g.d[2]) bound = fmin(bound, (oz + (c.z1 + 1) * s) - me.qz);
  return bound - g.slack;  // covers fp32 cell-assignment rounding
}

__device__ __forceinline__ bool settled(const Query& me, const Box& cells, const Grid& g, int kk) {
  if (me.t.last(kk) == INFINITY) return false;
  const double bound = outside_bound(me, cells, g);
  return bound == INFINITY || (bound > 0 && me.t.last(kk) < bound * bound);
}

// amdgpu_waves_per_eu(4): 128 VGPRs (4 spilled) instead of 138, so 4 waves per SIMD (the LDS
// allows 4 work-groups per CU) instead of 3: the ~5000 chunks of a step run in fewer rounds
// (driver window 2379-2398 -> 2400-2429 steps/s, A/B on one box).
// The layout-specific arrays of the query and outlier launches.  Compact layout (pcst_knn3_build):
// per CFG row b, refs cell-sorted in [0, M), the packed start words give a cell's ref range.
// Rows layout (pcst_knn3_rows_*): the cloud cl = b % C holds the grid, the rows in cell order and
// the chunks; row b's refs sit at the front of their cell's row range (count rcnt[b][cell]), the
// known rows are skipped by the query (their value is the coarse one, copied there) and the
// overflow refs (repeated indices) are offered to every query.
struct KArgs {
  int64_t C;                  // clouds holding the grid / rows / chunks (compact: B)
  const uint32_t* known;      // [B][N] by cell-order position (rows layout)
  const float4* xs;           // [C][N] the rows in cell order (rows layout)
  const uint32_t* rcnt;       // [B][Cpad] refs placed per cell (rows layout)
  const float4* over;         // [B][M] overflow refs (rows layout)
  const int32_t* ovn;         // [B] their counts (rows layout)
  int32_t* err;               // bit 4: a chunk outside [0, N], bit 8: a ref range outside the refs
                              // (bit 1: a bad coarse index, bit 16: a brick over-full -- phase B)
  const int32_t* refs_err;    // rows layout: phase B's wait error word (nonzero: nothing placed)
  int32_t* qctr;              // [B][kQueryShards][kCtrStride] chunk counters (zero at launch);
                              // rows layout: [B..2B) the brick-batch counters
  float4* brefs;              // [B][N] rows layout: the placed refs per brick (outlier pass)
  uint32_t* bcnt;             // [B][Cpad / 64] their counts (zero unless written)
};

// The consumer side of the build -> query dependency (the `built_flag` / `built_value` of
// pcst_knn3_query / _rows_query): the workspace is read only once the build's flag holds its
// value.  The stream waited for the flag before this launch (pcst_signal_wait, or the MLP's last
// work-group); a wait that gave up lets the launch run anyway, and then every work-group finds
// the flag short -- or, rows layout, phase B's wait error word set (then the workspace holds no
// placement of this step) -- and leaves the workspace alone (its rows of the output get 0)
// instead of reading a half-built one.  The caller raises on the waits' error words after the
// loop.
__device__ __forceinline__ bool query_pending(const uint32_t* flag, uint32_t value,
                                             const int32_t* refs_err) {
  __shared__ int s_pending;
  if (threadIdx.x == 0)
    s_pending = (flag != nullptr &&
                 __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < value) ||
                (refs_err != nullptr &&
                 __hip_atomic_load(refs_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0);
  __syncthreads();
  return s_pending != 0;
}

// Persistent chunk waves (header comment, "Chunk scheduling"): the grid is G = B * Gr
// work-groups, row b = blockIdx.x % B, m = blockIdx.x / B its work-group index in the row.  Wave
// (m, wv) takes chunk m * 4 + wv first, then chunks Wr + s + S * k (Wr = 4 Gr waves per row,
// S = min(8, Gr) shards, s = m % S, k from counter s of the row) until the row's list ends.  The
// counters' item sets are disjoint and together cover [Wr, nch), and every shard of every row has
// work-groups (Gr >= S), so every chunk is processed exactly once whatever the residency.
template <int kk, bool ROWS>  // kk = min(M, 3), a compile-time constant so the top-3 stays in registers
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void knn_query_kernel(
    const float* __restrict__ orig, const float* __restrict__ vals, int64_t B, int64_t N, int64_t M,
    int64_t Cpad, const float* __restrict__ gp, const uint64_t* __restrict__ start,
    const float4* __restrict__ refs, const int32_t* __restrict__ qorder,
    const uint2* __restrict__ chunks, int64_t maxch, const int32_t* __restrict__ nchunk,
    int32_t* __restrict__ olist, float* __restrict__ obound, int32_t* __restrict__ ocount,
    float* __restrict__ out, const uint32_t* __restrict__ bflag, uint32_t bvalue, const KArgs ka) {
  __shared__ __attribute__((aligned(16))) float cand[4][4][kCandCap];
  const unsigned Gr = gridDim.x / (unsigned)B;
  const int b = (int)(blockIdx.x % (unsigned)B);
  const unsigned m = blockIdx.x / (unsigned)B;
  if (m >= Gr) return;  // (the host launches a multiple of B)
  const int64_t cl = ROWS ? b % ka.C : b;
  // the stream waited for the build's flag before this launch (a wait launch, or the MLP's last
  // work-group), so the work-groups only check it: no wait here (the resident grid fills every
  // CU's LDS, so a waiting query could hold the CUs its producer needs) and no acquire fence per
  // work-group, which at 4 work-groups per CU cost the step ~11 us (r05/s2r)
  const bool pending = query_pending(bflag, bvalue, ROWS ? ka.refs_err : nullptr);
  if (pending) {
    for (int64_t n = (int64_t)m * 256 + threadIdx.x; n < N * 3; n += (int64_t)Gr * 256)
      out[b * N * 3 + n] = 0.0f;
    return;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  Grid g;
  g.load(gp + cl * 8);
  const uint64_t* S = start + cl * Cpad;
  const float4* R = refs + b * (ROWS ? N : M);
  const float* V = vals + b * M * 3;
  const uint32_t* RC = ROWS ? ka.rcnt + b * Cpad : nullptr;
  const uint32_t rlim = (uint32_t)(ROWS ? N : M);
  // the ref range of cell u0, checked against the ref array (a bad build raises, never faults)
  auto rng = [&](int u0, uint64_t& lo, uint64_t& hi) {
    uint32_t a, e;
    if constexpr (ROWS) {  // the refs at the front of the cell's row range
      a = (uint32_t)(S[u0] >> 32);
      const uint32_t rows = (uint32_t)(S[u0 + 1] >> 32) - a;
      e = a + min(RC[u0], rows);
    } else {
      a = (uint32_t)S[u0];
      e = (uint32_t)S[u0 + 1];
    }
    if (e < a || e > rlim) {
      atomicOr(ka.err, 8);
      a = e = 0;
    }
    lo = a;
    hi = e;
  };
  const Win W = {cand[wv][0], cand[wv][1], cand[wv][2], reinterpret_cast<int*>(cand[wv][3])};
  const Box none = {1, 0, 1, 0, 1, 0};
  const int nch = nchunk[cl];  // the scan kernel's counts: total, and the wide list's length
  const int nwide = (int)(reinterpret_cast<const uint64_t*>(nchunk + nchunk_stride(ka.C))[cl] >> 32);
  // the row's overflow refs (rows layout; a few dozen in the bench), staged once per work-group
  // with their cell coordinates: a pass offers a query only those inside the box it scanned (the
  // settled test covers every ref outside it, as for the cell-placed refs)
  __shared__ float4 ovl[ROWS ? kOvlLds : 1];
  __shared__ uint64_t ovc[ROWS ? kOvlLds : 1];
  const int novr = ROWS ? ka.ovn[b] : 0;
  auto ov_cell = [&](float4 r) {  // cell coordinates x | y << 16 | z << 32 (each < 2048)
    return (uint64_t)cell_coord(r.x, g.o[0], g.inv, g.d[0]) |
           ((uint64_t)cell_coord(r.y, g.o[1], g.inv, g.d[1]) << 16) |
           ((uint64_t)cell_coord(r.z, g.o[2], g.inv, g.d[2]) << 32);
  };
  if constexpr (ROWS) {
    for (int i = threadIdx.x; i < min(novr, kOvlLds); i += 256) {
      const float4 r = ka.over[b * M + i];
      ovl[i] = r;
      ovc[i] = ov_cell(r);
    }
    __syncthreads();
  }
  // offer every overflow ref whose cell lies in bx but not in prev (wave-uniform)
  auto offer_overflow = [&](const Box& bx, const Box& prev, Query& me) {
    for (int o0 = 0; o0 < novr; o0 += 64) {
      const int i = o0 + lane;
      float4 r = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      uint64_t c = 0;
      if (i < novr) {
        if (i < kOvlLds) {
          r = ovl[i];
          c = ovc[i];
        } else {
          r = ka.over[b * M + i];
          c = ov_cell(r);
        }
      }
      const int x = (int)(c & 0xffffu), y = (int)((c >> 16) & 0xffffu), z = (int)(c >> 32);
      uint64_t in = __ballot(i < novr && bx.has(x, y, z) && !prev.has(x, y, z));
      while (in) {
        const int k = __builtin_ctzll(in);
        in &= in - 1;
        float4 rk;
        rk.x = __shfl(r.x, k); rk.y = __shfl(r.y, k); rk.z = __shfl(r.z, k); rk.w = __shfl(r.w, k);
        me.consider(rk, kk);
      }
    }
  };
  const unsigned Sh = min((unsigned)kQueryShards, Gr), sh = m % Sh;
  const int Wr = (int)Gr * 4;
  int32_t* ctr = ka.qctr + (b * kQueryShards + sh) * kCtrStride;
  // the wave's next chunk from its row's counter (taken as late as the chunk allows: once its
  // passes are done, so the counter's latency hides under the result writes and no chunk waits
  // behind a long one)
  auto take = [&]() {
    int nk = 0;
    if (lane == 0) nk = atomicAdd(ctr, 1);
    return Wr + (int)sh + (int)Sh * __shfl(nk, 0);
  };
#ifdef PCST_KNN_CHUNK_TRACE  // experiment builds only: per chunk (start, end, wave, pass-1 open
  // lanes | pass-2 ran << 8 | outliers << 16) in 10 ns ticks, in the row's obound array past 4096
  uint4* trace = reinterpret_cast<uint4*>(obound + b * N + 4096);
  const uint32_t gw = blockIdx.x * 4 + wv;
  uint32_t tr0 = 0, tr_open1 = 0, tr_p2 = 0;
  int tr_vol = 0;
#endif
  for (int item = (int)m * 4 + wv; item < nch;) {
#ifdef PCST_KNN_CHUNK_TRACE
    tr0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    tr_open1 = tr_p2 = 0;
#endif
    const uint2 ch = chunks[cl * maxch + (item < nwide ? item : maxch - 1 - (item - nwide))];
    if (ch.x > ch.y || ch.y > (uint32_t)N || ch.y - ch.x > 64u) {  // wave-uniform
      if (lane == 0) atomicOr(ka.err, 4);
      item = take();
      continue;
    }
    bool valid = ch.x + lane < ch.y;
    const uint32_t pos = valid ? ch.x + lane : ch.x;
    int64_t n;
    float qx, qy, qz;
    if constexpr (ROWS) {  // the row and its known mark by cell-order position, loaded together
      const float4 q = ka.xs[cl * N + pos];
      const uint32_t kn = valid ? ka.known[b * N + pos] : 0u;
      n = __float_as_int(q.w);
      qx = q.x; qy = q.y; qz = q.z;
      if (kn) {  // a known row takes its coarse value (the last coarse row naming it)
        const float* v = V + (int64_t)(kn - 1) * 3;
        float* o = out + (b * N + n) * 3;
        o[0] = v[0]; o[1] = v[1]; o[2] = v[2];
        valid = false;
      }
      if (!__any(valid)) {
        item = take();
        continue;
      }
    } else {
      n = qorder[cl * N + pos];
      const float* qp = orig + (cl * N + n) * 3;
      qx = qp[0]; qy = qp[1]; qz = qp[2];
    }
    Query me;
    me.init(qx, qy, qz);
    const int cx = cell_coord(me.fx, g.o[0], g.inv, g.d[0]);
    const int cy = cell_coord(me.fy, g.o[1], g.inv, g.d[1]);
    const int cz = cell_coord(me.fz, g.o[2], g.inv, g.d[2]);
    const int lx = wave_min(cx), hx = wave_max(cx), ly = wave_min(cy), hy = wave_max(cy),
              lz = wave_min(cz), hz = wave_max(cz);
    // 1. the chunk's cell box grown by one cell -- by two when the chunk spans more than an octant
    // (a sparse region: there pass 1 with one ring settles almost no lane and pass 2 ran in 90-96 %
    // of such chunks, each pass a full chain of dependent loads; tools/knn_chunk_trace.py, r6n)
    const int gr = (hx - lx + 3) * (hy - ly + 3) * (hz - lz + 3) >= kWideBoxVol ? 2 : 1;
    Box pb = {max(lx - gr, 0), min(hx + gr, g.d[0] - 1), max(ly - gr, 0), min(hy + gr, g.d[1] - 1),
              max(lz - gr, 0), min(hz + gr, g.d[2] - 1)};
    uint32_t unlimited = 0xffffffffu;
    scan_box(pb, none, g, rng, R, W, me, kk, unlimited);
    if constexpr (ROWS) offer_overflow(pb, none, me);
    bool open = valid && !settled(me, pb, g, kk);
    bool ok = true;
#ifdef PCST_KNN_CHUNK_TRACE
    tr_open1 = (uint32_t)__popcll(__ballot(open));
    tr_vol = pb.volume();
#endif
    // 2. the balls of the open lanes that hold kk refs
    if (__any(open)) {
      const double dk = me.t.last(kk);
      bool ball = open && dk != INFINITY;
      int bx0 = 0x7fffffff, bx1 = -1, by0 = 0x7fffffff, by1 = -1, bz0 = 0x7fffffff, bz1 = -1;
      if (ball) {
        const float r = (float)(sqrt(dk) * (1.0 + 1e-5) + 2.0 * g.slack);
        const Box lb = {cell_coord(me.fx - r, g.o[0], g.inv, g.d[0]),
                        cell_coord(me.fx + r, g.o[0], g.inv, g.d[0]),
                        cell_coord(me.fy - r, g.o[1], g.inv, g.d[1]),
                        cell_coord(me.fy + r, g.o[1], g.inv, g.d[1]),
                        cell_coord(me.fz - r, g.o[2], g.inv, g.d[2]),
                        cell_coord(me.fz + r, g.o[2], g.inv, g.d[2])};
        if (lb.volume() <= kBallCells) {
          bx0 = lb.x0; bx1 = lb.x1; by0 = lb.y0; by1 = lb.y1; bz0 = lb.z0; bz1 = lb.z1;
        } else {
          ball = false;
        }
      }
      if (__any(ball)) {
        const Box bb = {min(pb.x0, wave_min(bx0)), max(pb.x1, wave_max(bx1)),
                        min(pb.y0, wave_min(by0)), max(pb.y1, wave_max(by1)),
                        min(pb.z0, wave_min(bz0)), max(pb.z1, wave_max(bz1))};
        if (bb.volume() <= kBallUnion) {
#ifdef PCST_KNN_CHUNK_TRACE
          tr_p2 = 1;
#endif
          uint32_t budget = kBallBudget;
          ok = scan_box(bb, pb, g, rng, R, W, me, kk, budget);
          if constexpr (ROWS) {
            if (ok) offer_overflow(bb, pb, me);
          }
          if (ok) {
            pb = bb;
            open = open && !settled(me, pb, g, kk);
          }
        }
      }
    }
    const int next = take();
    // the rest (sparse neighbourhoods, ball too large, budget exceeded): the outlier pass
    const uint64_t rest = __ballot(open);
    if (rest) {
      int at = 0;
      if (lane == 0) at = atomicAdd(&ocount[b], (int)__popcll(rest));
      at = __shfl(at, 0);
      if (open) {
        const int64_t o = b * N + at + (int)__popcll(rest & lanemask_lt());
        olist[o] = (int32_t)n;
        const double dk = me.t.last(kk);  // exact, from refs already seen: >= the true kk-th
        obound[o] = dk == INFINITY ? INFINITY : (float)(dk * (1.0 + 1e-6)) * 1.000001f;
      }
    }
    if (valid && !open) idw_write(me.t, kk, V, out + (b * N + n) * 3);
#ifdef PCST_KNN_CHUNK_TRACE
    if (lane == 0 && item < 16384)
      trace[item] = make_uint4(tr0, (uint32_t)__builtin_amdgcn_s_memrealtime(),
                               gw | ((uint32_t)__popcll(rest) << 16),
                               min(tr_open1, 127u) | (tr_p2 << 7) | ((ch.y - ch.x) << 8) |
                                   ((uint32_t)min(tr_vol, 65535) << 16));
#endif
    item = next;
  }
  // Rows layout: the brick copy of the placed refs for the outlier launch, by waves out of chunks.
  // Batches of kBrickBatch bricks from the row's brick-batch counters (sharded as the chunks);
  // per brick, lane = cell: the cells' placed counts, their prefix, then the brick's refs copied
  // to the front of its row range (slot v of the run: the lane whose prefix holds v, found by a
  // binary search over the lanes' offsets).  A brick without refs writes nothing (its count
  // stays the build's zero).
  if constexpr (ROWS) {
    const int64_t nbr = Cpad / 64;
    const int64_t nbatch = (nbr + kBrickBatch - 1) / kBrickBatch;
    int32_t* bctr = ka.qctr + ((B + b) * kQueryShards + sh) * kCtrStride;
    const float4* Rc = refs + b * N;
    float4* Rb = ka.brefs + b * N;
    for (;;) {
      int k = 0;
      if (lane == 0) k = atomicAdd(bctr, 1);
      const int64_t gb = (int64_t)sh + (int64_t)Sh * __shfl(k, 0);
      if (gb >= nbatch) break;
      uint32_t ca[kBrickBatch], cn[kBrickBatch];
#pragma unroll
      for (int i = 0; i < kBrickBatch; ++i) {  // every brick's loads in flight together
        const int64_t c = (gb * kBrickBatch + i) * 64 + lane;
        ca[i] = cn[i] = 0;
        if (c < Cpad) {
          ca[i] = (uint32_t)(S[c] >> 32);
          const uint32_t e = c + 1 < Cpad ? (uint32_t)(S[c + 1] >> 32) : ca[i];
          if (e < ca[i] || e > rlim) {  // a bad build: skipped and reported, never read
            atomicOr(ka.err, 8);
            ca[i] = 0;
          } else {
            cn[i] = min(RC[c], e - ca[i]);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < kBrickBatch; ++i) {
        uint32_t off = cn[i];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = __shfl_up(off, o);
          if (lane >= o) off += y;
        }
        const uint32_t tot = __shfl(off, 63);
        off -= cn[i];
        if (tot == 0) continue;  // wave-uniform
        const int64_t brick = gb * kBrickBatch + i;
        const uint32_t ba = __shfl(ca[i], 0);
        if (tot > rlim - ba) {  // more refs than the brick's rows: impossible for a sound build
          if (lane == 0) atomicOr(ka.err, 16);
          continue;
        }
        if (lane == 0) ka.bcnt[b * nbr + brick] = tot;
        for (uint32_t t0 = 0; t0 < tot; t0 += 64) {
          const uint32_t v = t0 + lane;
          int l = 0;  // last lane whose offset <= v (it owns slot v: zero-count lanes never do)
#pragma unroll
          for (int st = 32; st >= 1; st >>= 1)
            if (__shfl(off, l + st) <= v) l += st;
          const uint32_t src = __shfl(ca[i], l) + (v - __shfl(off, l));
          if (v < tot) Rb[ba + v] = Rc[src];
        }
      }
    }
  }
}

// butterfly merge of the lanes' top-3 lists (lanes differing in bits below 2*top): every lane
// ends with the merged list; lexicographic (d, j) keeps it deterministic
__device__ __forceinline__ void wave_merge_top3(Top3& t, int top = 32) {
  for (int off = top; off >= 1; off >>= 1) {
    const double e0 = __shfl_xor(t.d0, off), e1 = __shfl_xor(t.d1, off), e2 = __shfl_xor(t.d2, off);
    const int i0 = __shfl_xor(t.j0, off), i1 = __shfl_xor(t.j1, off), i2 = __shfl_xor(t.j2, off);
    t.push(e0, i0);
    t.push(e1, i1);
    t.push(e2, i2);
  }
}

// Brick-shell search of the outlier queries: one wave per query.  Bricks (4x4x4 cells) are the
// grid's coarse level for free: a brick's refs are one contiguous range of the cell-sorted refs,
// [start(64 id), start(64 id + 64)).  The wave scans the box of bricks within Chebyshev brick
// distance R of the query's brick, each step only the new shell, skipping every brick whose box
// lies farther than the current 3rd-best distance; it stops once that distance is below the
// distance to everything outside the scanned box (outside_bound, the query pass's settled test)
// or the box covers the grid.  R grows by one until kk refs are known, then jumps to the radius
// whose box faces lie beyond the kk-th distance (normally the last shell).  The float64 top-3 is
// the exhaustive one: every ref not scanned is provably farther than the 3rd best (brick lower
// bounds carry the same cell-rounding slack).  A shell's refs are split over the lanes
// (scan_units_1q); after every shell the lanes' lists are merged into lane 0 (the others restart
// empty with the merged screen), so no ref is offered twice.
// Rows layout (ROWS): a brick's placed refs are one run at the front of its row range in the
// brick copy (brefs); the overflow refs are offered first; the known rows were copied by the
// query.
// The launch also zeroes the query's work counters (the query before it on the stream is done
// with them), so the next query on the workspace starts from zero as after a build.
template <int kk, bool ROWS>
__global__ __launch_bounds__(256) void knn_outlier_brick_kernel(
    const float* __restrict__ vals, int64_t N, int64_t M, const float* __restrict__ orig,
    const float* __restrict__ gp, int64_t Cpad, const uint64_t* __restrict__ start,
    const float4* __restrict__ refs, const int32_t* __restrict__ olist,
    const float* __restrict__ obound, const int32_t* __restrict__ ocount,
    const uint32_t* __restrict__ known, float* __restrict__ out,
    const uint32_t* __restrict__ bflag, uint32_t bvalue, const KArgs ka) {
  const int b = blockIdx.y;
  const int64_t cl = ROWS ? b % ka.C : b;
  if (blockIdx.x == 0 && threadIdx.x < kQueryShards) {
    ka.qctr[(b * kQueryShards + threadIdx.x) * kCtrStride] = 0;
    if (ROWS) ka.qctr[((gridDim.y + b) * kQueryShards + threadIdx.x) * kCtrStride] = 0;
  }
  if (query_pending(bflag, bvalue, ROWS ? ka.refs_err : nullptr)) return;
  // rows that are coarse points take the coarse value (result[idx] = coarse; the last coarse
  // row writing a point wins, as in the reference's index assignment); the rows layout's query
  // copied them already
  for (int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x; !ROWS && n < N;
       n += (int64_t)gridDim.x * 256) {
    const uint32_t kn = known[b * N + n];
    if (kn) {
      const float* v = vals + (b * M + (int64_t)(kn - 1)) * 3;
      float* o = out + (b * N + n) * 3;
      o[0] = v[0]; o[1] = v[1]; o[2] = v[2];
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  Grid g;
  g.load(gp + cl * 8);
  const int nbx = g.bx, nby = g.by, nbz = (g.d[2] + 3) >> 2;
  const uint64_t* S = start + cl * Cpad;
  const float4* R = ROWS ? ka.brefs + b * N : refs + b * M;
  const uint32_t* BC = ROWS ? ka.bcnt + b * (Cpad / 64) : nullptr;
  const float* V = vals + b * M * 3;
  const int cnt = ocount[b];
  const int novr = ROWS ? ka.ovn[b] : 0;
  const uint32_t rlim = (uint32_t)(ROWS ? N : M);
  const double bs = 4.0 * (double)g.s;  // brick edge
  for (int q = blockIdx.x * 4 + wv; q < cnt; q += gridDim.x * 4) {
#ifdef PCST_KNN_OUTLIER_TRACE  // experiment builds only: per outlier query (start, end, shells |
    // initial bound infinite << 15 | final radius << 16, staged refs) in 10 ns ticks, in the row's
    // obound array past 80000
    const uint32_t tr0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    uint32_t tr_shells = 0, tr_staged = 0;
#endif
    const int64_t n = olist[b * N + q];
    const float* qp = orig + (cl * N + n) * 3;
    Query me;
    me.init(qp[0], qp[1], qp[2]);
    for (int i = lane; i < novr; i += 64) me.consider(ka.over[b * M + i], kk);  // merged below
    const int qbx = cell_coord(me.fx, g.o[0], g.inv, g.d[0]) >> 2;
    const int qby = cell_coord(me.fy, g.o[1], g.inv, g.d[1]) >> 2;
    const int qbz = cell_coord(me.fz, g.o[2], g.inv, g.d[2]) >> 2;
    Box prev = {1, 0, 1, 0, 1, 0};
    // the pruning radius^2: the query pass's kk-th best so far (an upper bound of the true
    // kk-th distance: the refs behind it lie inside it and are found again), then the merged
    // kk-th best of this search
    double best = (double)obound[b * N + q];
#ifdef PCST_KNN_OUTLIER_TRACE
    const uint32_t tr_inf = best == INFINITY ? 1u : 0u;
#endif
    int r = 1;
    if (best != INFINITY) r = max(1, (int)fmin(floor(sqrt(best) * (1.0 + 1e-6) / bs) + 1.0, 4096.0));
    for (;;) {
      const Box bx = {max(qbx - r, 0), min(qbx + r, nbx - 1), max(qby - r, 0), min(qby + r, nby - 1),
                      max(qbz - r, 0), min(qbz + r, nbz - 1)};
      const int nx = bx.x1 - bx.x0 + 1, ny = bx.y1 - bx.y0 + 1;
      const int vol = bx.volume();
      const float rnx = 1.0f / nx, rnxy = 1.0f / (nx * ny);
      const double lim = best;
      auto unit = [&](int li, uint64_t& lo, uint64_t& hi) {
        lo = hi = 0;
        if (li < vol) {
          const int qz = (int)(((float)li + 0.5f) * rnxy), rz = li - qz * nx * ny;
          const int qy = (int)(((float)rz + 0.5f) * rnx), qx = rz - qy * nx;
          const int x = bx.x0 + qx, y = bx.y0 + qy, z = bx.z0 + qz;
          if (prev.has(x, y, z)) return;
          // squared distance from the query to the brick's box, less the cell-rounding slack
          const double x0 = g.o[0] + x * bs, y0 = g.o[1] + y * bs, z0 = g.o[2] + z * bs;
          const double ex = fmax(fmax(x0 - me.qx, me.qx - (x0 + bs)), 0.0);
          const double ey = fmax(fmax(y0 - me.qy, me.qy - (y0 + bs)), 0.0);
          const double ez = fmax(fmax(z0 - me.qz, me.qz - (z0 + bs)), 0.0);
          const double e = fmax(sqrt(ex * ex + ey * ey + ez * ez) - g.slack, 0.0);
          if (e * e > lim) return;
          const int u0 = ((z * nby + y) * nbx + x) << 6;
          uint32_t ra, re;
          if constexpr (ROWS) {  // the brick's placed refs, at the front of its row range
            ra = (uint32_t)(S[u0] >> 32);
            re = ra + min(BC[u0 >> 6], (uint32_t)(S[u0 + 64] >> 32) - ra);
          } else {
            ra = (uint32_t)S[u0];
            re = (uint32_t)S[u0 + 64];
          }
          if (re < ra || re > rlim) {
            atomicOr(ka.err, 8);
            return;
          }
          lo = ra;
          hi = re;
        }
      };
      uint32_t staged = 0;
      scan_units_1q(vol, unit, R, me, kk, staged);
#ifdef PCST_KNN_OUTLIER_TRACE
      ++tr_shells;
      tr_staged += staged;
#endif
      // merge the lanes' lists into lane 0; the others restart empty with the merged screen
      Top3 t = me.t;
      wave_merge_top3(t);
      best = fmin(best, t.last(kk));
      if (lane == 0) me.t = t;
      else me.t.init();
      if (best != INFINITY) me.thr = fminf(me.thr, (float)(best * (1.0 + 2e-6)) + 1e-30f);
      if (bx.x0 == 0 && bx.y0 == 0 && bx.z0 == 0 && bx.x1 == nbx - 1 && bx.y1 == nby - 1 &&
          bx.z1 == nbz - 1)
        break;
      const Box cells = {bx.x0 * 4, min(bx.x1 * 4 + 3, g.d[0] - 1), bx.y0 * 4,
                         min(bx.y1 * 4 + 3, g.d[1] - 1), bx.z0 * 4, min(bx.z1 * 4 + 3, g.d[2] - 1)};
      if (best != INFINITY) {  // wave-uniform: the merged list, the query's own box
        const double ob = outside_bound(me, cells, g);
        if (ob == INFINITY || (ob > 0 && best < ob * ob)) break;
      }
      prev = bx;
      // next box: once kk refs are known, the one whose faces (R bricks from the query's brick)
      // lie beyond the current kk-th distance -- the last shell unless rounding says otherwise;
      // before that, double the radius
      if (best != INFINITY) {
        const double need = floor(sqrt(best) * (1.0 + 1e-6) / bs) + 1.0;
        r = max(r + 1, (int)fmin(need, 4096.0));
      } else {
        r += 1;  // sparse shells are cheap; a doubled box can reach into the dense core unpruned
      }
    }
    if (lane == 0) idw_write(me.t, kk, V, out + (b * N + n) * 3);
#ifdef PCST_KNN_OUTLIER_TRACE
    if (lane == 0 && q < 8192)
      reinterpret_cast<uint4*>(const_cast<float*>(obound) + b * N + 80000)[q] =
          make_uint4(tr0, (uint32_t)__builtin_amdgcn_s_memrealtime(),
                     min(tr_shells, 32767u) | (tr_inf << 15) | ((uint32_t)min(r, 65535) << 16), tr_staged);
#endif
  }
}

}  // namespace pcst

using namespace pcst;

extern "C" int pcst_knn_workspace_size(int64_t B, int64_t N, int64_t M, size_t* bytes) {
  PCST_CHECK_ARG(B >= 0 && N >= 0 && M >= 0 && bytes, "knn_workspace_size: bad args");
  *bytes = carve_knn(nullptr, B, N, M).bytes;
  return PCST_OK;
}

// LDS floor of the build workgroups (the `lds_floor` argument of pcst_knn3_build): a kernel
// whose own static LDS is below it gets the difference as dynamic LDS.  A build that runs on a
// side stream during the noise MLP then cannot co-reside with an MLP workgroup (155 KiB of the
// CU's 160): it only takes the CUs the MLP leaves idle in its last partial round, and a floor just
// above the MLP's leftover (8 KiB) keeps as many build workgroups per idle CU as their own LDS
// allows.  A pure function of the kernel and the floor (no state kept between calls).
// The kernels' static LDS is a compile-time constant (their __shared__ arrays), so no runtime
// attribute query sits on the launch path (hipFuncGetAttributes cost ~5 us of host time each).
constexpr unsigned kLdsPre = 0;
constexpr unsigned kLdsCount = 8 * sizeof(float) + kKnnMaxTiles * sizeof(unsigned long long);
constexpr unsigned kLdsScan = (kKnnTile + kKnnTile / 32 + 8) * sizeof(unsigned long long);
constexpr unsigned kLdsFill = 0;
static unsigned pad_for(unsigned static_lds, unsigned floor_bytes) {
  return static_lds >= floor_bytes ? 0u : floor_bytes - static_lds;
}

// Phase 1 (positions only: the coarse set's points and the full cloud): grid statistics, the
// packed cell counts, scan, fill.  Phase 2 (needs the coarse values, i.e. the noise MLP's
// output): known rows, the query passes and the outlier pass.  Splitting them lets a caller run
// phase 1 on a second stream while the MLP runs (guided_sample_loop).
// max_wg (> 0): at most this many work-groups per build launch over all clouds (each kernel
// strides over its work), so a build on a side stream holds at most max_wg CUs -- the noise MLP's
// last partial round of work-groups leaves ~40 of 256 idle and never waits for one held by the
// build.  0 = the kernels' natural grids.
extern "C" int pcst_knn3_build(const float* orig, const int64_t* idx, int64_t B, int64_t N,
                               int64_t M, int64_t lds_floor, int64_t max_wg, void* workspace,
                               void* stream) {
  PCST_CHECK_ARG(B >= 0 && N > 0 && M > 0 && N < (1ll << 31) && M < (1ll << 27) &&
                     M + N < (1ll << 31),
                 "knn3_build: bad shape");
  PCST_CHECK_ARG(lds_floor >= 0 && lds_floor <= 98304, "knn3_build: lds_floor is 0..98304 bytes");
  PCST_CHECK_ARG(max_wg >= 0, "knn3_build: max_wg < 0");
  if (B == 0) return PCST_OK;
  PCST_CHECK_ARG(orig && idx && workspace, "knn3_build: null pointer");
  hipStream_t s = as_stream(stream);
  KnnWS w = carve_knn(workspace, B, N, M);
  const int b = (int)B;
  const unsigned f = (unsigned)lds_floor;
  const unsigned pad_pre = pad_for(kLdsPre, f), pad_count = pad_for(kLdsCount, f),
                 pad_scan = pad_for(kLdsScan, f), pad_fill = pad_for(kLdsFill, f);
  // per-cloud grid of each launch: natural size, capped at max_wg / B (at least one)
  const int64_t cap = max_wg > 0 ? std::max<int64_t>(1, max_wg / B) : (int64_t)1 << 30;
  auto grid = [&](int64_t natural) { return (unsigned)std::min<int64_t>(natural, cap); };
  // error word, counters, known rows, tile sums and packed counts are contiguous in the carve
  PCST_HIP(hipMemsetAsync(w.err, 0, (size_t)(w.bytes - ((char*)w.err - (char*)workspace)), s),
           "knn: memset");
  hipLaunchKernelGGL(knn_pre_kernel, dim3(grid(kStatBlocks + kPreKnownBlocks), b), dim3(256), pad_pre,
                     s, orig, idx, (int)N, M, w.stats, w.known, w.err);
  hipLaunchKernelGGL(knn_count_kernel, dim3(grid(cdiv(M + N, kCountPerBlock)), b), dim3(256),
                     pad_count, s, orig, idx, w.stats, w.known, N, M, M, w.Cmax, w.T, w.Cpad, w.gp,
                     w.cnt, w.tsum, w.crank);
  hipLaunchKernelGGL(knn_scan_kernel, dim3(grid(w.T), b), dim3(256), pad_scan, s, w.cnt, w.tsum,
                     w.T, w.Cpad, w.chunks, w.maxch, w.nchunk);
  const unsigned gf = grid(std::min<int64_t>(cdiv(M + N, 256), 2048));
  hipLaunchKernelGGL(knn_fill_kernel, dim3(gf, b), dim3(256), pad_fill, s, orig, idx, N, M, w.Cpad,
                     w.cnt, w.crank, w.refs, w.qorder);
  PCST_LAUNCH_CHECK("knn3_build");
  return PCST_OK;
}

// The query and outlier launches.  Both layouts: the per-layout pointers (the compact workspace's
// or the rows workspace's) come in as arguments; ka carries the rows layout's extras, the error
// word and the work counters.  The query grid is the resident one (kQueryBlocksPerCU per CU,
// grid_cap > 0 caps it), a multiple of B, and no larger than the rows' chunk lists need.
template <bool ROWS>
static void launch_knn_query(int64_t nch_max, const float* gp, const uint64_t* cnt, const float4* refs,
                             const int32_t* qorder, const uint2* chunks, const int32_t* nchunk,
                             int32_t* olist, float* obound, int32_t* ocount, const uint32_t* known,
                             int64_t Cpad, const KArgs& ka, const float* coarse, const float* orig,
                             int64_t B, int64_t N, int64_t M, float* out, const uint32_t* bflag,
                             uint32_t bvalue, int64_t grid_cap, hipStream_t s) {
  const int64_t cap = grid_cap > 0 ? grid_cap : (int64_t)device_cus() * kQueryBlocksPerCU;
  const int64_t Gr = std::max<int64_t>(1, std::min<int64_t>(cdiv(nch_max, 4), cap / B));
  auto qk = M >= 3 ? knn_query_kernel<3, ROWS>
                   : (M == 2 ? knn_query_kernel<2, ROWS> : knn_query_kernel<1, ROWS>);
  hipLaunchKernelGGL(qk, dim3((unsigned)(Gr * B)), dim3(256), 0, s, orig, coarse, B, N, M, Cpad, gp, cnt,
                     refs, qorder, chunks, nch_max, nchunk, olist, obound, ocount, out, bflag, bvalue, ka);
  auto ok = M >= 3 ? knn_outlier_brick_kernel<3, ROWS>
                   : (M == 2 ? knn_outlier_brick_kernel<2, ROWS> : knn_outlier_brick_kernel<1, ROWS>);
  hipLaunchKernelGGL(ok, dim3(kOutlierBrickBlocks, (unsigned)B), dim3(256), 0, s, coarse, N, M, orig, gp,
                     Cpad, cnt, refs, olist, obound, ocount, known, out, bflag, bvalue, ka);
}

static void launch_knn_query(const KnnWS& w, const float* coarse, const float* orig, int64_t B,
                             int64_t N, int64_t M, float* out, const uint32_t* bflag,
                             uint32_t bvalue, int64_t grid_cap, hipStream_t s) {
  const KArgs ka = {B, nullptr, nullptr, nullptr, nullptr, nullptr, w.err, nullptr, w.qctr, nullptr,
                    nullptr};
  launch_knn_query<false>(w.maxch, w.gp, w.cnt, w.refs, w.qorder, w.chunks, w.nchunk, w.olist,
                          w.obound, w.ocount, w.known, w.Cpad, ka, coarse, orig, B, N, M, out,
                          bflag, bvalue, grid_cap, s);
}

#define PCST_KNN_SHAPE_CHECK(name)                                                      \
  PCST_CHECK_ARG(B >= 0 && N > 0 && M > 0 && N < (1ll << 31) && M < (1ll << 27) &&      \
                     M + N < (1ll << 31),                                               \
                 name ": bad shape")

extern "C" int pcst_knn3_query(const float* coarse, const float* orig, int64_t B, int64_t N,
                               int64_t M, float* out, void* workspace, const uint32_t* built_flag,
                               uint32_t built_value, int64_t grid_cap, void* stream) {
  PCST_KNN_SHAPE_CHECK("knn3_query");
  if (B == 0) return PCST_OK;
  PCST_CHECK_ARG(coarse && orig && out && workspace, "knn3_query: null pointer");
  KnnWS w = carve_knn(workspace, B, N, M);
  launch_knn_query(w, coarse, orig, B, N, M, out, built_flag, built_value, grid_cap,
                   as_stream(stream));
  PCST_LAUNCH_CHECK("knn3_query");
  return PCST_OK;
}

extern "C" int pcst_knn3_interp(const float* coarse, const float* orig, const int64_t* idx,
                                int64_t B, int64_t N, int64_t M, float* out, void* workspace,
                                void* stream) {
  int rc = pcst_knn3_build(orig, idx, B, N, M, 0, 0, workspace, stream);
  if (rc) return rc;
  return pcst_knn3_query(coarse, orig, B, N, M, out, workspace, nullptr, 0u, 0, stream);
}


// diagnostics: out[0] = error flag, out[1..B] = query chunks, out[1+B..2B] = outlier queries of
// the last pcst_knn3_query on this workspace
extern "C" int pcst_knn_stats(void* workspace, int64_t B, int64_t N, int64_t M, int32_t* out,
                              void* stream) {
  KnnWS w = carve_knn(workspace, B, N, M);
  hipStream_t s = as_stream(stream);
  PCST_HIP(hipMemcpyAsync(out, w.err, sizeof(int32_t), hipMemcpyDeviceToDevice, s), "knn_stats");
  PCST_HIP(hipMemcpyAsync(out + 1, w.nchunk, sizeof(int32_t) * B, hipMemcpyDeviceToDevice, s), "knn_stats");
  PCST_HIP(hipMemcpyAsync(out + 1 + B, w.ocount, sizeof(int32_t) * B, hipMemcpyDeviceToDevice, s),
           "knn_stats");
  return PCST_OK;
}

extern "C" int pcst_knn_error(void* workspace, int64_t B, int64_t N, int64_t M, int32_t* err_out,
                              void* stream) {
  KnnWS w = carve_knn(workspace, B, N, M);
  PCST_HIP(hipMemcpyAsync(err_out, w.err, sizeof(int32_t), hipMemcpyDeviceToDevice,
                          as_stream(stream)), "knn_error");
  return PCST_OK;
}

// ---- rows layout ABI (pcst.h) ----
#define PCST_KNN_ROWS_CHECK(name)                                                             \
  PCST_CHECK_ARG(C >= 0 && copies >= 1 && N > 0 && M > 0 && N < (1ll << 31) && M < (1ll << 27), \
                 name ": bad shape")

extern "C" int pcst_knn_rows_workspace_size(int64_t C, int64_t copies, int64_t N, int64_t M,
                                            size_t* bytes) {
  PCST_KNN_ROWS_CHECK("knn_rows_workspace_size");
  PCST_CHECK_ARG(bytes != nullptr, "knn_rows_workspace_size: null pointer");
  *bytes = carve_knn_rows(nullptr, C, copies, N, M).bytes;
  return PCST_OK;
}

extern "C" int pcst_knn3_rows_build(const float* x, int64_t C, int64_t copies, int64_t N, int64_t M,
                                    void* workspace, uint32_t* refs_flag, uint32_t refs_value,
                                    uint32_t* done_flag, uint32_t done_value, void* stream) {
  PCST_KNN_ROWS_CHECK("knn3_rows_build");
  if (C == 0) return PCST_OK;
  PCST_CHECK_ARG(x && workspace, "knn3_rows_build: null pointer");
  hipStream_t s = as_stream(stream);
  KnnRowsWS w = carve_knn_rows(workspace, C, copies, N, M);
  const int c = (int)C;
  const size_t zbytes = (size_t)(w.bytes - ((char*)w.err - (char*)workspace));  // 256-B multiple
  hipLaunchKernelGGL(knn_pre_kernel, dim3(kStatBlocks + kPreZeroBlocks, c), dim3(256), 0, s, x,
                     (const int64_t*)nullptr, (int)N, (int64_t)0, w.stats, w.known, w.err,
                     reinterpret_cast<uint4*>(w.err), (int64_t)(zbytes / 16));
  hipLaunchKernelGGL(knn_count_kernel, dim3((unsigned)cdiv(N, kCountPerBlock), c), dim3(256), 0, s, x,
                     (const int64_t*)nullptr, w.stats, (const uint32_t*)nullptr, N, (int64_t)0, M, w.Cmax,
                     w.T, w.Cpad, w.gp, w.cnt, w.tsum, w.crank);
  hipLaunchKernelGGL(knn_scan_kernel, dim3((unsigned)w.T, c), dim3(256), 0, s, w.cnt, w.tsum, w.T,
                     w.Cpad, w.chunks, w.maxch, w.nchunk);
  // the ref placement reads the starts and the rows' cells, not the fill's row order
  if (refs_flag) hipLaunchKernelGGL(knn_flag_kernel, dim3(1), dim3(64), 0, s, refs_flag, refs_value);
  hipLaunchKernelGGL(knn_rows_fill_kernel, dim3((unsigned)std::min<int64_t>(cdiv(N, 256), 2048), c),
                     dim3(256), 0, s, x, N, w.Cpad, w.cnt, w.crank, w.xs);
  if (done_flag) hipLaunchKernelGGL(knn_flag_kernel, dim3(1), dim3(64), 0, s, done_flag, done_value);
  PCST_LAUNCH_CHECK("knn3_rows_build");
  return PCST_OK;
}

// Phase B as a launch of its own (pcst_knn3_rows_refs; the downsample when its emit grid is too
// large to wait in-kernel): the work-groups load their indices, then wait for phase A's flag.  At
// most max(CUs, rows) work-groups (grid-stride over the refs), so the waiting ones never hold
// every CU while phase A still needs some.
int pcst::rows_place_launch(const KnnRowsWS& w, const float* x, const int64_t* idx, int64_t N, int64_t M,
                            const uint32_t* wflag, uint32_t wvalue, int32_t* werr, int64_t max_polls,
                            hipStream_t s) {
  const int64_t per = std::max<int64_t>(1, std::min<int64_t>(cdiv(M, 256), device_cus() / w.B));
  hipLaunchKernelGGL(knn_rows_place_kernel, dim3((unsigned)per, (unsigned)w.B), dim3(256), 0, s, x, idx,
                     rows_place_args(w, N, M), w.err, wflag, wvalue, werr,
                     max_polls > 0 ? max_polls : (int64_t)kSignalPolls);
  return PCST_OK;
}

extern "C" int pcst_knn3_rows_refs(const float* x, const int64_t* idx, int64_t C, int64_t copies,
                                   int64_t N, int64_t M, void* workspace, const uint32_t* wait_flag,
                                   uint32_t wait_value, int32_t* wait_err, int64_t max_polls,
                                   void* stream) {
  PCST_KNN_ROWS_CHECK("knn3_rows_refs");
  if (C == 0) return PCST_OK;
  PCST_CHECK_ARG(x && idx && workspace, "knn3_rows_refs: null pointer");
  KnnRowsWS w = carve_knn_rows(workspace, C, copies, N, M);
  rows_place_launch(w, x, idx, N, M, wait_flag, wait_value, wait_err, max_polls, as_stream(stream));
  PCST_LAUNCH_CHECK("knn3_rows_refs");
  return PCST_OK;
}

extern "C" int pcst_knn3_rows_query(const float* coarse, const float* x, int64_t C, int64_t copies,
                                    int64_t N, int64_t M, float* out, void* workspace,
                                    const uint32_t* built_flag, uint32_t built_value,
                                    int32_t* wait_err, int64_t max_polls, const int32_t* refs_err,
                                    int64_t grid_cap, void* stream) {
  PCST_KNN_ROWS_CHECK("knn3_rows_query");
  if (C == 0) return PCST_OK;
  PCST_CHECK_ARG(coarse && x && out && workspace, "knn3_rows_query: null pointer");
  KnnRowsWS w = carve_knn_rows(workspace, C, copies, N, M);
  const KArgs ka = {C, w.known, w.xs, w.rcnt, w.over, w.ovn, w.err, refs_err, w.qctr, w.brefs, w.bcnt};
  // a wait for the build: one work-group before the query (never the query's own work-groups)
  if (built_flag && wait_err) {
    const int rc = pcst_signal_wait(built_flag, built_value, wait_err, max_polls, stream);
    if (rc) return rc;
  }
  launch_knn_query<true>(w.maxch, w.gp, w.cnt, w.refs, nullptr, w.chunks, w.nchunk, w.olist,
                         w.obound, w.ocount, w.known, w.Cpad, ka, coarse, x, w.B, N, M, out,
                         built_flag, built_value, grid_cap, as_stream(stream));
  PCST_LAUNCH_CHECK("knn3_rows_query");
  return PCST_OK;
}

// out[0] = error word, out[1..C] = chunks per cloud, out[1+C..C+B] = outlier queries and
// out[1+C+B..C+2B] = overflow refs per CFG row of the last build / refs / query on this workspace
extern "C" int pcst_knn_rows_stats(void* workspace, int64_t C, int64_t copies, int64_t N, int64_t M,
                                   int32_t* out, void* stream) {
  PCST_KNN_ROWS_CHECK("knn_rows_stats");
  PCST_CHECK_ARG(workspace && out, "knn_rows_stats: null pointer");
  KnnRowsWS w = carve_knn_rows(workspace, C, copies, N, M);
  hipStream_t s = as_stream(stream);
  PCST_HIP(hipMemcpyAsync(out, w.err, sizeof(int32_t), hipMemcpyDeviceToDevice, s), "knn_rows_stats");
  PCST_HIP(hipMemcpyAsync(out + 1, w.nchunk, sizeof(int32_t) * C, hipMemcpyDeviceToDevice, s), "knn_rows_stats");
  PCST_HIP(hipMemcpyAsync(out + 1 + C, w.ocount, sizeof(int32_t) * w.B, hipMemcpyDeviceToDevice, s),
           "knn_rows_stats");
  PCST_HIP(hipMemcpyAsync(out + 1 + C + w.B, w.ovn, sizeof(int32_t) * w.B, hipMemcpyDeviceToDevice, s),
           "knn_rows_stats");
  return PCST_OK;
}
