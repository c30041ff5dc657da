// The kNN-3 upsample's rows-layout workspace (knn.hip: pcst_knn3_rows_*), shared with the voxel
// downsample (voxel.hip), whose emit launch can place the coarse refs itself (phase B fused into
// the downsample that produces them: pcst_voxel_downsample_copies_prepped's rows arguments).
#pragma once
#include "common.h"
#include "cloud.h"

namespace pcst {

constexpr int kKnnTile = 4096;           // scan tile (256 threads x 16)
constexpr int kKnnMaxTiles = 1024;       // per-block LDS tile histogram in the count kernel
constexpr int kQueryShards = 8;          // work counters per CFG row (one per XCD)
constexpr int kCtrStride = 64;           // int32 words between counters: each on its own 256-B line

// CUs of the current device (queried per call: the library keeps no process-global state)
static inline int device_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    return 256;
  return n;
}

// the chunk counters: [stride] totals per cloud, then per cloud one u64 (wide list length << 32 |
// narrow list length) on lines of their own (the scan reserves both lists with one atomic)
__host__ __device__ inline int64_t nchunk_stride(int64_t C) { return (C + 63) & ~(int64_t)63; }

static int64_t knn_cells(int64_t M) {
  return std::min<int64_t>(std::max<int64_t>(4096, 16 * M), (int64_t)kKnnMaxTiles * kKnnTile - 1);
}

struct KnnRowsWS {
  StatRec* stats;    // [C][kStatBlocks]
  float* gp;         // [C][8]
  float4* xs;        // [C][N] rows in cell order: (x, y, z, point index n)
  int2* crank;       // [C][N] (cell, rank in cell)
  uint2* chunks;     // [C][maxch] row ranges [q0, q1) of <= 64 rows inside one brick
  float4* refs;      // [B][N] refs (x, y, z, j) at the front of their cell's row range
  float4* brefs;     // [B][N] the placed refs at the front of their brick's row range (outlier
                     // pass; built by the query's waves)
  float4* over;      // [B][M] overflow refs (an index named again)
  int32_t* olist;    // [B][N] outlier query rows
  float* obound;     // [B][N]
  // zeroed every build (contiguous):
  int32_t* err;
  int32_t* qctr;     // [B][2][8][kCtrStride] the query's work counters (chunks, brick batches)
  int32_t* nchunk;   // [nchunk_stride(C)] chunks, then [C] u64 wide (list front) << 32 | narrow (back)
  int32_t* ocount;   // [B]
  int32_t* ovn;      // [B] overflow refs
  uint32_t* known;   // [B][N] j+1 of the last ref naming the row at cell-order position p, 0 = a query
  uint32_t* rcnt;    // [B][Cpad] refs ranked per cell
  uint32_t* bcnt;    // [B][Cpad / 64] the brick copy's ref counts (written if nonzero)
  uint64_t* tsum;    // [C][T]
  uint64_t* cnt;     // [C][Cpad] packed counts (0 | rows << 32) -> starts
  int64_t B, C, Cmax, T, Cpad, maxch;
  size_t bytes;
};

static KnnRowsWS carve_knn_rows(void* base, int64_t C, int64_t copies, int64_t N, int64_t M) {
  Carver c(base);
  KnnRowsWS w;
  w.C = C;
  w.B = C * copies;
  w.Cmax = knn_cells(M);
  w.T = cdiv(w.Cmax + 1, kKnnTile);
  w.Cpad = w.T * kKnnTile;
  w.maxch = cdiv(N, 64) + 8 * (w.Cmax / 64) + 1;
  w.stats = c.take<StatRec>(C * kStatBlocks);
  w.gp = c.take<float>(C * 8);
  w.xs = c.take<float4>(C * N);
  w.crank = c.take<int2>(C * N);
  w.chunks = c.take<uint2>(C * w.maxch);
  w.refs = c.take<float4>(w.B * N);
  w.brefs = c.take<float4>(w.B * N);
  w.over = c.take<float4>(w.B * M);
  w.olist = c.take<int32_t>(w.B * N);
  w.obound = c.take<float>(w.B * N);
  w.err = c.take<int32_t>(4);
  w.qctr = c.take<int32_t>(w.B * 2 * kQueryShards * kCtrStride);
  w.nchunk = c.take<int32_t>(3 * nchunk_stride(C));
  w.ocount = c.take<int32_t>(w.B);
  w.ovn = c.take<int32_t>(w.B);
  w.known = c.take<uint32_t>(w.B * N);
  w.rcnt = c.take<uint32_t>(w.B * w.Cpad);
  w.bcnt = c.take<uint32_t>(w.B * (w.Cpad / 64));
  w.tsum = c.take<uint64_t>(C * w.T);
  w.cnt = c.take<uint64_t>(C * w.Cpad);
  w.bytes = c.bytes();
  return w;
}

// The arrays phase B writes (the placement of one ref), by value into the kernels.
struct RowsPlace {
  const uint64_t* start;  // [C][Cpad] packed starts (rows in the high word)
  const int2* crank;      // [C][N] (cell, rank in cell) of every row
  uint32_t* known;        // [B][N] by cell-order position
  uint32_t* rcnt;         // [B][Cpad]
  float4* refs;           // [B][N]
  float4* over;           // [B][M]
  int32_t* ovn;           // [B]
  int64_t C, N, M, Cpad;
};

static RowsPlace rows_place_args(const KnnRowsWS& w, int64_t N, int64_t M) {
  return RowsPlace{w.cnt, w.crank, w.known, w.rcnt, w.refs, w.over, w.ovn, w.C, N, M, w.Cpad};
}

// phase B's own launch (knn.hip)
int rows_place_launch(const KnnRowsWS& w, const float* x, const int64_t* idx, int64_t N, int64_t M,
                      const uint32_t* wflag, uint32_t wvalue, int32_t* werr, int64_t max_polls,
                      hipStream_t s);

// The consumer side of a flag hand-off inside a kernel (MI355X_MICROARCH.md, inter-workgroup
// visibility): thread 0 polls (relaxed, agent scope) until the flag holds `value`, at most
// max_polls times, then one agent-scope acquire; the block barrier lets every wave load after it.
// A wait that gives up sets *werr and returns false for the whole block.
__device__ bool block_wait_flag(const uint32_t* flag, uint32_t value, int32_t* werr, int64_t max_polls) {
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    bool ok = false;
    for (int64_t i = 0; i < max_polls; ++i) {
      if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= value) {
        ok = true;
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!ok && werr) __hip_atomic_store(werr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

// Phase B, one ref: ref j (point n, position p) of CFG row b (cloud b % C): its known mark at
// n's cell-order position (the last j wins), its rank in n's cell (both atomics issued together)
// and its slot start(cell) + rank at the front of the cell's row range; a rank beyond the cell's
// rows sends the ref to the overflow list instead.
__device__ __forceinline__ void rows_place(const RowsPlace& rp, int b, int64_t n, int64_t j,
                                           const float* __restrict__ p) {
  const int64_t cl = b % rp.C, N = rp.N;
  const int2 cr = rp.crank[cl * N + n];
  const uint64_t* S = rp.start + cl * rp.Cpad;
  const uint32_t rank = atomicAdd(&rp.rcnt[b * rp.Cpad + cr.x], 1u);
  const uint32_t a = (uint32_t)(S[cr.x] >> 32), rows = (uint32_t)(S[cr.x + 1] >> 32) - a;
  atomicMax(&rp.known[b * N + a + (uint32_t)cr.y], (uint32_t)(j + 1));
  const float4 r = make_float4(p[0], p[1], p[2], __int_as_float((int)j));
  if (rank < rows) rp.refs[b * N + a + rank] = r;
  else rp.over[b * rp.M + atomicAdd(&rp.ovn[b], 1)] = r;
}

}  // namespace pcst
