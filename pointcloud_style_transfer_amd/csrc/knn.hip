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
// Exact search on a uniform grid whose cell size follows the cloud's PEAK density (estimated
// from the per-axis spread, ~3 refs per cell where the cloud is densest), so a dense core is
// not searched through overfull cells.  Refs and queries are both counting-sorted by cell:
// neighbouring lanes search neighbouring cells (coherent loads, similar trip counts).  Each
// candidate is screened with an fp32 distance (relative error < 3e-7, screened against the
// current 3rd-best x (1 + 2e-6)) and only survivors are ranked in exact float64.
#include "common.h"
#include "cloud.h"

namespace pcst {

constexpr int kRingMax = 4;  // shells searched per query before the exhaustive outlier pass

struct KnnWS {
  StatRec* stats;    // [B][kStatBlocks]
  float* gp;         // [B][8]: origin xyz, cell size, inv size, dims xyz (int bits)
  uint32_t* tsum;    // scan scratch
  float4* refs;      // [B][M]   (x, y, z, j) cell-sorted
  int32_t* qorder;   // [B][N]   point index in cell order
  int32_t* olist;    // [B][N]   queries left to the exhaustive pass
  // zeroed every call (contiguous):
  int32_t* err;
  int32_t* ocount;   // [B]
  uint32_t* known;   // [B][N]  (j+1 of the last coarse row writing n, 0 = query)
  uint32_t* rstart;  // [B][C+1] ref counts -> starts
  uint32_t* qstart;  // [B][C+1] query counts -> starts
  uint32_t* rcur;    // [B][C]   fill cursors (offsets from the starts)
  uint32_t* qcur;    // [B][C]
  int64_t C;
  size_t bytes;
};

static int64_t knn_cells(int64_t M) { return std::max<int64_t>(4096, 16 * M); }

static KnnWS carve_knn(void* base, int64_t B, int64_t N, int64_t M) {
  Carver c(base);
  KnnWS w;
  w.C = knn_cells(M);
  w.stats = c.take<StatRec>(B * kStatBlocks);
  w.gp = c.take<float>(B * 8);
  w.tsum = c.take<uint32_t>(scan_tsum_words((int)B, w.C + 1));
  w.refs = c.take<float4>(B * M);
  w.qorder = c.take<int32_t>(B * N);
  w.olist = c.take<int32_t>(B * N);
  w.err = c.take<int32_t>(4);
  w.ocount = c.take<int32_t>(B);
  w.known = c.take<uint32_t>(B * N);
  w.rstart = c.take<uint32_t>(B * (w.C + 1));
  w.qstart = c.take<uint32_t>(B * (w.C + 1));
  w.rcur = c.take<uint32_t>(B * w.C);
  w.qcur = c.take<uint32_t>(B * w.C);
  w.bytes = c.bytes();
  return w;
}

// Cell size from the peak density of a Gaussian with the cloud's per-axis spread:
// rho_max = M / ((2 pi)^1.5 sx sy sz); s^3 = 3 / rho_max.  Capped so the bounding box holds
// at most C cells (and at most 2048 per axis).
__global__ __launch_bounds__(64) void knn_grid_params_kernel(const StatRec* __restrict__ stats,
                                                             int B, int64_t N, int64_t M, int64_t C,
                                                             float* __restrict__ gp) {
  const int b = blockIdx.x;  // one wave per cloud
  const StatRec r = fold_stats_wave(stats, b);
  if (threadIdx.x != 0) return;
  double ext[3], sig[3];
  for (int c = 0; c < 3; ++c) {
    ext[c] = (double)r.mx[c] - (double)r.mn[c];
    if (!(ext[c] > 1e-9)) ext[c] = 1e-9;
    const double mean = r.s[c] / (double)N;
    double var = r.ss[c] / (double)N - mean * mean;
    sig[c] = sqrt(fmax(var, 0.0));
    sig[c] = fmax(sig[c], 1e-3 * ext[c]);
  }
  const double rho = (double)M / (15.7496099457 * sig[0] * sig[1] * sig[2]);
  double s = cbrt(6.0 / rho);
  // a cell must not be smaller than a thin dimension forces: keep at least ~1 ref per
  // cell on average over the occupied extent
  int d[3];
  for (int it = 0; it < 200; ++it) {
    int64_t tot = 1;
    for (int c = 0; c < 3; ++c) {
      d[c] = (int)fmin(2048.0, fmax(1.0, ceil(ext[c] / s)));
      tot *= d[c];
    }
    if (tot <= C) break;
    s *= 1.1;
  }
  float* G = gp + b * 8;
  G[0] = r.mn[0]; G[1] = r.mn[1]; G[2] = r.mn[2];
  G[3] = (float)s;
  G[4] = (float)(1.0 / s);
  G[5] = __int_as_float(d[0]); G[6] = __int_as_float(d[1]); G[7] = __int_as_float(d[2]);
}

__device__ __forceinline__ int cell_coord(float p, float o, float inv, int d) {
  int c = (int)floorf((p - o) * inv);
  return c < 0 ? 0 : (c >= d ? d - 1 : c);
}

__device__ __forceinline__ int64_t cell_of(const float* p, const float* G) {
  const int dx = __float_as_int(G[5]), dy = __float_as_int(G[6]), dz = __float_as_int(G[7]);
  const int cx = cell_coord(p[0], G[0], G[4], dx), cy = cell_coord(p[1], G[1], G[4], dy),
            cz = cell_coord(p[2], G[2], G[4], dz);
  return ((int64_t)cz * dy + cy) * dx + cx;
}

__global__ void knn_known_kernel(const int64_t* __restrict__ idx, int64_t N, int64_t M,
                                 uint32_t* __restrict__ known, int32_t* __restrict__ err) {
  const int b = blockIdx.y;
  for (int64_t j = blockIdx.x * 256 + threadIdx.x; j < M; j += gridDim.x * 256) {
    const int64_t n = idx[b * M + j];
    if (n < 0 || n >= N) { atomicOr(err, 1); continue; }
    atomicMax(&known[b * N + n], (uint32_t)(j + 1));
  }
}

// count refs (j < M, point orig[idx[j]]) and queries (all N points) per cell
__global__ void knn_count_kernel(const float* __restrict__ orig, const int64_t* __restrict__ idx,
                                 int64_t N, int64_t M, int64_t C, const float* __restrict__ gp,
                                 uint32_t* __restrict__ rcount, uint32_t* __restrict__ qcount) {
  const int b = blockIdx.y;
  const float* G = gp + b * 8;
  for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < M + N; e += gridDim.x * 256) {
    if (e < M) {
      int64_t n = idx[b * M + e];
      n = n < 0 ? 0 : (n >= N ? N - 1 : n);
      atomicAdd(&rcount[b * (C + 1) + cell_of(orig + (b * N + n) * 3, G)], 1u);
    } else {
      const int64_t n = e - M;
      atomicAdd(&qcount[b * (C + 1) + cell_of(orig + (b * N + n) * 3, G)], 1u);
    }
  }
}

__global__ void knn_fill_kernel(const float* __restrict__ orig, const int64_t* __restrict__ idx,
                                int64_t N, int64_t M, int64_t C, const float* __restrict__ gp,
                                const uint32_t* __restrict__ rstart,
                                const uint32_t* __restrict__ qstart, uint32_t* __restrict__ rcur,
                                uint32_t* __restrict__ qcur, float4* __restrict__ refs,
                                int32_t* __restrict__ qorder) {
  const int b = blockIdx.y;
  const float* G = gp + b * 8;
  for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < M + N; e += gridDim.x * 256) {
    if (e < M) {
      int64_t n = idx[b * M + e];
      n = n < 0 ? 0 : (n >= N ? N - 1 : n);
      const float* p = orig + (b * N + n) * 3;
      const int64_t c = cell_of(p, G);
      const uint32_t pos = rstart[b * (C + 1) + c] + atomicAdd(&rcur[b * C + c], 1u);
      refs[b * M + pos] = make_float4(p[0], p[1], p[2], __int_as_float((int)e));
    } else {
      const int64_t n = e - M;
      const int64_t c = cell_of(orig + (b * N + n) * 3, G);
      const uint32_t pos = qstart[b * (C + 1) + c] + atomicAdd(&qcur[b * C + c], 1u);
      qorder[b * N + pos] = (int32_t)n;
    }
  }
}

struct Top3 {
  double d[3];
  int j[3];
  __device__ void init() {
    for (int k = 0; k < 3; ++k) { d[k] = INFINITY; j[k] = 0x7fffffff; }
  }
  __device__ __forceinline__ void push(double dd, int jj) {
    // lexicographic (distance, j): deterministic whatever the in-cell order
    if (dd > d[2] || (dd == d[2] && jj >= j[2])) return;
    if (dd < d[1] || (dd == d[1] && jj < j[1])) {
      d[2] = d[1]; j[2] = j[1];
      if (dd < d[0] || (dd == d[0] && jj < j[0])) {
        d[1] = d[0]; j[1] = j[0];
        d[0] = dd; j[0] = jj;
      } else {
        d[1] = dd; j[1] = jj;
      }
    } else {
      d[2] = dd; j[2] = jj;
    }
  }
};

// IDW of the reference (float64, sequential sums), rounded to float32
__device__ __forceinline__ void idw_write(const Top3& t, int kk, const float* __restrict__ V,
                                          float* __restrict__ O) {
  double w[3], wsum = 0.0;
  for (int i = 0; i < kk; ++i) {
    w[i] = __ddiv_rn(1.0, dadd(__dsqrt_rn(t.d[i]), 1e-8));
    wsum = i == 0 ? w[0] : dadd(wsum, w[i]);
  }
  for (int i = 0; i < kk; ++i) w[i] = __ddiv_rn(w[i], wsum);
  for (int c = 0; c < 3; ++c) {
    double acc = 0.0;
    for (int i = 0; i < kk; ++i) {
      const double term = dmul((double)V[(int64_t)t.j[i] * 3 + c], w[i]);
      acc = i == 0 ? term : dadd(acc, term);
    }
    O[c] = (float)acc;
  }
}

__global__ __launch_bounds__(256) void knn_query_kernel(
    const float* __restrict__ orig, const float* __restrict__ vals, int64_t N, int64_t M,
    int64_t C, const float* __restrict__ gp, const uint32_t* __restrict__ known,
    const uint32_t* __restrict__ rstart, const float4* __restrict__ refs,
    const int32_t* __restrict__ qorder, int32_t* __restrict__ olist, int32_t* __restrict__ ocount,
    float* __restrict__ out) {
  const int b = blockIdx.y;
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= N) return;
  const int64_t n = qorder[b * N + k];
  const float* V = vals + b * M * 3;
  float* O = out + (b * N + n) * 3;
  const uint32_t kn = known[b * N + n];
  if (kn) {
    const float* v = V + (int64_t)(kn - 1) * 3;
    O[0] = v[0]; O[1] = v[1]; O[2] = v[2];
    return;
  }
  const float* G = gp + b * 8;
  const int dx = __float_as_int(G[5]), dy = __float_as_int(G[6]), dz = __float_as_int(G[7]);
  const float* q = orig + (b * N + n) * 3;
  const float fx = q[0], fy = q[1], fz = q[2];
  const double qx = fx, qy = fy, qz = fz;
  const int cx = cell_coord(fx, G[0], G[4], dx), cy = cell_coord(fy, G[1], G[4], dy),
            cz = cell_coord(fz, G[2], G[4], dz);
  const double ox = G[0], oy = G[1], oz = G[2], s = G[3];
  const double slack = 1e-5 * s;  // covers fp32 cell-assignment rounding
  const uint32_t* RS = rstart + b * (C + 1);
  const float4* R = refs + b * M;
  const int kk = M < 3 ? (int)M : 3;
  Top3 t;
  t.init();
  float thr = INFINITY;  // fp32 screen: candidates above it cannot enter the top k
  const int rall = max(dx, max(dy, dz));
  const int rmax = min(rall, kRingMax);
  bool done = false;
  // refs of consecutive cells of one (z, y) row are contiguous (row-major counting sort), so
  // a shell is visited as row RANGES: whole rows on its faces, the two end cells inside
  auto scan = [&](uint32_t a, uint32_t e) {
    for (uint32_t i = a; i < e; ++i) {
      const float4 ref = R[i];
      const float ex = fx - ref.x, ey = fy - ref.y, ez = fz - ref.z;
      const float d32 = fmaf(ez, ez, fmaf(ey, ey, ex * ex));
      if (d32 > thr) continue;
      const double ux = dsub(qx, (double)ref.x), uy = dsub(qy, (double)ref.y),
                   uz = dsub(qz, (double)ref.z);
      const double d = dadd(dadd(dmul(ux, ux), dmul(uy, uy)), dmul(uz, uz));
      t.push(d, __float_as_int(ref.w));
      if (t.d[kk - 1] != INFINITY) thr = (float)(t.d[kk - 1] * (1.0 + 2e-6)) + 1e-30f;
    }
  };
  for (int r = 0; r <= rmax; ++r) {
    const int z0 = max(cz - r, 0), z1 = min(cz + r, dz - 1);
    const int y0 = max(cy - r, 0), y1 = min(cy + r, dy - 1);
    const int xl = max(cx - r, 0), xh = min(cx + r, dx - 1);
    for (int z = z0; z <= z1; ++z) {
      for (int y = y0; y <= y1; ++y) {
        const int64_t row = ((int64_t)z * dy + y) * dx;
        const bool face = (r == 0 || z == cz - r || z == cz + r || y == cy - r || y == cy + r);
        if (face) {
          scan(RS[row + xl], RS[row + xh + 1]);
        } else {
          const bool lo = cx - r >= 0, hi = cx + r < dx;
          const uint32_t a0 = lo ? RS[row + cx - r] : 0u, e0 = lo ? RS[row + cx - r + 1] : 0u;
          const uint32_t a1 = hi ? RS[row + cx + r] : 0u, e1 = hi ? RS[row + cx + r + 1] : 0u;
          scan(a0, e0);
          scan(a1, e1);
        }
      }
    }
    if (t.d[kk - 1] == INFINITY) continue;
    // distance from q to the unvisited region outside the (2r+1)^3 block
    double bound = INFINITY;
    if (cx - r > 0) bound = fmin(bound, qx - (ox + (cx - r) * s));
    if (cx + r + 1 < dx) bound = fmin(bound, (ox + (cx + r + 1) * s) - qx);
    if (cy - r > 0) bound = fmin(bound, qy - (oy + (cy - r) * s));
    if (cy + r + 1 < dy) bound = fmin(bound, (oy + (cy + r + 1) * s) - qy);
    if (cz - r > 0) bound = fmin(bound, qz - (oz + (cz - r) * s));
    if (cz + r + 1 < dz) bound = fmin(bound, (oz + (cz + r + 1) * s) - qz);
    bound -= slack;
    if (bound == INFINITY || (bound > 0 && t.d[kk - 1] < bound * bound)) {
      done = true;
      break;
    }
  }
  if (!done) {  // sparse neighbourhood: leave it to the exhaustive wave-per-query pass
    olist[b * N + atomicAdd(&ocount[b], 1)] = (int32_t)n;
    return;
  }
  idw_write(t, kk, V, O);
}

// Exhaustive 3-NN for the queries the shell search left: one wave per query, each lane scans
// M/64 refs with its own top-3, then a butterfly merge (lexicographic (d, j): deterministic).
__global__ __launch_bounds__(256) void knn_outlier_kernel(
    const float* __restrict__ orig, const float* __restrict__ vals, int64_t N, int64_t M,
    const float4* __restrict__ refs, const int32_t* __restrict__ olist,
    const int32_t* __restrict__ ocount, float* __restrict__ out) {
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wg = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int cnt = ocount[b];
  const float4* R = refs + b * M;
  const float* V = vals + b * M * 3;
  const int kk = M < 3 ? (int)M : 3;
  for (int q = wg; q < cnt; q += gridDim.x * 4) {
    const int64_t n = olist[b * N + q];
    const float* p = orig + (b * N + n) * 3;
    const float fx = p[0], fy = p[1], fz = p[2];
    const double qx = fx, qy = fy, qz = fz;
    Top3 t;
    t.init();
    float thr = INFINITY;
    for (int64_t i = lane; i < M; i += 64) {
      const float4 ref = R[i];
      const float ex = fx - ref.x, ey = fy - ref.y, ez = fz - ref.z;
      const float d32 = fmaf(ez, ez, fmaf(ey, ey, ex * ex));
      if (d32 > thr) continue;
      const double ux = dsub(qx, (double)ref.x), uy = dsub(qy, (double)ref.y),
                   uz = dsub(qz, (double)ref.z);
      t.push(dadd(dadd(dmul(ux, ux), dmul(uy, uy)), dmul(uz, uz)), __float_as_int(ref.w));
      if (t.d[kk - 1] != INFINITY) thr = (float)(t.d[kk - 1] * (1.0 + 2e-6)) + 1e-30f;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      double od[3];
      int oj[3];
      for (int k = 0; k < 3; ++k) { od[k] = __shfl_xor(t.d[k], off); oj[k] = __shfl_xor(t.j[k], off); }
      for (int k = 0; k < 3; ++k) t.push(od[k], oj[k]);
    }
    if (lane == 0) idw_write(t, kk, V, out + (b * N + n) * 3);
  }
}

}  // namespace pcst

using namespace pcst;

extern "C" int pcst_knn_workspace_size(int64_t B, int64_t N, int64_t M, size_t* bytes) {
  PCST_CHECK_ARG(B >= 0 && N >= 0 && M >= 0 && bytes, "knn_workspace_size: bad args");
  *bytes = carve_knn(nullptr, B, N, M).bytes;
  return PCST_OK;
}

extern "C" int pcst_knn3_interp(const float* coarse, const float* orig, const int64_t* idx,
                                int64_t B, int64_t N, int64_t M, float* out, void* workspace,
                                void* stream) {
  PCST_CHECK_ARG(B >= 0 && N > 0 && M > 0 && N < (1ll << 31) && M < (1ll << 27),
                 "knn3_interp: bad shape");
  if (B == 0) return PCST_OK;
  PCST_CHECK_ARG(coarse && orig && idx && out && workspace, "knn3_interp: null pointer");
  hipStream_t s = as_stream(stream);
  KnnWS w = carve_knn(workspace, B, N, M);
  const int b = (int)B;
  const int64_t C = w.C;
  // counters, known flags, count and cursor arrays are contiguous in the carve: one memset
  PCST_HIP(hipMemsetAsync(w.err, 0, (size_t)(w.bytes - ((char*)w.err - (char*)workspace)), s),
           "knn: memset");
  launch_cloud_stats(orig, b, (int)N, w.stats, s);
  hipLaunchKernelGGL(knn_grid_params_kernel, dim3((unsigned)B), dim3(64), 0, s, w.stats, b, N, M,
                     C, w.gp);
  const unsigned gm = (unsigned)std::min<int64_t>(cdiv(M, 256), 1024);
  hipLaunchKernelGGL(knn_known_kernel, dim3(gm, b), dim3(256), 0, s, idx, N, M, w.known, w.err);
  const unsigned ga = (unsigned)std::min<int64_t>(cdiv(M + N, 256), 2048);
  hipLaunchKernelGGL(knn_count_kernel, dim3(ga, b), dim3(256), 0, s, orig, idx, N, M, C, w.gp,
                     w.rstart, w.qstart);
  seg_scan_long(w.rstart, b, C + 1, C + 1, w.tsum, nullptr, s);
  seg_scan_long(w.qstart, b, C + 1, C + 1, w.tsum, nullptr, s);
  hipLaunchKernelGGL(knn_fill_kernel, dim3(ga, b), dim3(256), 0, s, orig, idx, N, M, C, w.gp,
                     w.rstart, w.qstart, w.rcur, w.qcur, w.refs, w.qorder);
  hipLaunchKernelGGL(knn_query_kernel, dim3((unsigned)cdiv(N, 256), b), dim3(256), 0, s, orig,
                     coarse, N, M, C, w.gp, w.known, w.rstart, w.refs, w.qorder, w.olist, w.ocount,
                     out);
  hipLaunchKernelGGL(knn_outlier_kernel, dim3(256, b), dim3(256), 0, s, orig, coarse, N, M, w.refs,
                     w.olist, w.ocount, out);
  PCST_LAUNCH_CHECK("knn3_interp");
  return PCST_OK;
}

extern "C" int pcst_knn_error(void* workspace, int64_t B, int64_t N, int64_t M, int32_t* err_out,
                              void* stream) {
  KnnWS w = carve_knn(workspace, B, N, M);
  PCST_HIP(hipMemcpyAsync(err_out, w.err, sizeof(int32_t), hipMemcpyDeviceToDevice,
                          as_stream(stream)), "knn_error");
  return PCST_OK;
}
