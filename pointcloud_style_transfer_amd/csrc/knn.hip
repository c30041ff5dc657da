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
// Exact search on a uniform grid over the cloud's bounding box (refs counting-sorted by cell,
// ~2 refs per cell), shell-by-shell around the query's cell until the 3rd-best distance is
// below the distance to the unvisited region.  All distance/weight arithmetic is float64 with
// *_rn intrinsics (no contraction), so neighbour sets and weights match the reference.
#include "common.h"
#include "sort.h"
#include "cloud.h"

namespace pcst {

struct KnnWS {
  int32_t* mm;       // [B][6]
  float* gp;         // [B][8]: origin xyz, cell size, inv size, dims xyz (as float bits)
  uint32_t* known;   // [B][N]  (j+1 of the last coarse row writing n, 0 = query)
  uint32_t* ccount;  // [B][C]  counts, then (after the scan) cell starts
  uint32_t* cursor;  // [B][C]  fill cursors
  float4* refs;      // [B][M]  (x, y, z, j as bits), cell-sorted
  int32_t* err;
  int64_t C;
  size_t bytes;
};

static KnnWS carve_knn(void* base, int64_t B, int64_t N, int64_t M) {
  Carver c(base);
  KnnWS w;
  w.C = std::max<int64_t>(64, 2 * M);
  w.mm = c.take<int32_t>(B * 6);
  w.gp = c.take<float>(B * 8);
  w.err = c.take<int32_t>(4);
  w.known = c.take<uint32_t>(B * N);
  w.ccount = c.take<uint32_t>(B * w.C);
  w.cursor = c.take<uint32_t>(B * w.C);
  w.refs = c.take<float4>(B * M);
  w.bytes = c.bytes();
  return w;
}

// Grid: ~2 refs per cell over the bounding box, at most C cells, each dim in [1, 1024].
__global__ void knn_grid_params_kernel(const int32_t* __restrict__ mm, int B, int64_t M, int64_t C,
                                       float* __restrict__ gp) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int32_t* Mm = mm + b * 6;
  double lo[3], ext[3];
  for (int c = 0; c < 3; ++c) {
    lo[c] = ord2f(Mm[c]);
    ext[c] = (double)ord2f(Mm[3 + c]) - lo[c];
    if (!(ext[c] > 1e-12)) ext[c] = 1e-12;
  }
  const double cells = fmax(1.0, (double)M / 2.0);
  double s = cbrt(ext[0] * ext[1] * ext[2] / cells);
  // thin dimensions: shrink s so the other dims carry the cells
  for (int it = 0; it < 3; ++it) {
    int flat = 0;
    double vol = 1.0;
    for (int c = 0; c < 3; ++c) {
      if (ext[c] < s) ++flat;
      else vol *= ext[c];
    }
    if (flat == 0 || flat == 3) break;
    s = pow(vol / cells, 1.0 / (3 - flat));
  }
  int d[3];
  for (;;) {
    int64_t tot = 1;
    for (int c = 0; c < 3; ++c) {
      d[c] = (int)fmin(1024.0, fmax(1.0, ceil(ext[c] / s)));
      tot *= d[c];
    }
    if (tot <= C) break;
    s *= 1.1;
  }
  float* G = gp + b * 8;
  G[0] = (float)lo[0]; G[1] = (float)lo[1]; G[2] = (float)lo[2];
  G[3] = (float)s;
  G[4] = (float)(1.0 / s);
  G[5] = __int_as_float(d[0]); G[6] = __int_as_float(d[1]); G[7] = __int_as_float(d[2]);
}

__device__ __forceinline__ int cell_coord(float p, float o, float inv, int d) {
  int c = (int)floorf((p - o) * inv);
  return c < 0 ? 0 : (c >= d ? d - 1 : c);
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

__global__ void knn_count_kernel(const float* __restrict__ orig, const int64_t* __restrict__ idx,
                                 int64_t N, int64_t M, int64_t C, const float* __restrict__ gp,
                                 uint32_t* __restrict__ ccount) {
  const int b = blockIdx.y;
  const float* G = gp + b * 8;
  const int dx = __float_as_int(G[5]), dy = __float_as_int(G[6]), dz = __float_as_int(G[7]);
  for (int64_t j = blockIdx.x * 256 + threadIdx.x; j < M; j += gridDim.x * 256) {
    int64_t n = idx[b * M + j];
    n = n < 0 ? 0 : (n >= N ? N - 1 : n);
    const float* p = orig + (b * N + n) * 3;
    const int cx = cell_coord(p[0], G[0], G[4], dx), cy = cell_coord(p[1], G[1], G[4], dy),
              cz = cell_coord(p[2], G[2], G[4], dz);
    atomicAdd(&ccount[b * C + ((int64_t)cz * dy + cy) * dx + cx], 1u);
  }
}

// After the exclusive scan ccount[c] = start of cell c; refs are placed through a copy of
// the starts used as atomic cursors (in-cell order is irrelevant: ties break on j).
__global__ void knn_fill_kernel(const float* __restrict__ orig, const int64_t* __restrict__ idx,
                                int64_t N, int64_t M, int64_t C, const float* __restrict__ gp,
                                uint32_t* __restrict__ cursor, float4* __restrict__ refs) {
  const int b = blockIdx.y;
  const float* G = gp + b * 8;
  const int dx = __float_as_int(G[5]), dy = __float_as_int(G[6]), dz = __float_as_int(G[7]);
  for (int64_t j = blockIdx.x * 256 + threadIdx.x; j < M; j += gridDim.x * 256) {
    int64_t n = idx[b * M + j];
    n = n < 0 ? 0 : (n >= N ? N - 1 : n);
    const float* p = orig + (b * N + n) * 3;
    const int cx = cell_coord(p[0], G[0], G[4], dx), cy = cell_coord(p[1], G[1], G[4], dy),
              cz = cell_coord(p[2], G[2], G[4], dz);
    const uint32_t pos = atomicAdd(&cursor[b * C + ((int64_t)cz * dy + cy) * dx + cx], 1u);
    refs[b * M + pos] = make_float4(p[0], p[1], p[2], __int_as_float((int)j));
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

__global__ __launch_bounds__(256) void knn_query_kernel(
    const float* __restrict__ orig, const float* __restrict__ vals, int64_t N, int64_t M,
    int64_t C, const float* __restrict__ gp, const uint32_t* __restrict__ known,
    const uint32_t* __restrict__ cstart, const float4* __restrict__ refs, float* __restrict__ out) {
  const int b = blockIdx.y;
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
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
  const double qx = q[0], qy = q[1], qz = q[2];
  const int cx = cell_coord(q[0], G[0], G[4], dx), cy = cell_coord(q[1], G[1], G[4], dy),
            cz = cell_coord(q[2], G[2], G[4], dz);
  const double ox = G[0], oy = G[1], oz = G[2], s = G[3];
  const double slack = 1e-5 * s;  // covers fp32 cell-assignment rounding
  const uint32_t* CS = cstart + b * C;
  const float4* R = refs + b * M;
  const int k = M < 3 ? (int)M : 3;
  Top3 t;
  t.init();
  const int rmax = max(dx, max(dy, dz));
  for (int r = 0; r <= rmax; ++r) {
    for (int z = cz - r; z <= cz + r; ++z) {
      if (z < 0 || z >= dz) continue;
      for (int y = cy - r; y <= cy + r; ++y) {
        if (y < 0 || y >= dy) continue;
        const bool face = (z == cz - r || z == cz + r || y == cy - r || y == cy + r);
        const int step = (face || r == 0) ? 1 : 2 * r;
        for (int x = cx - r; x <= cx + r; x += step) {
          if (x < 0 || x >= dx) continue;
          const int64_t cell = ((int64_t)z * dy + y) * dx + x;
          const uint32_t a = CS[cell];
          const uint32_t e = cell + 1 < C ? CS[cell + 1] : (uint32_t)M;
          for (uint32_t i = a; i < e; ++i) {
            const float4 ref = R[i];
            const double ex = dsub(qx, (double)ref.x), ey = dsub(qy, (double)ref.y),
                         ez = dsub(qz, (double)ref.z);
            const double d = dadd(dadd(dmul(ex, ex), dmul(ey, ey)), dmul(ez, ez));
            t.push(d, __float_as_int(ref.w));
          }
        }
      }
    }
    if (t.d[k - 1] == INFINITY) continue;
    // distance from q to the unvisited region outside the (2r+1)^3 block
    double bound = INFINITY;
    if (cx - r > 0) bound = fmin(bound, qx - (ox + (cx - r) * s));
    if (cx + r + 1 < dx) bound = fmin(bound, (ox + (cx + r + 1) * s) - qx);
    if (cy - r > 0) bound = fmin(bound, qy - (oy + (cy - r) * s));
    if (cy + r + 1 < dy) bound = fmin(bound, (oy + (cy + r + 1) * s) - qy);
    if (cz - r > 0) bound = fmin(bound, qz - (oz + (cz - r) * s));
    if (cz + r + 1 < dz) bound = fmin(bound, (oz + (cz + r + 1) * s) - qz);
    bound -= slack;
    if (bound == INFINITY || (bound > 0 && t.d[k - 1] < bound * bound)) break;
  }
  double w[3], wsum = 0.0;
  for (int i = 0; i < k; ++i) {
    w[i] = __ddiv_rn(1.0, dadd(__dsqrt_rn(t.d[i]), 1e-8));
    wsum = i == 0 ? w[0] : dadd(wsum, w[i]);
  }
  for (int i = 0; i < k; ++i) w[i] = __ddiv_rn(w[i], wsum);
  for (int c = 0; c < 3; ++c) {
    double acc = 0.0;
    for (int i = 0; i < k; ++i) {
      const double term = dmul((double)V[(int64_t)t.j[i] * 3 + c], w[i]);
      acc = i == 0 ? term : dadd(acc, term);
    }
    O[c] = (float)acc;
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
  PCST_CHECK_ARG(B >= 0 && N > 0 && M > 0 && N < (1ll << 31) && M < (1ll << 31),
                 "knn3_interp: bad shape");
  if (B == 0) return PCST_OK;
  PCST_CHECK_ARG(coarse && orig && idx && out && workspace, "knn3_interp: null pointer");
  hipStream_t s = as_stream(stream);
  KnnWS w = carve_knn(workspace, B, N, M);
  const int b = (int)B;
  PCST_HIP(hipMemsetAsync(w.err, 0, 16, s), "knn: memset");
  PCST_HIP(hipMemsetAsync(w.known, 0, sizeof(uint32_t) * B * N, s), "knn: memset");
  PCST_HIP(hipMemsetAsync(w.ccount, 0, sizeof(uint32_t) * B * w.C, s), "knn: memset");
  launch_cloud_minmax(orig, b, (int)N, w.mm, s);
  hipLaunchKernelGGL(knn_grid_params_kernel, dim3((unsigned)cdiv(B, 64)), dim3(64), 0, s, w.mm, b,
                     M, w.C, w.gp);
  const unsigned gm = (unsigned)std::min<int64_t>(cdiv(M, 256), 1024);
  hipLaunchKernelGGL(knn_known_kernel, dim3(gm, b), dim3(256), 0, s, idx, N, M, w.known, w.err);
  hipLaunchKernelGGL(knn_count_kernel, dim3(gm, b), dim3(256), 0, s, orig, idx, N, M, w.C, w.gp,
                     w.ccount);
  SegCounts cc{nullptr, (int32_t)w.C};
  hipLaunchKernelGGL(seg_scan_kernel, dim3(b), dim3(1024), 0, s, w.ccount, 1, (int)w.C, cc, 1,
                     (int32_t*)nullptr);
  PCST_HIP(hipMemcpyAsync(w.cursor, w.ccount, sizeof(uint32_t) * B * w.C,
                          hipMemcpyDeviceToDevice, s), "knn: copy starts");
  hipLaunchKernelGGL(knn_fill_kernel, dim3(gm, b), dim3(256), 0, s, orig, idx, N, M, w.C, w.gp,
                     w.cursor, w.refs);
  hipLaunchKernelGGL(knn_query_kernel, dim3((unsigned)cdiv(N, 256), b), dim3(256), 0, s, orig,
                     coarse, N, M, w.C, w.gp, w.known, w.ccount, w.refs, out);
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
