// Offline voxel-grid downsample of PointCloudPreprocessor._voxel_grid_downsample_numpy
// (data/preprocessing.py:45-104), per-point part on the device.  The
// representative rule differs from the model's mean-index rule (diffusion_model.py:69-122): a
// voxel keeps the point nearest to its centre.  For every point this kernel writes
//   key  = the voxel's integer coordinates floor(f32(f32(p - min) / vs)) (numpy float32 math),
//          packed 21 bits per axis;
//   dist = float64 |p - centre|, centre = f64(min) + (coord + 0.5) * f64(vs), the norm summed
//          (dx^2 + dy^2) + dz^2 as np.linalg.norm(axis=1) does for three columns.
// The host groups by key (first-appearance order, argmin with the lowest index on ties).
#include "common.h"

namespace pcst {

__global__ __launch_bounds__(256) void voxel_center_dist_kernel(const float* __restrict__ pts,
                                                                int64_t n, float mnx, float mny,
                                                                float mnz, float vs,
                                                                int64_t* __restrict__ key,
                                                                double* __restrict__ dist,
                                                                int* __restrict__ overflow) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float* p = pts + i * 3;
    const float mn[3] = {mnx, mny, mnz};
    int64_t k = 0;
    double s = 0.0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float c = floorf(__fdiv_rn(fsub(p[a], mn[a]), vs));
      const int64_t ci = (int64_t)c;
      if (ci < 0 || ci >= (1 << 21)) atomicOr(overflow, 1);
      k = (k << 21) | (ci & ((1 << 21) - 1));
      const double ctr = dadd((double)mn[a], dmul(dadd((double)ci, 0.5), (double)vs));
      const double d = dsub((double)p[a], ctr);
      s = a == 0 ? dmul(d, d) : dadd(s, dmul(d, d));
    }
    key[i] = k;
    dist[i] = __dsqrt_rn(s);
  }
}

}  // namespace pcst

using namespace pcst;

extern "C" int pcst_voxel_center_dist(const float* pts, int64_t n, const float* xyz_min,
                                      float voxel_size, int64_t* key, double* dist, int* overflow,
                                      void* stream) {
  PCST_CHECK_ARG(n >= 0 && xyz_min && voxel_size > 0.0f, "voxel_center_dist: bad args");
  if (n == 0) return PCST_OK;
  PCST_CHECK_ARG(pts && key && dist && overflow, "voxel_center_dist: null pointer");
  const int64_t g = std::min<int64_t>(cdiv(n, 256), 4096);
  hipLaunchKernelGGL(voxel_center_dist_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream),
                     pts, n, xyz_min[0], xyz_min[1], xyz_min[2], voxel_size, key, dist, overflow);
  PCST_LAUNCH_CHECK("voxel_center_dist");
  return PCST_OK;
}
