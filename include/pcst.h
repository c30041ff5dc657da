/*
 * pcst.h -- C ABI of libpcst_hip.so, the MI355X (gfx950) kernels behind the
 * PointNet++-conditioned diffusion hot path of wangxy0820/PointCloud_style_transfer.
 *
 * The reference has no FFI layer (it is pure Python/ATen); each
 * entry point below replaces the ATen op chain of the reference function cited
 * next to it, and is bound from Python by pointcloud_style_transfer_amd/_hip.py
 * (ctypes) -- see INTEGRATION.md for the binding a maintainer would add.
 *
 * Conventions:
 *   - every pointer is a DEVICE pointer owned by the caller; the library never
 *     allocates or frees, and keeps no global mutable state except a
 *     thread-local last-error string;
 *   - index tensors are int64 at the boundary;
 *   - `stream` is a hipStream_t passed as void*; no call synchronises the host,
 *     so every call can be captured into a hipGraph;
 *   - return 0 on success, else a hipError_t value or PCST_E*; the message is
 *     in pcst_last_error().
 *   - layouts are the reference's: point clouds [B, N, 3] float32 row-major.
 */
#ifndef PCST_H_
#define PCST_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCST_OK 0
#define PCST_EINVAL 1001
#define PCST_EUNSUPPORTED 1002

/* Library version string, e.g. "pcst 0.1.0 gfx950". */
const char* pcst_version(void);
/* Message of the last failing call on this thread ("" if none). */
const char* pcst_last_error(void);

/* ---- models/pointnet2_encoder.py ------------------------------------------------------- */

/* square_distance (pointnet2_encoder.py:8-15): out[b,s,n] = ((-2*dot) + |src|^2) + |dst|^2,
 * reproducing the reference's CPU rounding (dot = fma chain, unfused norms).  Bit-exact. */
int pcst_square_distance(const float* src, const float* dst, int64_t B, int64_t S, int64_t N,
                         float* out, void* stream);

/* index_points (pointnet2_encoder.py:17-28): out[b,k,:] = points[b, clamp(idx[b,k],0,N-1), :]
 * for K = prod(idx.shape[1:]) indices per batch and C channels. */
int pcst_index_points(const float* points, int64_t B, int64_t N, int64_t C, const int64_t* idx,
                      int64_t K, float* out, void* stream);

/* farthest_point_sample (pointnet2_encoder.py:30-45): start_idx[B] is the reference's CPU
 * randint draw (copied to the device by the caller).  Bit-exact indices. */
int pcst_fps(const float* xyz, int64_t B, int64_t N, int64_t npoint, const int64_t* start_idx,
             int64_t* out_idx, void* stream);

/* query_ball_point (pointnet2_encoder.py:47-59): first nsample in-radius indices in ascending
 * order, padded with the first; N when none.  Bit-exact. */
int pcst_ball_query(double radius, int64_t nsample, const float* xyz, const float* new_xyz,
                    int64_t B, int64_t N, int64_t S, int64_t* out_idx, void* stream);

/* SetAbstraction grouping (pointnet2_encoder.py:92-99): new_xyz = xyz[fps_idx];
 * grouped[b,s,k,:] = [xyz[g]-new_xyz[b,s] || feats[b,g,:]] with g = clamp(group_idx[b,s,k]).
 * feats may be NULL (C = 0).  Output [B,S,ns,3+C]. */
int pcst_group_gather(const float* xyz, const float* feats, int64_t B, int64_t N, int64_t C,
                      const int64_t* fps_idx, const int64_t* group_idx, int64_t S, int64_t ns,
                      float* new_xyz, float* grouped, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PCST_H_ */
