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
 *     thread-local last-error string (no setters, no environment variables:
 *     every choice a call makes is one of its arguments);
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

/* FPS with a caller workspace of pcst_fps_workspace_size() bytes (0 when a one-work-group
 * kernel applies): clouds larger than 30720 points keep their running distances there; for
 * 8192 < N <= 32768 with B * ceil(N / 1024) <= 32 (and npoint < 65536) it holds the round slots
 * of the multi-CU kernel, which spreads each cloud over ceil(N / 1024) work-groups (same bits as
 * pcst_fps; a cloud whose work-groups could not exchange within the poll bound gets -1 samples). */
int pcst_fps_workspace_size(int64_t B, int64_t N, size_t* bytes);
int pcst_fps_ws(const float* xyz, int64_t B, int64_t N, int64_t npoint, const int64_t* start_idx,
                int64_t* out_idx, void* workspace, void* stream);

/* SetAbstraction.apply_mlp layer (pointnet2_encoder.py:106-112) and other per-point linear
 * layers: Y[m,o] = act(scale[o]*(X[m,:].W[o,:]) + shift[o]) on exact-f32 MFMA, X [M,K],
 * W [O,K] (Conv2d 1x1 weight), scale/shift may be NULL (1/0).  pool_ns > 0: Y[g,o] = max over
 * rows g*ns..g*ns+ns-1 (torch.max(points, 3)); requires relu. */
int pcst_pointwise_linear(const float* X, int64_t M, int64_t K, const float* W, int64_t O,
                          const float* scale, const float* shift, int relu, int64_t pool_ns,
                          float* Y, void* stream);
/* Train-mode BatchNorm statistics of Z [M,O]: mean and biased variance per channel (float64),
 * deterministic.  workspace: pcst_channel_stats_workspace_size() bytes. */
int pcst_channel_stats_workspace_size(int64_t O, size_t* bytes);
int pcst_channel_stats(const float* Z, int64_t M, int64_t O, double* mean, double* var,
                       void* workspace, void* stream);
/* Y = act(scale*Z + shift) per channel, optional max-pool over groups of pool_ns rows. */
int pcst_affine_act(const float* Z, int64_t M, int64_t O, const float* scale, const float* shift,
                    int relu, int64_t pool_ns, float* Y, void* stream);

/* Training half of SetAbstraction (pointnet2_encoder.py:106-112 under autograd; replaces
 * F.batch_norm / F.relu / torch.max and the advanced-index backward on the trainer's path).
 * bn_train_coeffs: from the batch mean / biased var (pcst_channel_stats) -> scale =
 *   gamma/sqrt(var+eps), shift = beta - mean*scale (fp32, as F.batch_norm's affine), invstd
 *   (float64); updates running_mean / running_var in place with `momentum` (unbiased var) when
 *   they are non-NULL (BatchNorm2d train mode).
 * bn_relu_maxpool: Y [M/ns, O] = max over each group of ns rows of relu(scale*Z + shift) and
 *   arg [M/ns, O] = the group row of the maximum (the first on ties).
 * bn_relu_bwd: backward of relu(BN_train(Z)) (+ the max-pool when dY is NULL and dP/arg/ns
 *   are given): dZ [M,O], dgamma, dbeta [O] (may be NULL); deterministic (float64 chunk sums
 *   combined in order).  workspace: pcst_bn_relu_bwd_workspace_size() bytes.
 * group_gather_bwd: backward of pcst_group_gather's feature part: dpoints [B,N,C] =
 *   sum over the entries (s, k) with clamp(group_idx[b,s,k]) == n of dgrouped[b,s,k,3:];
 *   each destination sums in ascending entry order after a stable sort (deterministic). */
int pcst_bn_train_coeffs(const double* mean, const double* var, int64_t M, int64_t O,
                         const float* gamma, const float* beta, double eps, double momentum,
                         float* running_mean, float* running_var, float* scale, float* shift,
                         double* invstd, void* stream);
/* pcst_channel_stats followed by pcst_bn_train_coeffs in two launches instead of three (the
 * statistics' combine and the coefficients in one kernel), the same bits: mean / var (float64),
 * scale / shift / invstd and the running-stat update.  workspace:
 * pcst_channel_stats_workspace_size() bytes.  (Round 4.) */
int pcst_bn_train_stats(const float* Z, int64_t M, int64_t O, const float* gamma,
                        const float* beta, double eps, double momentum, float* running_mean,
                        float* running_var, double* mean, double* var, float* scale, float* shift,
                        double* invstd, void* workspace, void* stream);
int pcst_bn_relu_maxpool(const float* Z, int64_t M, int64_t O, const float* scale,
                         const float* shift, int64_t ns, float* Y, int32_t* arg, void* stream);
int pcst_bn_relu_bwd_workspace_size(int64_t O, size_t* bytes);
int pcst_bn_relu_bwd(const float* Z, int64_t M, int64_t O, const float* scale, const float* shift,
                     const double* mean, const double* invstd, const float* gamma, const float* dY,
                     const float* dP, const int32_t* arg, int64_t ns, float* dZ, float* dgamma,
                     float* dbeta, void* workspace, void* stream);
int pcst_group_gather_bwd_workspace_size(int64_t B, int64_t E, size_t* bytes);
int pcst_group_gather_bwd(const float* dgrouped, const int64_t* group_idx, int64_t B, int64_t S,
                          int64_t ns, int64_t N, int64_t C, float* dpoints, void* workspace,
                          void* stream);
/* Per-cloud column sums of a 16-bit matrix G [B*N, C] (f16 = 1: float16, 0: bfloat16 storage):
 * out [B, C] float32 = 16-bit-rounded float sum over cloud b's N rows -- autograd's reduction of
 * the broadcast time / style rows of x = (pf + tf) + sf under autocast (diffusion_model.py:56-58,
 * trainer.py:78-106 backward).  Deterministic (row slices combined in slice order); C % 8 == 0,
 * G 16-byte aligned.  workspace: pcst_group_colsum16_workspace_size() bytes. */
/* One residual block of NoisePredictorFn's 16-bit residual stream (diffusion_model.py:48-52,57-58
 * under autocast) in one launch: h [M,512] = 16-bit(relu(x W1^T + b1)), x_out [M,256] =
 * 16-bit(x + Dropout_p(h W2^T + b2)); x [M,256], W1 [512,256], W2 [256,512] in the 16-bit format
 * f16 selects (1 float16, 0 bfloat16), b1 / b2 fp32.  The bits of pcst_gemm_ex EP_BF16 followed
 * by EP_RESID_DROP16 with the same (seed, p); h is written for the backward but never re-read.
 * hbits (may be NULL): [M,16] uint32, bit j of word w of row m = [h[m, 32w + j] > 0] (the ReLU
 * mask the backward needs, 64 B per row instead of h's 1 KiB).
 * 16-byte aligned pointers, x_out != x, M * 1024 < 2^31. */
int pcst_resblock_fwd16(const uint16_t* x, int64_t M, const uint16_t* w1, const float* b1,
                        const uint16_t* w2, const float* b2, uint64_t seed, float drop_p,
                        uint16_t* h, uint16_t* x_out, uint32_t* hbits, int f16, void* stream);
/* The same block's backward products in one launch (the autograd backward of the block above,
 * trainer.py:106): dz [M,512] = 16-bit((dd W2) * [h > 0]), g_out [M,256] = 16-bit(g + dz W1) and,
 * if dd_out is not NULL, dd_out [M,256] = 16-bit(g_out keep / (1 - p)) with keep the dropout mask
 * of (seed, p) -- the previous block's, as pcst_gemm_ex's EP_ADD16 dropout copy.  w2t = W2^T
 * [512,256] and w1t = W1^T [256,512] in the 16-bit format.  The bits of pcst_gemm_ex EP_RELU_MASK
 * (aux h) followed by EP_ADD16 (aux g); dz is written for dW1 = dz^T x but never re-read here.
 * hbits (may be NULL): the forward's mask bits, read instead of h (h may then be NULL).
 * 16-byte aligned pointers, g_out != dd, dz != h, M * 1024 < 2^31. */
int pcst_resblock_bwd16(const uint16_t* dd, int64_t M, const uint16_t* w2t, const uint16_t* w1t,
                        const uint16_t* h, const uint16_t* g, uint64_t seed, float drop_p,
                        uint16_t* dz, uint16_t* g_out, uint16_t* dd_out, const uint32_t* hbits,
                        int f16, void* stream);
/* The step's 2-D fp32 weights to the 16-bit format f16 selects, n <= 64 tensors in one launch:
 * dst[i] = 16-bit(src[i]) [rows, cols] row-major, or its transpose [cols, rows] if transpose[i]
 * (round to nearest even, as torch's .to(dtype)).  Host arrays of n entries. */
int pcst_cast16_batch(const float* const* src, uint16_t* const* dst, const int32_t* rows,
                      const int32_t* cols, const int32_t* transpose, int n, int f16, void* stream);
int pcst_group_colsum16_workspace_size(int64_t B, int64_t C, size_t* bytes);
int pcst_group_colsum16(const uint16_t* G, int f16, int64_t B, int64_t N, int64_t C, float* out,
                        void* workspace, void* stream);

/* Weight / bias gradient of a per-point linear layer for the training path (autograd of
 * nn.Linear / Conv2d-1x1, trainer.py:106 backward): dW [O,I] = dZ^T X, db [O] = column sums of
 * dZ (db may be NULL), with dZ [M,O] and X [M,I] row-major.  Split over row chunks on exact-f32
 * MFMA, partials combined in chunk order in float64 (deterministic).
 * workspace: pcst_linear_wgrad_workspace_size() bytes. */
/* ReLU backward of the same layers: dz[i] = dy[i] * (y[i] > 0 ? 1 : 0), one pass. */
int pcst_relu_bwd(const float* dy, const float* y, int64_t n, float* dz, void* stream);
int pcst_linear_wgrad_workspace_size(int64_t M, int64_t I, int64_t O, size_t* bytes);
int pcst_linear_wgrad(const float* dZ, const float* X, int64_t M, int64_t I, int64_t O, float* dW,
                      float* db, void* workspace, void* stream);

/* 16-bit-MFMA variants for the training path under torch.autocast (trainer.py:81-106; the
 * reference's CUDA autocast runs Linear layers in half precision): operands are fp32 tensors
 * rounded in LDS to bf16 (f16 = 0) or fp16 (f16 = 1, torch's default CUDA autocast dtype),
 * accumulation and outputs fp32.
 * gemm_nt: C [M,O] = act(scale*(A [M,K] . B [O,K]^T) + shift) (scale/shift may be NULL).
 * linear_wgrad_bf16: as pcst_linear_wgrad (db from the unrounded fp32 dZ). */
int pcst_gemm_nt_bf16(const float* A, int64_t M, int64_t K, const float* B, int64_t O,
                      const float* scale, const float* shift, int relu, float* C, int f16,
                      void* stream);
int pcst_linear_wgrad_bf16_workspace_size(int64_t M, int64_t I, int64_t O, size_t* bytes);
int pcst_linear_wgrad_bf16(const float* dZ, const float* X, int64_t M, int64_t I, int64_t O,
                           float* dW, float* db, void* workspace, int f16, void* stream);

/* Training GEMMs with 16-bit activation storage and fused epilogues (csrc/train_mlp.hip): the
 * NoisePredictor residual block x + Dropout(Linear2(ReLU(Linear1(x)))) (diffusion_model.py:48-52,
 * 57-58) and its backward.  16-bit buffers are uint16_t raw bits, bfloat16 (f16 = 0) or IEEE
 * half (f16 = 1: the reference trainer's CUDA autocast dtype, trainer.py:50,78); "bf16" in the
 * names and flags below means "16-bit" in either format.  A [M,K] and B [O,K]
 * are fp32 (rounded to bf16 when staged) or bf16 per a_bf16/b_bf16; O % 4 == 0, K % 8 == 0 for a
 * bf16 operand (% 4 for fp32); all pointers 16-byte aligned.  epilogue:
 *   0 EP_F32         C fp32 = act(acc + bias)
 *   1 EP_BF16        C bf16 = act(acc + bias)
 *   2 EP_RESID_DROP  C fp32 = aux_fp32 + keep(e) * (acc + bias) / (1 - drop_p)
 *   3 EP_RELU_MASK   C bf16 = acc * [aux_bf16 > 0]
 *   4 EP_ADD         C fp32 = acc + aux_fp32
 *   5 EP_COND        C fp32 = ((acc + bias) + aux[g,0,:]) + aux[g,1,:],  g = m / group_rows
 *   6 EP_RESID_DROP16 C bf16 = aux_bf16 + keep(e) * (acc + bias) / (1 - drop_p)
 *   7 EP_ADD16       C bf16 = acc + aux_bf16
 *     (6, 7: the residual stream in the autocast format, as the reference's autocast keeps it)
 * C2 (may be NULL): bf16 copy of an fp32 C (EP_F32, EP_RESID_DROP, EP_COND -- C may then be NULL
 * for EP_COND), or for EP_BF16 / EP_ADD16 the next Dropout backward fused: C2 = bf16(C * keep(e)
 * / (1 - drop_p)) from the stored bf16 C, pcst_dropout_grad_bf16's result on it (those two
 * epilogues apply no dropout of their own).  O % 4 == 0 except for EP_F32/EP_BF16.
 * keep(e) for element e = m*O + o is hash(seed, e) >= drop_p * 2^32: a pure function of
 * (seed, e), regenerated by pcst_dropout_grad_bf16 (out bf16 = g * keep * 1/(1-p), n % 4 == 0).
 * bf16 A with bf16 B runs the pipelined kernel (64-deep K slices, two in flight). */
int pcst_gemm_ex(const void* A, int a_bf16, int64_t M, int64_t K, const void* B, int b_bf16,
                 int64_t O, const float* bias, int relu, int epilogue, const void* aux,
                 uint64_t seed, float drop_p, int64_t group_rows, void* C, uint16_t* C2, int f16,
                 void* stream);
int pcst_dropout_grad_bf16(const float* g, int64_t n, uint64_t seed, float drop_p, uint16_t* out,
                           int f16, void* stream);
/* dW [O,I] = dZ^T X, db [O] = column sums of dZ (may be NULL), dZ [M,O] / X [M,I] fp32 or bf16;
 * I % 8 == 0, O % 8 == 0.  Deterministic (chunk partials combined in order). */
int pcst_linear_wgrad_ex_workspace_size(int64_t M, int64_t I, int64_t O, size_t* bytes);
int pcst_linear_wgrad_ex(const void* dZ, int dz_bf16, const void* X, int x_bf16, int64_t M,
                         int64_t I, int64_t O, float* dW, float* db, void* workspace, int f16,
                         void* stream);

/* ---- models/diffusion_model.py --------------------------------------------------------- */

/* HierarchicalProcessor._voxel_grid_downsample_torch (diffusion_model.py:69-122) for all B
 * clouds (N > target) on the device.  Split into stats (unique voxels U, pool size P; written
 * to counts_out[0..B) and [B..2B) if non-NULL) and select.  select with perm == NULL draws the
 * random subset on the device from `seed` (random keys + sort, torch.randperm's construction);
 * with perm != NULL it replays per-cloud permutations (perm + perm_off[b], length perm_len[b]
 * must be U when U > target, P when U < target, 0 when U == target).
 * Outputs: out_idx [B,target] int64, out_pts [B,target,3]. */
int pcst_voxel_workspace_size(int64_t B, int64_t N, size_t* bytes);
int pcst_voxel_stats(const float* pts, int64_t B, int64_t N, int64_t target, void* workspace,
                     int32_t* counts_out, void* stream);
int pcst_voxel_select(const float* pts, int64_t B, int64_t N, int64_t target, void* workspace,
                      const int64_t* perm, const int64_t* perm_off, const int64_t* perm_len,
                      uint64_t seed, int64_t* out_idx, float* out_pts, void* stream);
int pcst_voxel_downsample(const float* pts, int64_t B, int64_t N, int64_t target, void* workspace,
                          uint64_t seed, int64_t* out_idx, float* out_pts, void* stream);
/* The device-drawn downsample of cat([pts] * copies) (the CFG batch of guided_sample_loop,
 * diffusion_model.py:244-247) from the B distinct clouds: the voxel table and representatives
 * are built once per cloud, the subset is drawn per row (row = c*B + b) with the row's own keys,
 * so every row keeps the same set as pcst_voxel_downsample on the concatenated batch with the
 * same seed.  out_idx [copies*B,target], out_pts [copies*B,target,3]. */
int pcst_voxel_copies_workspace_size(int64_t B, int64_t N, int64_t copies, size_t* bytes);
int pcst_voxel_downsample_copies(const float* pts, int64_t B, int64_t N, int64_t copies,
                                 int64_t target, void* workspace, uint64_t seed, int64_t* out_idx,
                                 float* out_pts, void* stream);
/* The sampling step's CFG + DDIM update (pcst_cfg_ddim_step over a CFG batch: eps [2C,N,3] whose
 * rows c and C + c are cloud c's conditional and unconditional eps; source [C,N,3] or NULL; x_out
 * [C,N,3] and x_cat [2C,N,3] = the new x and the next CFG batch) fused with the first stage of the
 * next downsample of x_out on vox_workspace (a pcst_voxel_copies_workspace_size(C, N, copies)
 * workspace): the new points' min / max partials and the zeroing of the per-call state.  The next
 * call on that workspace must then be pcst_voxel_downsample_copies_prepped with pts = x_out (the
 * same arguments as pcst_voxel_downsample_copies, one launch fewer; the same result bit for bit).
 * pool != 0 (N <= 4M): the update also makes that downsample's pool-key histogram for the seed
 * pool_seed it will be called with (the keys depend on (seed, row, index) only), which the
 * downsample's insert otherwise makes on the step's critical path; that call must then pass
 * pool = 1 and seed = pool_seed.  A pool prep adds into the workspace's pool histogram, which only
 * that downsample clears (its emit, after reading it): every pool prep must be followed by its
 * matching prepped downsample on the same workspace before the next prep, or the histogram keeps
 * stale counts (a caller whose step raised in between must re-zero the workspace). */
int pcst_cfg_ddim_voxel_prep(const float* x, const float* eps, const float* source, int64_t C,
                             int64_t N, float guidance_scale, float sqrt_1m_at, float sqrt_at_eps,
                             float sqrt_aprev, float sqrt_1m_aprev, float* x_out, float* x_cat,
                             void* vox_workspace, int64_t copies, uint64_t pool_seed, int pool,
                             void* stream);
/* start_flag (NULL: none): written with start_value as the downsample's first launch begins,
 * i.e. once every launch ahead of it on `stream` has completed -- the pts are final -- for work
 * on another stream that waits for it (the sampling step's kNN rows build, pcst_signal_wait). */
int pcst_voxel_downsample_copies_prepped(const float* pts, int64_t B, int64_t N, int64_t copies,
                                         int64_t target, void* workspace, uint64_t seed, int pool,
                                         int64_t* out_idx, float* out_pts, uint32_t* start_flag,
                                         uint32_t start_value, void* stream);
/* The device-drawn downsample of the CFG batch (pcst_voxel_downsample_copies, or _prepped with
 * prepped = 1: pool and start_flag as there) that also places its coarse points as the refs of the
 * kNN rows layout (phase B of pcst_knn3_rows_refs, inside the emit launch): knn_workspace is the
 * rows workspace of B clouds x copies rows with M = target that pcst_knn3_rows_build is binning
 * (on another stream); every emit work-group first writes its rows of out_idx / out_pts, then
 * waits for wait_flag >= wait_value (the build's refs flag; NULL: the stream is ordered after the
 * build already), at most max_polls polls (<= 0: ~10 s), and places its kept points -- the same
 * placement as pcst_knn3_rows_refs(out_idx).  That in-launch wait is used only while the emit
 * launch has at most one work-group per CU (one cloud: 236), so waiting work-groups never hold
 * every CU while the build still needs some; a larger emit launch places nothing itself and is
 * followed by pcst_knn3_rows_refs's own launch (the same wait, at most max(CUs, rows)
 * work-groups).  A work-group whose wait gives up places nothing and sets *wait_err: pass it to
 * pcst_knn3_rows_query as refs_err. */
int pcst_voxel_downsample_rows(const float* pts, int64_t B, int64_t N, int64_t copies,
                               int64_t target, void* workspace, uint64_t seed, int prepped,
                               int pool, int64_t* out_idx, float* out_pts, uint32_t* start_flag,
                               uint32_t start_value, void* knn_workspace, const uint32_t* wait_flag,
                               uint32_t wait_value, int32_t* wait_err, int64_t max_polls,
                               void* stream);
/* Copies the replay-validation error word (0 = ok) to err_out (device int32). */
int pcst_voxel_error(void* workspace, int64_t B, int64_t N, int32_t* err_out, void* stream);

/* HierarchicalProcessor.upsample_knn (diffusion_model.py:127-153): coarse [B,M,3] values at
 * orig[idx] ([B,M] int64), orig [B,N,3] -> out [B,N,3]; exact float64 3-NN IDW (bit-exact vs
 * the reference's sklearn KD-tree path). */
int pcst_knn_workspace_size(int64_t B, int64_t N, int64_t M, size_t* bytes);
int pcst_knn3_interp(const float* coarse, const float* orig, const int64_t* idx, int64_t B,
                     int64_t N, int64_t M, float* out, void* workspace, void* stream);
/* The same computation in two phases on one workspace (knn3_interp = build then query):
 * build reads only positions (orig, idx) -- the grid statistics, cell counts, scan and fill --
 * so it can run on a second stream while the noise MLP produces `coarse`; query reads `coarse`
 * and writes out.  The caller orders query after build on the workspace.
 * lds_floor (bytes, 0..96 KiB): LDS floor of the build-phase workgroups (a kernel whose static LDS
 * is below it gets the difference as dynamic LDS), so that a build on a side stream runs only on
 * CUs the noise MLP leaves idle; 0 = no floor (knn3_interp passes 0).  max_wg (> 0): at most
 * this many workgroups per build launch over all clouds (each kernel strides over its work), so a
 * side-stream build holds few CUs; 0 = the natural grids (knn3_interp passes 0).
 * built_flag / built_value (query; NULL: none): the flag the build's
 * producer publishes (pcst_signal_write) -- the consumer reads the workspace only if the flag
 * holds the value when its work-groups start; otherwise (a cross-stream wait that gave up) it
 * leaves the workspace alone and writes 0 for eps, so a timed-out wait can never make it read a
 * half-built workspace.  The caller reports the wait's error word.
 * grid_cap (query): at most this many query work-groups over all clouds of the launch (the result
 * does not depend on it); <= 0: the resident grid (4 work-groups per CU).  The query's waves are
 * persistent: a wave's first chunk is its index, the next ones come from work counters of its CFG
 * row (eight per row), which the build zeroes and the query's outlier launch zeroes again. */
int pcst_knn3_build(const float* orig, const int64_t* idx, int64_t B, int64_t N, int64_t M,
                    int64_t lds_floor, int64_t max_wg, void* workspace, void* stream);
int pcst_knn3_query(const float* coarse, const float* orig, int64_t B, int64_t N, int64_t M,
                    float* out, void* workspace, const uint32_t* built_flag, uint32_t built_value,
                    int64_t grid_cap, void* stream);
/* diagnostics of the last query on a workspace: out[0] error flag, out[1..B] query chunks per
 * cloud, out[1+B..2B] outlier queries per cloud (device int32 buffer of 1 + 2B) */
int pcst_knn_stats(void* workspace, int64_t B, int64_t N, int64_t M, int32_t* out, void* stream);
int pcst_knn_error(void* workspace, int64_t B, int64_t N, int64_t M, int32_t* err_out,
                   void* stream);
/* The same upsample in the rows layout (the sampling step's): the CFG batch's B = C * copies rows,
 * row b a copy of cloud b % C of x [C,N,3] (guided_sample_loop's cat([x, x])).
 *   rows_build (positions of x only, before the coarse indices exist): every point of every
 *     cloud binned by cell -- the grid statistics (those of pcst_knn3_build, sized for M refs),
 *     per-cell counts, scan, the query chunks over all points, the points in cell order.
 *     refs_flag / done_flag (NULL: none): written with their values once rows_refs may run on
 *     another stream (after the scan) and once the whole build is done (after the fill);
 *   rows_refs (idx [B,M] int64), one launch: each ref marks its point known (the last j wins),
 *     takes a rank in its point's cell and the slot start(cell) + rank at the front of the cell's
 *     row range (the build marks every slot empty first); a ref beyond its cell's rows (repeated
 *     indices piling up) goes to the row's overflow list, which the query offers wherever its
 *     scanned box holds them.  wait_flag (NULL: none): the kernel first waits, in every
 *     work-group, until the flag holds wait_value (the side stream's pcst_signal_write after
 *     rows_build), at most max_polls polls (<= 0: ~10 s); a work-group whose wait gives up sets
 *     *wait_err and writes nothing (pass wait_err to rows_query as refs_err).  At most max(CUs,
 *     B) work-groups (each strides over its row's refs), so the waiting ones leave CUs free;
 *   rows_query (coarse [B,M,3] -> out [B,N,3]): the query and outlier passes of pcst_knn3_query
 *     over every point, known points copying their coarse value; built_flag (the build's
 *     done_flag) with wait_err: a one-work-group wait launch (pcst_signal_wait) precedes the query
 *     (the query's resident grid never waits itself: it would hold the CUs the build needs); with
 *     wait_err == NULL the stream has already waited for it (e.g. pcst_noise_mlp_ex's wait in the
 *     MLP launch before the query); either way the work-groups check the flag (short of
 *     built_value: eps = 0, nothing read); refs_err (NULL: none): the
 *     rows_refs wait's error word -- nonzero: eps = 0, nothing read; grid_cap as pcst_knn3_query.
 * Same bits as pcst_knn3_interp on cat([x] * copies).  An index outside [0, N) sets bit 1 of the
 * error word, a chunk or ref range outside the workspace's arrays bits 4 / 8 (the range is then
 * skipped, never read); pcst_knn_rows_stats copies out[0] = error word, out[1..C] chunks per
 * cloud, out[1+C..C+B] outlier queries, out[1+C+B..C+2B] overflow refs per row. */
int pcst_knn_rows_workspace_size(int64_t C, int64_t copies, int64_t N, int64_t M, size_t* bytes);
int pcst_knn3_rows_build(const float* x, int64_t C, int64_t copies, int64_t N, int64_t M,
                         void* workspace, uint32_t* refs_flag, uint32_t refs_value,
                         uint32_t* done_flag, uint32_t done_value, void* stream);
int pcst_knn3_rows_refs(const float* x, const int64_t* idx, int64_t C, int64_t copies, int64_t N,
                        int64_t M, void* workspace, const uint32_t* wait_flag, uint32_t wait_value,
                        int32_t* wait_err, int64_t max_polls, void* stream);
int pcst_knn3_rows_query(const float* coarse, const float* x, int64_t C, int64_t copies, int64_t N,
                         int64_t M, float* out, void* workspace, const uint32_t* built_flag,
                         uint32_t built_value, int32_t* wait_err, int64_t max_polls,
                         const int32_t* refs_err, int64_t grid_cap, void* stream);
int pcst_knn_rows_stats(void* workspace, int64_t C, int64_t copies, int64_t N, int64_t M,
                        int32_t* out, void* stream);

/* NoisePredictor.forward (diffusion_model.py:38-61), fused.  precision: 0 = exact f32 MFMA
 * (v_mfma_f32_32x32x2_f32, the parity mode); 1 = bf16 operands on v_mfma_f32_16x16x32_bf16 with
 * fp32 accumulation and an fp32 residual stream (the product mode).  blob/bias are the packed
 * weights of packing.py for that precision (blob 16-byte aligned, pcst_noise_mlp_blob_bytes()
 * bytes; -1 for any other precision).  Any other precision is PCST_EINVAL (codes 2 and 3 of
 * rounds 2-4 are retired).
 * pcst_noise_cond computes cond[c] = b4 + time_proj(TimeEmbedding(t_c)) + style_proj(style_c)
 * (freqs = the reference's 64-entry exp table; wt = time_proj.weight^T [128,256] and
 * ws = style_proj.weight^T [256,256], transposed for coalesced reads).  pts [P,3] cloud-major with
 * points_per_cloud points per cloud; out [P,3]. */
int64_t pcst_noise_mlp_blob_bytes(int precision);
int pcst_noise_cond(const int64_t* t, const float* style, int64_t nclouds, const float* freqs,
                    const float* wt, const float* bt, const float* ws, const float* bs,
                    const float* b4, float* cond, void* stream);
int pcst_noise_mlp(const float* pts, int64_t P, int64_t points_per_cloud, const float* cond,
                   int64_t nclouds, const void* blob, int64_t blob_bytes, const float* bias,
                   int precision, float* out, void* stream);
/* pcst_noise_mlp with optional cross-stream signalling folded into the launch (all optional):
 * start_flag: *start_flag = start_value (agent-scope store) as the launch begins, i.e. once every
 * kernel queued before it on `stream` has completed -- the producer side of pcst_signal_wait
 * without a pcst_signal_write launch; start_counter (with start_flag; a caller-owned uint32 that
 * is zero before the call and zero again after it): the store happens once EVERY work-group of
 * the launch has begun instead (precision 0: once the launch has completed), so work another
 * stream starts behind the flag only finds the CUs the MLP leaves idle; wait_flag: the launch completes only once *wait_flag >=
 * wait_value as well -- after writing its rows, the MLP's last work-group (counted out by
 * wait_counter, a caller-owned uint32 that is zero before the call and zero again after it) polls
 * the flag with agent-scope loads (the producer on another stream writes it with
 * pcst_signal_write), at most max_polls times (<= 0: ~10 s; then *wait_err = 1 and the launch
 * completes anyway: the caller must read it); work queued after it on the stream is then ordered
 * after the flag's producer without a wait launch.  Precision 1 folds both into the MLP kernel;
 * precision 0 uses separate one-lane launches (same ordering). */
int pcst_noise_mlp_ex(const float* pts, int64_t P, int64_t points_per_cloud, const float* cond,
                      int64_t nclouds, const void* blob, int64_t blob_bytes, const float* bias,
                      int precision, float* out, uint32_t* start_flag, uint32_t start_value,
                      uint32_t* start_counter, const uint32_t* wait_flag, uint32_t wait_value,
                      uint32_t* wait_counter,
                      int32_t* wait_err, int64_t max_polls, void* stream);

/* CFG + DDIM update of guided_sample_loop (diffusion_model.py:248-260); eps_u == NULL gives
 * ddim_sample_loop's update (:283-290), source == NULL skips the source pull.  x_cat (optional,
 * [2,n]) receives the new x twice: the next step's CFG batch. */
int pcst_cfg_ddim_step(const float* x, const float* eps_c, const float* eps_u, const float* source,
                       int64_t n, float guidance_scale, float sqrt_1m_at, float sqrt_at_eps,
                       float sqrt_aprev, float sqrt_1m_aprev, float* x_out, float* x_cat,
                       void* stream);
/* hipGraph-replayable forms of the per-step calls (BASELINE configs[4]: a captured denoise
 * step): the per-step scalars live in device memory the caller updates between replays --
 * coef_dev[4] = (sqrt_1m_at, sqrt_at_eps, sqrt_aprev, sqrt_1m_aprev); seed_dev[1] the subset
 * seed.  x_out may equal x (elementwise, in place). */
int pcst_cfg_ddim_step_dcoef(const float* x, const float* eps_c, const float* eps_u,
                             const float* source, int64_t n, float guidance_scale,
                             const float* coef_dev, float* x_out, float* x_cat, void* stream);
int pcst_voxel_downsample_copies_dseed(const float* pts, int64_t B, int64_t N, int64_t copies,
                                       int64_t target, void* workspace, const uint64_t* seed_dev,
                                       int64_t* out_idx, float* out_pts, void* stream);

/* ---- models/losses.py ------------------------------------------------------------------ */

/* chamfer_distance_chunked_optimized (losses.py:8-63), never materialising N x M:
 * min1/arg1 [B,N] = row minima pred->target of clamp((|p|^2+|q|^2) + (-2 p.q), 0) (first index
 * on ties), min2/arg2 [B,M] target->pred, out [B] = mean(min1) + mean(min2) (may be NULL).
 * workspace: the clouds repacked as point pairs (exhaustive row-min) or counting-sorted into
 * uniform grids (grid-pruned row-min). */
int pcst_chamfer_fwd_workspace_size(int64_t B, int64_t N, int64_t M, size_t* bytes);
/* mode: 0 default (= 3), 1 exhaustive, 2 grid-pruned (fast for overlapping clouds, slow for
 * rows far outside the other cloud), 3 hybrid (the grid search under a ring budget; the rows
 * over it go to a box-pruned search over 64-point runs of the sorted cloud, one wave per row:
 * faster than 1 on every measured cloud pair, about as fast as 2 on overlapping clouds); all
 * give bit-identical minima and first-index argmins. */
int pcst_chamfer_fwd(const float* pred, const float* target, int64_t B, int64_t N, int64_t M,
                     float* min1, int32_t* arg1, float* min2, int32_t* arg2, float* out, int mode,
                     void* workspace, void* stream);
/* Gradient of sum_b grad_out[b]*chamfer[b]; ACCUMULATES into grad_pred [B,N,3] and/or
 * grad_target [B,M,3] (either may be NULL).  Deterministic (sorted scatter, no float atomics). */
int pcst_chamfer_bwd_workspace_size(int64_t B, int64_t N, int64_t M, size_t* bytes);
int pcst_chamfer_bwd(const float* pred, const float* target, int64_t B, int64_t N, int64_t M,
                     const int32_t* arg1, const int32_t* arg2, const float* grad_out,
                     float* grad_pred, float* grad_target, void* workspace, void* stream);

/* F.l1_loss mean reduction (losses.py:90): out[0] = mean|a-b| (fixed-order float64 sum);
 * backward grad_a = sign(a-b) * grad_out[0] / n. */
int pcst_l1_workspace_size(size_t* bytes);
int pcst_l1_fwd(const float* a, const float* b, int64_t n, float* out, void* workspace,
                void* stream);
int pcst_l1_bwd(const float* a, const float* b, int64_t n, const float* grad_out, float* grad_a,
                void* stream);

/* ---- data/preprocessing.py (offline) ------------------------------------------------------ */

/* Per-point part of PointCloudPreprocessor._voxel_grid_downsample_numpy (preprocessing.py:45-104):
 * key [n] = voxel coordinates floor(f32(f32(p - min) / voxel_size)) packed 21 bits per axis,
 * dist [n] = float64 distance to the voxel centre min + (coord + 0.5) * voxel_size.  xyz_min is a
 * HOST pointer (3 floats); *overflow (device int, zeroed by the caller) is set when a coordinate
 * leaves [0, 2^21). */
int pcst_voxel_center_dist(const float* pts, int64_t n, const float* xyz_min, float voxel_size,
                           int64_t* key, double* dist, int* overflow, void* stream);

/* ---- evaluation/metrics.py, compare.py (measurement only) -------------------------------- */

/* K nearest rows of Q [B,M,3] for every row of P [B,N,3] (1 <= k <= 16): dist [B,N,k] float64
 * Euclidean distances, ascending (ties to the lower index), idx [B,N,k] int32 (may be NULL).
 * Replaces torch.cdist + min (metrics.py:31-41,100-104), sklearn NearestNeighbors
 * (metrics.py:124-127,146-148) and cKDTree.query (compare.py:22-34). */
int pcst_knn_dist(const float* P, const float* Q, int64_t B, int64_t N, int64_t M, int64_t k,
                  double* dist, int32_t* idx, void* stream);
/* earth_mover_distance's greedy matching (metrics.py:46-90), bit-exact: out [B] float32 =
 * (sum over i in order of the nearest unused target's float64 distance) / N.  M <= 262144. */
int pcst_emd_greedy(const float* P, const float* Q, int64_t B, int64_t N, int64_t M, float* out,
                    void* stream);

/* Stream-ordering events with device-scope fences only (hipEventDisableSystemFence; timing = 0
 * also disables timing).  Used by the Python host for the sampling loop's cross-stream
 * dependencies and the bench's kernel timing; plain HIP, no kernel. */
int pcst_event_create(int timing, void** event);
int pcst_event_destroy(void* event);
int pcst_event_record(void* event, void* stream);
int pcst_stream_wait_event(void* stream, void* event);
int pcst_event_elapsed_ms(void* start, void* end, float* ms);

/* Kernel-side stream signal: a one-lane kernel on `stream` publishes *flag = value (agent-scope
 * release, after everything enqueued before it on that stream); pcst_signal_wait enqueues a
 * one-workgroup kernel that polls *flag until it is >= value (agent-scope acquire), so the
 * work enqueued after it on ITS stream starts after the signal.  A cross-stream dependency
 * without an event marker on the producer's queue (an event that another queue waits on costs
 * that queue ~17 us; this ~3 us, tools/sync_probe.hip).  The wait gives up after max_polls polls
 * (<= 0: the default, ~10 s) and then sets *err = 1 (err may be NULL) and lets its stream go on:
 * the caller must read *err after the stream's work (the Python host raises, _hip.DeviceSignal).
 * Values must grow monotonically per flag.  flag: one uint32 of device memory, zero-initialised
 * by the caller. */
int pcst_signal_write(uint32_t* flag, uint32_t value, void* stream);
int pcst_signal_wait(const uint32_t* flag, uint32_t value, int32_t* err, int64_t max_polls,
                     void* stream);

/* Caller-owned streams for the sampling loop (one pair per loop invocation / host thread, so two
 * loops on one device never share a queue).  priority < 0: the device's greatest priority, else
 * its default; non-blocking w.r.t. the null stream.  Plain HIP, no kernel. */
int pcst_stream_create(int priority, void** stream);
int pcst_stream_destroy(void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PCST_H_ */
