// Fused per-point noise-prediction MLP of NoisePredictor.forward
// (models/diffusion_model.py:38-61) on MFMA, one launch for the whole stack:
//   h1 = relu(W0 p + b0)            3 -> 128       (VALU: K = 3)
//   h2 = relu(W2 h1 + b2)           128 -> 256     (MFMA)
//   x  = W4 h2 + cond[cloud]        256 -> 256     cond = b4 + time_proj(emb(t)) + style_proj(s)
//   6x x += W2_i relu(W1_i x + b1_i) + b2_i        256 -> 512 -> 256 (hidden streamed in 32-row chunks)
//   o  = W_o4 relu(W_o2 relu(W_o0 x + b) + b) + b  256 -> 256 -> 128 -> 3
//
// Layout: features on MFMA rows, points on MFMA columns (lanes).  A 32x32 accumulator of
// v_mfma_f32_32x32x16_bf16 / v_mfma_f32_32x32x2_f32 holds 32 features of 32 points with the
// point on the lane, so it is (after bias/ReLU and, for bf16, cvt_pk) directly the B operand
// of the next layer -- no LDS round trip between layers.  The k-order this induces is
// absorbed by the host-side weight packing (packing.py), which also lays every A fragment
// out as one contiguous 1 KiB (bf16) / 256 B (f32) block in streaming order.
//
// Weights stream through LDS in 32 KiB parts (double-buffered, global_load_lds 16 B/lane),
// shared by all waves of the workgroup; bias tables and the per-cloud cond rows sit in LDS.
// bf16 mode: 8 waves x 32 points per workgroup (2 waves/SIMD), fp32 accumulate, fp32 residual.
// f32 mode (parity): exact-f32 MFMA, 4 waves x 32 points (1 wave/SIMD).
#include "common.h"

namespace pcst {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int kPart = 32768;  // bytes per streamed weight part
// bias table offsets (floats) -- must match packing.py
constexpr int kOffW0 = 0, kOffB0 = 384, kOffB2 = 512, kOffB1 = 768, kOffBB2 = 3840,
              kOffO0 = 5376, kOffO2 = 5632, kOffO4 = 5760, kBiasFloats = 5792;
constexpr int kCondSlots = 4;

struct TrBF16 {
  static constexpr int KS = 16;          // K per MFMA
  static constexpr int FRAG = 1024;      // bytes per A fragment
  static constexpr int OPB = 2;          // operands per 32-row block
  static constexpr int THREADS = 256;
  using A = bf16x8;
  using Op = bf16x8;
  __device__ static f32x16 mfma(A a, Op b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  // registers 8s..8s+7 of a C block -> operand s of that block (element j <-> row
  // 16s + 8(j>>2) + 4h + (j&3), absorbed by the weight packing)
  __device__ static void to_op(const float (&v)[16], Op* o) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      Op t;
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = (__bf16)v[8 * s + j];
      o[s] = t;
    }
  }
};

struct TrF32 {
  static constexpr int KS = 2;
  static constexpr int FRAG = 256;
  static constexpr int OPB = 16;
  static constexpr int THREADS = 256;
  using A = float;
  using Op = float;
  __device__ static f32x16 mfma(A a, Op b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
  // register r of a C block is the operand of k-step r (rows (r&3)+8(r>>2)+4h)
  __device__ static void to_op(const float (&v)[16], Op* o) {
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = v[r];
  }
};

// row of accumulator register r for lane half h inside a 32-row block
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <class TR>
struct Streamer {
  const char* blob;
  char* lds;  // two kPart buffers
  int part;   // part being computed
  int nparts;
  __device__ void issue(int q) {
    if (q >= nparts) return;
    constexpr int waves = TR::THREADS / 64;
    constexpr int per_wave = kPart / 1024 / waves;  // 1 KiB wave-instructions per wave
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    char* dst = lds + (q & 1) * kPart;
    const char* src = blob + (int64_t)q * kPart;
#pragma unroll
    for (int i = 0; i < per_wave; ++i) {
      const int chunk = w * per_wave + i;
      __builtin_amdgcn_global_load_lds((const void*)(src + chunk * 1024 + lane * 16),
                                       (__attribute__((address_space(3))) void*)(dst + chunk * 1024),
                                       16, 0, 0);
    }
  }
  __device__ void begin() {  // part 0 resident, part 1 in flight
    issue(0);
    __syncthreads();
    issue(1);
  }
  __device__ void next() {  // finish `part`, make part+1 resident, prefetch part+2
    __syncthreads();
    ++part;
    issue(part + 1);
  }
  __device__ typename TR::A frag(int f) const {  // fragment f of the current part
    const char* p = lds + (part & 1) * kPart + f * TR::FRAG +
                    (threadIdx.x & 63) * (int)sizeof(typename TR::A);
    return *reinterpret_cast<const typename TR::A*>(p);
  }
};

// acc = sum_s A(frag base+s) * in[s] for s in [S, NS): compile-time recursion so every
// operand register index is static (a runtime index would send the operands to scratch).
template <class TR, int S, int NS>
struct KSteps {
  __device__ static __forceinline__ void run(const Streamer<TR>& st, int base,
                                             const typename TR::Op* in, f32x16& acc) {
    acc = TR::mfma(st.frag(base + S), in[S], acc);
    KSteps<TR, S + 1, NS>::run(st, base, in, acc);
  }
};
template <class TR, int NS>
struct KSteps<TR, NS, NS> {
  __device__ static __forceinline__ void run(const Streamer<TR>&, int, const typename TR::Op*,
                                             f32x16&) {}
};

// Dense layer over NOB output blocks with K = KB 32-row input blocks.  Every layer starts on a
// fresh part (the packing pads each layer to whole parts); inside a layer a part holds
// FPP/NS whole output blocks.
template <class TR, int NOB, int KB>
__device__ __forceinline__ void dense(Streamer<TR>& st, const typename TR::Op* in, f32x16* acc) {
  constexpr int NS = KB * TR::OPB;
  constexpr int FPP = kPart / TR::FRAG;
  constexpr int OBPP = FPP / NS;
  static_assert(OBPP >= 1 && FPP % NS == 0, "part must hold whole output blocks");
#pragma unroll
  for (int ob = 0; ob < NOB; ++ob) {
    if (ob > 0 && ob % OBPP == 0) st.next();
    KSteps<TR, 0, NS>::run(st, (ob % OBPP) * NS, in, acc[ob]);
  }
}

template <class TR>
__device__ __forceinline__ void epilogue_op(const f32x16& acc, const float* bias, int h, bool relu,
                                            typename TR::Op* out) {
  float v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float x = acc[r] + bias[crow(r, h)];
    v[r] = relu ? fmaxf(x, 0.0f) : x;
  }
  TR::to_op(v, out);
}

template <class TR>
__global__ __launch_bounds__(TR::THREADS) void noise_mlp_kernel(
    const float* __restrict__ pts, int64_t P, int64_t T, const float* __restrict__ cond,
    int64_t nclouds, const char* __restrict__ blob, int nparts, const float* __restrict__ bias,
    float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sb = reinterpret_cast<float*>(smem + 2 * kPart);
  float* sc = sb + kBiasFloats;  // kCondSlots x 256
  using Op = typename TR::Op;
  constexpr int PTS = TR::THREADS / 64 * 32;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5;
  const int64_t p0 = (int64_t)blockIdx.x * PTS;
  const int64_t c0 = p0 / T;
  for (int i = tid; i < kBiasFloats; i += TR::THREADS) sb[i] = bias[i];
  for (int i = tid; i < kCondSlots * 256; i += TR::THREADS) {
    const int64_t c = c0 + i / 256;
    sc[i] = c < nclouds ? cond[c * 256 + (i % 256)] : 0.0f;
  }
  const int64_t p = p0 + wid * 32 + (lane & 31);
  const bool valid = p < P;
  const int64_t pc = valid ? p : (P - 1);
  const float px = pts[pc * 3 + 0], py = pts[pc * 3 + 1], pz = pts[pc * 3 + 2];
  const int64_t myc = pc / T;
  const int slot = (int)(myc - c0);
  __syncthreads();

  // ---- h1 = relu(W0 p + b0), 128 rows, VALU, straight into operand form
  Op h1[4 * TR::OPB];
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) {
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = ob * 32 + crow(r, h);
      float x = sb[kOffB0 + row];
      x = fmaf(sb[kOffW0 + row * 3 + 0], px, x);
      x = fmaf(sb[kOffW0 + row * 3 + 1], py, x);
      x = fmaf(sb[kOffW0 + row * 3 + 2], pz, x);
      v[r] = fmaxf(x, 0.0f);
    }
    TR::to_op(v, &h1[ob * TR::OPB]);
  }

  Streamer<TR> st{blob, smem, 0, nparts};
  st.begin();
  f32x16 acc[8];
  Op xb[8 * TR::OPB];

  // ---- h2 = relu(W2 h1 + b2)
#pragma unroll
  for (int ob = 0; ob < 8; ++ob) acc[ob] = f32x16{};
  dense<TR, 8, 4>(st, h1, acc);
#pragma unroll
  for (int ob = 0; ob < 8; ++ob) epilogue_op<TR>(acc[ob], sb + kOffB2 + ob * 32, h, true, &xb[ob * TR::OPB]);

  // ---- x = W4 h2 + cond[cloud]   (cond already contains b4)
  f32x16 x[8];
#pragma unroll
  for (int ob = 0; ob < 8; ++ob) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = ob * 32 + crow(r, h);
      x[ob][r] = (slot >= 0 && slot < kCondSlots) ? sc[slot * 256 + row] : cond[myc * 256 + row];
    }
  }
  {
    Op h2[8 * TR::OPB];
#pragma unroll
    for (int i = 0; i < 8 * TR::OPB; ++i) h2[i] = xb[i];
    st.next();
    dense<TR, 8, 8>(st, h2, x);
  }
#pragma unroll
  for (int ob = 0; ob < 8; ++ob) {
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = x[ob][r];
    TR::to_op(v, &xb[ob * TR::OPB]);
  }

  // ---- 6 residual blocks, hidden 512 streamed in 16 chunks of 32 rows.  Per chunk the
  // packing holds W1 rows [32c, 32c+32) (all K) then W2 columns [32c, 32c+32) (all 8 output
  // blocks): one part in bf16, two parts (W1 | W2) in f32.
  constexpr int FPP = kPart / TR::FRAG;
  constexpr int NSX = 8 * TR::OPB;                  // k-steps over x (K = 256)
  constexpr bool W2_OWN_PART = (NSX + 8 * TR::OPB) > FPP;
  for (int layer = 0; layer < 6; ++layer) {
    const float* b1 = sb + kOffB1 + layer * 512;
    const float* b2 = sb + kOffBB2 + layer * 256;
    for (int c = 0; c < 16; ++c) {
      st.next();
      f32x16 hc = f32x16{};
      KSteps<TR, 0, NSX>::run(st, 0, xb, hc);
      Op hb[TR::OPB];
      epilogue_op<TR>(hc, b1 + c * 32, h, true, hb);
      if (W2_OWN_PART) st.next();
      const int base = W2_OWN_PART ? 0 : NSX;
#pragma unroll
      for (int ob = 0; ob < 8; ++ob) KSteps<TR, 0, TR::OPB>::run(st, base + ob * TR::OPB, hb, x[ob]);
    }
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) {
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        x[ob][r] += b2[ob * 32 + crow(r, h)];
        v[r] = x[ob][r];
      }
      TR::to_op(v, &xb[ob * TR::OPB]);
    }
  }

  // ---- output MLP 256 -> 256 -> 128 -> 3
#pragma unroll
  for (int ob = 0; ob < 8; ++ob) acc[ob] = f32x16{};
  st.next();
  dense<TR, 8, 8>(st, xb, acc);
#pragma unroll
  for (int ob = 0; ob < 8; ++ob) epilogue_op<TR>(acc[ob], sb + kOffO0 + ob * 32, h, true, &xb[ob * TR::OPB]);
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) acc[ob] = f32x16{};
  st.next();
  dense<TR, 4, 8>(st, xb, acc);
  Op o2[4 * TR::OPB];
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) epilogue_op<TR>(acc[ob], sb + kOffO2 + ob * 32, h, true, &o2[ob * TR::OPB]);
  acc[0] = f32x16{};
  st.next();
  dense<TR, 1, 4>(st, o2, acc);
  if (valid && h == 0) {
    out[p * 3 + 0] = acc[0][0] + sb[kOffO4 + 0];
    out[p * 3 + 1] = acc[0][1] + sb[kOffO4 + 1];
    out[p * 3 + 2] = acc[0][2] + sb[kOffO4 + 2];
  }
}

// cond[c] = b4 + time_proj(emb(t_c)) + style_proj(style_c)   (diffusion_model.py:15-26, 56-58)
// freqs[64] is the reference's exp table computed on the host with torch's own CPU exp.
__global__ __launch_bounds__(256) void cond_bias_kernel(
    const int64_t* __restrict__ t, const float* __restrict__ style, const float* __restrict__ freqs,
    const float* __restrict__ wt, const float* __restrict__ bt, const float* __restrict__ ws,
    const float* __restrict__ bs, const float* __restrict__ b4, float* __restrict__ cond) {
  const int c = blockIdx.x, o = threadIdx.x;
  __shared__ float emb[128];
  __shared__ float sty[256];
  const float tf = (float)t[c];
  if (o < 64) emb[o] = sinf(tf * freqs[o]);
  else if (o < 128) emb[o] = cosf(tf * freqs[o - 64]);
  sty[o] = style[c * 256 + o];
  __syncthreads();
  // wt / ws are the TRANSPOSED weights ([in][out]): lane o reads consecutive addresses
  float a = bt[o];
  for (int i = 0; i < 128; ++i) a = fmaf(wt[i * 256 + o], emb[i], a);
  float b = bs[o];
  for (int i = 0; i < 256; ++i) b = fmaf(ws[i * 256 + o], sty[i], b);
  cond[c * 256 + o] = (b4[o] + a) + b;
}

template <class TR>
static int launch_noise_mlp(const float* pts, int64_t P, int64_t T, const float* cond,
                            int64_t nclouds, const void* blob, int64_t blob_bytes,
                            const float* bias, float* out, hipStream_t s) {
  constexpr int PTS = TR::THREADS / 64 * 32;
  const int nparts = (int)(blob_bytes / kPart);
  const size_t lds = 2 * kPart + (kBiasFloats + kCondSlots * 256) * sizeof(float);
  hipLaunchKernelGGL(noise_mlp_kernel<TR>, dim3((unsigned)cdiv(P, PTS)), dim3(TR::THREADS), lds, s,
                     pts, P, T, cond, nclouds, (const char*)blob, nparts, bias, out);
  return PCST_OK;
}

}  // namespace pcst

using namespace pcst;

// Bytes of the packed weight blob for a precision: 0 = f32 (parity), 1 = bf16.
extern "C" int64_t pcst_noise_mlp_blob_bytes(int precision) {
  // every layer starts on a fresh 32 KiB part (see packing.py); residual chunks take one part
  // (bf16: W1c | W2c) or two (f32: W1c, W2c)
  const int64_t ks = precision == 1 ? 16 : 2;
  const int64_t fpp = kPart / (precision == 1 ? 1024 : 256);
  auto parts = [&](int64_t nob, int64_t k) { return cdiv(nob * (k / ks), fpp); };
  const int64_t chunk = (256 / ks + 8 * (32 / ks)) > fpp ? 2 : 1;
  const int64_t np = parts(8, 128) + parts(8, 256) + 6 * 16 * chunk + parts(8, 256) +
                     parts(4, 256) + parts(1, 128);
  return np * kPart;
}

extern "C" int pcst_noise_cond(const int64_t* t, const float* style, int64_t nclouds,
                               const float* freqs, const float* wt, const float* bt,
                               const float* ws, const float* bs, const float* b4, float* cond,
                               void* stream) {
  PCST_CHECK_ARG(nclouds >= 0, "noise_cond: bad shape");
  if (nclouds == 0) return PCST_OK;
  hipLaunchKernelGGL(cond_bias_kernel, dim3((unsigned)nclouds), dim3(256), 0, as_stream(stream), t,
                     style, freqs, wt, bt, ws, bs, b4, cond);
  PCST_LAUNCH_CHECK("noise_cond");
  return PCST_OK;
}

extern "C" int pcst_noise_mlp(const float* pts, int64_t P, int64_t points_per_cloud,
                              const float* cond, int64_t nclouds, const void* blob,
                              int64_t blob_bytes, const float* bias, int precision, float* out,
                              void* stream) {
  PCST_CHECK_ARG(P >= 0 && points_per_cloud > 0 && nclouds > 0, "noise_mlp: bad shape");
  PCST_CHECK_ARG(P <= points_per_cloud * nclouds, "noise_mlp: P exceeds clouds*points");
  PCST_CHECK_ARG(precision == 0 || precision == 1, "noise_mlp: precision must be 0 (f32) or 1 (bf16)");
  PCST_CHECK_ARG(blob_bytes == pcst_noise_mlp_blob_bytes(precision), "noise_mlp: blob size %lld != %lld",
                 (long long)blob_bytes, (long long)pcst_noise_mlp_blob_bytes(precision));
  PCST_CHECK_ARG(((uintptr_t)blob & 15) == 0, "noise_mlp: blob must be 16-byte aligned");
  if (P == 0) return PCST_OK;
  hipStream_t s = as_stream(stream);
  if (precision == 1)
    launch_noise_mlp<TrBF16>(pts, P, points_per_cloud, cond, nclouds, blob, blob_bytes, bias, out, s);
  else
    launch_noise_mlp<TrF32>(pts, P, points_per_cloud, cond, nclouds, blob, blob_bytes, bias, out, s);
  PCST_LAUNCH_CHECK("noise_mlp");
  return PCST_OK;
}
