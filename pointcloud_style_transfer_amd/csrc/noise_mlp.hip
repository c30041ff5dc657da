// Fused per-point noise-prediction MLP of NoisePredictor.forward
// (models/diffusion_model.py:38-61) on MFMA, one launch for the whole stack:
//   h1 = relu(W0 p + b0)            3 -> 128       (VALU: K = 3)
//   h2 = relu(W2 h1 + b2)           128 -> 256     (MFMA)
//   x  = W4 h2 + cond[cloud]        256 -> 256     cond = b4 + time_proj(emb(t)) + style_proj(s)
//   6x x += W2_i relu(W1_i x + b1_i) + b2_i        256 -> 512 -> 256 (hidden streamed in chunks)
//   o  = W_o4 relu(W_o2 relu(W_o0 x + b) + b) + b  256 -> 256 -> 128 -> 3
//
// Two kernels, one per precision code of the ABI:
//   0 (f32, parity): noise_mlp_kernel<TrF32>, exact-f32 v_mfma_f32_32x32x2_f32, 4 waves x 32 points,
//     features on MFMA rows and points on lanes, so a layer's accumulator (after bias / ReLU) is
//     the next layer's B operand with no LDS round trip; weights stream through LDS in 32 KiB parts;
//   1 (bf16, the product): solo::noise_mlp_solo_kernel, v_mfma_f32_16x16x32_bf16, 8 waves x 32
//     points, every wave computing all features of its points, the weights in 64 KiB superparts
//     (DESIGN.md section 3).
// The k-order each layout induces is absorbed by the host-side weight packing (packing.py), which
// lays every A fragment out as one contiguous block in streaming order.
#include "common.h"

namespace pcst {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int kPart = 32768;  // bytes per streamed weight part
// bias table offsets (floats) -- must match packing.py
constexpr int kOffW0 = 0, kOffB0 = 384, kOffB2 = 512, kOffB1 = 768, kOffBB2 = 3840,
              kOffO0 = 5376, kOffO2 = 5632, kOffO4 = 5760, kBiasFloats = 5792;
constexpr int kCondSlots = 4;

struct TrF32 {
  static constexpr int KS = 2;
  static constexpr int FRAG = 256;
  static constexpr int OPB = 16;
  static constexpr int THREADS = 256;
  static constexpr int NCB = 1;
  static constexpr int G = 8;
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

// Weight parts stream HBM/L2 -> LDS (global_load_lds, 16 B per lane, no registers) through a
// ring of kSlots 32 KiB slots, one part ahead of use: next() = barrier (part+1 has landed;
// every wave is done with part-1), advance, then DMA part+2 into the slot part-1 held.  Three
// slots let the residual loop read two consecutive parts at once (W2 of chunk c from part-1
// while W1 of chunk c+1 runs on part).
template <class TR>
struct Streamer {
  static constexpr int kSlots = 3;
  static constexpr int kWaves = TR::THREADS / 64;
  static constexpr int kPerWave = kPart / 1024 / kWaves;  // 1 KiB pieces per wave per part
  const char* blob;
  char* lds;   // kSlots x kPart
  int part;    // part being computed
  int nparts;
  int wave;    // wave index, wave-uniform (SGPR)

  __device__ void issue(int q) {
    if (q >= nparts) return;
    const int lane = threadIdx.x & 63;
    // uniform LDS destination (M0) and global base; only lane*16 varies per lane
    char* dst = lds + (q % kSlots) * kPart + wave * kPerWave * 1024;
    const char* src = blob + (int64_t)q * kPart + wave * kPerWave * 1024;
#pragma unroll
    for (int i = 0; i < kPerWave; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src + i * 1024 + lane * 16),
                                       (__attribute__((address_space(3))) void*)(dst + i * 1024),
                                       16, 0, 0);
  }
  __device__ void begin() {  // part 0 resident, part 1 in flight
    issue(0);
    __syncthreads();
    issue(1);
  }
  __device__ void next() {
    __syncthreads();
    ++part;
    issue(part + 1);
  }
  __device__ typename TR::A frag_at(int q, int f) const {
    return *reinterpret_cast<const typename TR::A*>(
        lds + (q % kSlots) * kPart + f * TR::FRAG + (threadIdx.x & 63) * (int)sizeof(typename TR::A));
  }
  __device__ typename TR::A frag(int f) const { return frag_at(part, f); }
};

// one bf16 fragment read at byte offset `off` from `addr` in inline asm (off a compile-time
// constant after unrolling goes into the instruction's offset field); the solo kernel waits for
// it with a counted, tied s_waitcnt (its RULE below)
__device__ __forceinline__ bf16x8 lds_read_one(uint32_t addr, int off) {
  bf16x8 v;
  if (__builtin_constant_p(off) && off >= 0 && off < 65536)
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
  else
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr + off));
  return v;
}

struct NoHook {
  __device__ void operator()(int) const {}
};

template <class TR, int N, int KPER, int ICB, int AST, int ACB, class Hook = NoHook, class ST>
__device__ __forceinline__ void run_seq(const ST& st, int q, int base,
                                        const typename TR::Op* in, f32x16* acc,
                                        const Hook& hook = Hook()) {
  constexpr int G = TR::G;
  static_assert(N % G == 0, "group size must divide the sequence");
  using A = typename TR::A;
  A cur[G];
#pragma unroll
  for (int j = 0; j < G; ++j) cur[j] = st.frag_at(q, base + j);
#pragma unroll
  for (int g = 0; g < N; g += G) {
    A nxt[G];
    if (g + G < N) {
#pragma unroll
      for (int j = 0; j < G; ++j) nxt[j] = st.frag_at(q, base + g + G + j);
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int i = g + j;
#pragma unroll
      for (int cb = 0; cb < TR::NCB; ++cb)
        acc[(i / KPER) * AST + cb * ACB] =
            TR::mfma(cur[j], in[cb * ICB + i % KPER], acc[(i / KPER) * AST + cb * ACB]);
    }
    hook(g / G);
    if (g + G < N) {
#pragma unroll
      for (int j = 0; j < G; ++j) cur[j] = nxt[j];
    }
  }
}

// Dense layer over NOB output blocks with K = KB 32-row input blocks; in[cb*KB*OPB + s],
// acc[cb*8 + ob].  Every layer starts on a fresh part (the packing pads each layer to whole
// parts); inside a layer a part holds OBPP whole output blocks.
template <class TR, int NOB, int KB, int OB0 = 0>
__device__ __forceinline__ void dense(Streamer<TR>& st, const typename TR::Op* in, f32x16* acc) {
  constexpr int NS = KB * TR::OPB;
  constexpr int FPP = kPart / TR::FRAG;
  constexpr int OBPP = FPP / NS;
  static_assert(OBPP >= 1 && FPP % NS == 0, "part must hold whole output blocks");
  constexpr int NOW = (NOB - OB0) < OBPP ? (NOB - OB0) : OBPP;
  run_seq<TR, NOW * NS, NS, NS, 1, 8>(st, st.part, 0, in, acc + OB0);
  if constexpr (OB0 + NOW < NOB) {
    st.next();
    dense<TR, NOB, KB, OB0 + NOW>(st, in, acc);
  }
}

// 16 bias values of a 32-row block in accumulator order (the accumulator's initial value)
__device__ __forceinline__ f32x16 bias_block(const float* b, int h) {
  f32x16 v;
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = b[crow(r, h)];
  return v;
}

template <class TR>
__device__ __forceinline__ void act_op(const f32x16& acc, bool relu, typename TR::Op* out) {
  float v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = relu ? fmaxf(acc[r], 0.0f) : acc[r];
  TR::to_op(v, out);
}

template <class TR>
__global__ __launch_bounds__(TR::THREADS) void noise_mlp_kernel(
    const float* __restrict__ pts, int64_t P, int64_t T, const float* __restrict__ cond,
    int64_t nclouds, const char* __restrict__ blob, int nparts, const float* __restrict__ bias,
    float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sb = reinterpret_cast<float*>(smem + Streamer<TR>::kSlots * kPart);
  float* sc = sb + kBiasFloats;  // kCondSlots x 256
  using Op = typename TR::Op;
  constexpr int NCB = TR::NCB, OPB = TR::OPB;
  constexpr int PTS = TR::THREADS / 64 * 32 * NCB;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5;
  const int64_t p0 = (int64_t)blockIdx.x * PTS;
  const int64_t c0 = p0 / T;
  for (int i = tid; i < kBiasFloats; i += TR::THREADS) sb[i] = bias[i];
  for (int i = tid; i < kCondSlots * 256; i += TR::THREADS) {
    const int64_t c = c0 + i / 256;
    sc[i] = c < nclouds ? cond[c * 256 + (i % 256)] : 0.0f;
  }
  int64_t p[NCB];
  int slot[NCB];
  float px[NCB], py[NCB], pz[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    p[cb] = p0 + (wid * NCB + cb) * 32 + (lane & 31);
    const int64_t pc = p[cb] < P ? p[cb] : (P - 1);
    px[cb] = pts[pc * 3 + 0];
    py[cb] = pts[pc * 3 + 1];
    pz[cb] = pts[pc * 3 + 2];
    slot[cb] = (int)(pc / T - c0);
  }
  __syncthreads();

  Streamer<TR> st{blob, smem, 0, nparts, __builtin_amdgcn_readfirstlane(wid)};
  st.begin();

  // ---- h1 = relu(W0 p + b0), 128 rows, VALU, straight into operand form
  Op h1[NCB * 4 * OPB];
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) {
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = ob * 32 + crow(r, h);
        float x = sb[kOffB0 + row];
        x = fmaf(sb[kOffW0 + row * 3 + 0], px[cb], x);
        x = fmaf(sb[kOffW0 + row * 3 + 1], py[cb], x);
        x = fmaf(sb[kOffW0 + row * 3 + 2], pz[cb], x);
        v[r] = fmaxf(x, 0.0f);
      }
      TR::to_op(v, &h1[cb * 4 * OPB + ob * OPB]);
    }
  }

  f32x16 acc[NCB * 8];
  Op xb[NCB * 8 * OPB];

  // ---- h2 = relu(W2 h1 + b2)
#pragma unroll
  for (int ob = 0; ob < 8; ++ob) {
    const f32x16 b = bias_block(sb + kOffB2 + ob * 32, h);
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) acc[cb * 8 + ob] = b;
  }
  dense<TR, 8, 4>(st, h1, acc);
#pragma unroll
  for (int i = 0; i < NCB * 8; ++i) act_op<TR>(acc[i], true, &xb[i * OPB]);

  // ---- x = W4 h2 + cond[cloud]   (cond already contains b4)
  f32x16 x[NCB * 8];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const bool in_lds = slot[cb] >= 0 && slot[cb] < kCondSlots;
    const float* crow_src = in_lds ? sc + slot[cb] * 256 : cond + (c0 + slot[cb]) * 256;
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) x[cb * 8 + ob] = bias_block(crow_src + ob * 32, h);
  }
  {
    Op h2[NCB * 8 * OPB];
#pragma unroll
    for (int i = 0; i < NCB * 8 * OPB; ++i) h2[i] = xb[i];
    st.next();
    dense<TR, 8, 8>(st, h2, x);
  }
#pragma unroll
  for (int i = 0; i < NCB * 8; ++i) act_op<TR>(x[i], false, &xb[i * OPB]);

  // ---- 6 residual blocks, hidden 512 streamed in 16 chunks of 32 rows.  Per chunk the
  // packing holds W1 rows [32c, 32c+32) (all K) then W2 columns [32c, 32c+32) (all 8 output
  // blocks): one part in bf16, two parts (W1 | W2) in f32.
  constexpr int FPP = kPart / TR::FRAG;
  constexpr int NSX = 8 * OPB;                  // k-steps over x (K = 256)
  constexpr bool W2_OWN_PART = (NSX + 8 * OPB) > FPP;
  for (int layer = 0; layer < 6; ++layer) {
    const float* b1 = sb + kOffB1 + layer * 512;
    const float* b2 = sb + kOffBB2 + layer * 256;
    static_assert(W2_OWN_PART, "f32: the W1 chunk and the W2 chunk each fill a part");
    for (int c = 0; c < 16; ++c) {
      st.next();
      f32x16 hc[NCB];
      const f32x16 bc = bias_block(b1 + c * 32, h);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) hc[cb] = bc;
      run_seq<TR, NSX, NSX, NSX, 1, 1>(st, st.part, 0, xb, hc);
      Op hb[NCB * OPB];
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) act_op<TR>(hc[cb], true, &hb[cb * OPB]);
      st.next();
      run_seq<TR, 8 * OPB, OPB, OPB, 1, 8>(st, st.part, 0, hb, x);
    }
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) {
      const f32x16 b = bias_block(b2 + ob * 32, h);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        x[cb * 8 + ob] += b;
        act_op<TR>(x[cb * 8 + ob], false, &xb[(cb * 8 + ob) * OPB]);
      }
    }
  }

  // ---- output MLP 256 -> 256 -> 128 -> 3
#pragma unroll
  for (int ob = 0; ob < 8; ++ob) {
    const f32x16 b = bias_block(sb + kOffO0 + ob * 32, h);
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) acc[cb * 8 + ob] = b;
  }
  st.next();
  dense<TR, 8, 8>(st, xb, acc);
#pragma unroll
  for (int i = 0; i < NCB * 8; ++i) act_op<TR>(acc[i], true, &xb[i * OPB]);
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) {
    const f32x16 b = bias_block(sb + kOffO2 + ob * 32, h);
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) acc[cb * 8 + ob] = b;
  }
  st.next();
  dense<TR, 4, 8>(st, xb, acc);
  Op o2[NCB * 4 * OPB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) act_op<TR>(acc[cb * 8 + ob], true, &o2[(cb * 4 + ob) * OPB]);
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) acc[cb * 8] = f32x16{};
  st.next();
  dense<TR, 1, 4>(st, o2, acc);
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    if (p[cb] < P && h == 0) {
      out[p[cb] * 3 + 0] = acc[cb * 8][0] + sb[kOffO4 + 0];
      out[p[cb] * 3 + 1] = acc[cb * 8][1] + sb[kOffO4 + 1];
      out[p[cb] * 3 + 2] = acc[cb * 8][2] + sb[kOffO4 + 2];
    }
  }
}

// v_mfma_f32_16x16x32_bf16: lane l holds A[16rb + (l & 15)][k-slot 8(l >> 4) + j]; C/D rows
// 4(l >> 4) + i of column l & 15
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// The MLP's side of a cross-stream wait (pcst_noise_mlp_ex's wait_flag): the last work-group to
// finish waits until `flag` holds `value` (at most max_polls polls; a timeout sets *err), so work
// queued after the MLP also waits for the other stream's producer, with no wait launch of its own.
__device__ __forceinline__ void last_group_wait(const uint32_t* flag, uint32_t value,
                                                uint32_t* counter, int32_t* err, int64_t max_polls,
                                                bool leader) {
  __syncthreads();  // this work-group's rows are written
  if (leader) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t prev = atomicAdd(counter, 1u);
    if (prev == gridDim.x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bool ok = false;
      for (int64_t i = 0; i < max_polls; ++i) {
        if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= value) {
          ok = true;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (!ok && err) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ============================================================================================
// bf16 "solo" kernel on v_mfma_f32_16x16x32_bf16 (precision code 1).  Every wave owns 32 points
// (two 16-point column blocks) and ALL features of every layer, so no wave ever needs another
// wave's activations: there is no partner exchange, and a 1 KiB weight fragment in LDS feeds all
// 8 waves of the work-group (2 MFMAs each) instead of the 4 waves of one role.  256 points per
// work-group, 8 waves = 2 per SIMD.
//
// Weights stream through a 2-slot ring of 64 KiB *superparts* (64 fragments, packing.py SOLO16)
// with ONE barrier per superpart: per barrier each wave runs 128 MFMAs (the pair kernel: 32), and
// each wave DMAs 8 KiB of the next superpart while computing the current one.  Inside a
// superpart the fragment reads run kD ahead of the MFMAs (asm reads, counted lgkmcnt waits), and
// the few other LDS reads (biases) are issued at fixed places in the same count.
//
// Register budget at two waves per SIMD (256): the residual stream x (32 points x 256 features,
// fp32) 128, its bf16 operand xb 64, one hidden chunk (32 rows) hc 16 + its operand hb 8, the
// fragment window 20, biases 8.
//
// Residual layers are software-pipelined by one hidden chunk: part k of a layer = [W1(k) | W2(k-1)]
// and the ReLU/bf16 epilogue of chunk k runs after W2(k-1)'s MFMAs are issued, so it never waits
// for an MFMA result; part 0 = [W2(15) of the previous layer | W1(0)], the layer-end conversion
// x -> xb between them (the stream order of packing.py SOLO16).
namespace solo {

constexpr int NCB = 2;                  // 16-point column blocks per wave
constexpr int NW = 8;                   // waves per work-group (two per SIMD)
constexpr int kThreads = NW * 64;
constexpr int kPts = NW * 16 * NCB;     // 256 points per work-group
constexpr int kSP = 65536;              // superpart bytes
constexpr int kNF = kSP / 1024;         // fragments per superpart
constexpr int kD = 2;                   // fragment reads in flight ahead of their MFMAs
constexpr int kBiasLds = 2 * kSP;       // LDS byte offset of the bias table
constexpr int kLds = kBiasLds + kBiasFloats * 4;
constexpr int kTailSP = 3 + 6 * 8;      // first superpart of the output MLP (after h2, x, 6 layers)
constexpr int kNSP = kTailSP + 4;       // 55

template <int I, int N, class F>
__device__ __forceinline__ void sfor(F& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

// LDS operations issued after the read of fragment f, at its wait in iteration f.  Iteration j
// issues S::nx(j) extra reads, then the read of fragment j + kD; fragments 0..kD-1 are read
// before iteration 0.
template <class S>
constexpr int frag_after(int f) {
  int n = (S::NF - 1 - f) < kD ? (S::NF - 1 - f) : kD;
  for (int j = (f - kD + 1 > 0 ? f - kD + 1 : 0); j <= f; ++j) n += S::nx(j);
  return n;
}
// LDS operations issued after the extra reads of iteration J, at a wait in iteration f >= J
template <class S>
constexpr int extra_after(int J, int f) {
  int n = 0;
  for (int j = J; j <= f; ++j) n += (j + kD < S::NF) ? 1 : 0;
  for (int j = J + 1; j <= f; ++j) n += S::nx(j);
  return n;
}

template <int N>
__device__ __forceinline__ void wait_frag(bf16x8& a) {
  static_assert(N >= 0 && N <= 15, "lgkmcnt range");
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "n"(N));
}
template <int N>
__device__ __forceinline__ void wait_f4(f32x4& a) {
  static_assert(N >= 0 && N <= 15, "lgkmcnt range");
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "n"(N));
}
template <int N>
__device__ __forceinline__ void wait_f4x2(f32x4& a, f32x4& b) {
  static_assert(N >= 0 && N <= 15, "lgkmcnt range");
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
}
// a uniform value re-materialised here (empty asm): address arithmetic that uses it cannot be
// hoisted out of its loop and kept live (at 256 VGPRs such a hoisted value spills)
__device__ __forceinline__ uint32_t here(uint32_t v) {
  v = __builtin_amdgcn_readfirstlane(v);
  asm volatile("" : "+s"(v));
  return v;
}
// this lane's index without keeping threadIdx.x live (v_mbcnt)
__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// one bias row (f32x4) from the LDS table; `off` is a compile-time byte offset.
// RULE for every asm LDS read here: its result must reach a tied wait (wait_frag / wait_f4) before
// anything else.  The compiler sees the read's output as written at the asm statement, so an
// unused result frees its registers at once -- and the data that lands later overwrites whatever
// the compiler put there (an unused bias read once clobbered a 64-bit address: a memory fault).
// tools/asm_hazard.py checks the built kernel for reads whose registers are touched before their
// wait.
__device__ __forceinline__ f32x4 lds_f4(uint32_t addr, int off) {
  f32x4 v;
  if (__builtin_constant_p(off) && off >= 0 && off < 65536)
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
  else
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr + off));
  return v;
}

// One superpart: S::NF fragments at lane address `a` (fragment f at a + 1024 f).  Iteration f:
// xr(f) (extra reads), the read of fragment f + kD, the counted wait for fragment f, mf(f, frag),
// dm(f) (DMA of the next superpart), po(f) (epilogues; a wait for extras uses extra_after).
template <class S, class XR, class MF, class DM, class PO>
__device__ __forceinline__ void run_sp(uint32_t a, XR& xr, MF& mf, DM& dm, PO& po) {
  constexpr int NPRO = kD < S::NF ? kD : S::NF;
  bf16x8 w[kD + 1];
  auto pro = [&](auto fc) {
    constexpr int f = decltype(fc)::value;
    w[f] = lds_read_one(a, f * 1024);
  };
  sfor<0, NPRO>(pro);
  auto it = [&](auto fc) {
    constexpr int f = decltype(fc)::value;
    xr(fc);
    if constexpr (f + kD < S::NF) w[(f + kD) % (kD + 1)] = lds_read_one(a, (f + kD) * 1024);
    wait_frag<frag_after<S>(f)>(w[f % (kD + 1)]);
    mf(fc, w[f % (kD + 1)]);
    dm(fc);
    po(fc);
  };
  sfor<0, S::NF>(it);
}

// every wave: its own DMAs have landed and it is done with the current slot; then the barrier
__device__ __forceinline__ void sp_barrier() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

__device__ __forceinline__ f32x4 relu4(f32x4 v) {
  f32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = fmaxf(v[i], 0.0f);
  return r;
}

// relu(bf16(v)) on packed bf16 pairs: a bf16 with its sign set is a negative int16, so a signed
// 16-bit max with 0 is the ReLU (-0 included) -- one v_pk_max_i16 per two values, after the
// conversion (relu then round == round then relu)
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
// accumulators of row blocks 2s, 2s+1 -> operand of k-step s, one v_cvt_pk_bf16_f32 per pair
// (pcst::op16 converts element by element: a convert-with-zero plus a v_perm per pair)
__device__ __forceinline__ bf16x8 opk(const f32x4& lo, const f32x4& hi) {
  const bf16x2 p0 = __builtin_convertvector((f32x2){lo[0], lo[1]}, bf16x2);
  const bf16x2 p1 = __builtin_convertvector((f32x2){lo[2], lo[3]}, bf16x2);
  const bf16x2 p2 = __builtin_convertvector((f32x2){hi[0], hi[1]}, bf16x2);
  const bf16x2 p3 = __builtin_convertvector((f32x2){hi[2], hi[3]}, bf16x2);
  return __builtin_shufflevector(__builtin_shufflevector(p0, p1, 0, 1, 2, 3),
                                 __builtin_shufflevector(p2, p3, 0, 1, 2, 3), 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8 relu_bf16(bf16x8 v) {
  // (a per-dword form through u32x4 element bit_casts miscompiled to a splat of dword 0 with this
  // clang, host builds included -- keep the whole-vector form)
  const s16x8 h = __builtin_elementwise_max(__builtin_bit_cast(s16x8, v), s16x8{0, 0, 0, 0, 0, 0, 0, 0});
  return __builtin_bit_cast(bf16x8, h);
}

// schedules: S::nx(j) = extra LDS reads (biases) issued in iteration j
struct SchH2 {  // h2: fragment f = (row block f/4, k-step f%4); bias of row block rb >= 1 at 4rb-3
  static constexpr int NF = kNF;
  static constexpr int nx(int j) { return j % 4 == 1 && j < 60 ? 1 : 0; }
};
struct SchX {  // x = W4 h2 (+ cond, loaded before): no extras
  static constexpr int NF = kNF;
  static constexpr int nx(int) { return 0; }
};
// A W1 chunk's first fragment of row half r (k-step 0) takes its bias b1 as the MFMA's C operand,
// read two iterations ahead (at iteration 0 for a fragment 0: the read then has the latency of
// the superpart's first fragment reads).
struct SchL0 {  // parts 0, 1 of a layer: W2(15)' 0-15, W1(0) 16-31, W1(1) 32-47, W2(0) 48-63;
                // b2 of row block rb at 15 + rb, b1 at 14, 22 (chunk 0) and 30, 38 (chunk 1)
  static constexpr int NF = kNF;
  static constexpr int nx(int j) {
    return (j >= 15 && j < 31 ? 1 : 0) + (j == 14 || j == 22 || j == 30 || j == 38 ? 1 : 0);
  }
};
struct SchR {  // parts 2m, 2m+1: W1(2m) 0-15, W2(2m-1) 16-31, W1(2m+1) 32-47, W2(2m) 48-63;
               // b1 at 0, 6 (chunk 2m) and 30, 38 (chunk 2m+1)
  static constexpr int NF = kNF;
  static constexpr int nx(int j) { return j == 0 || j == 6 || j == 30 || j == 38 ? 1 : 0; }
};
// output MLP: tail fragment t = 64 K + f: W2(15) of layer 5 [0, 16), out0 [16, 144) (bias of row
// block rb read at t = 21 + 8rb), out1 [144, 208) (bias at t = 149 + 8rb), out2 [208, 212)
template <int K>
struct SchT {
  static constexpr int NF = K < 3 ? kNF : 212 - 64 * 3;
  static constexpr int nx(int j) {
    const int t = 64 * K + j;
    return ((t >= 16 && t < 144 && (t - 16) % 8 == 5) || (t >= 144 && t < 208 && (t - 144) % 8 == 5)) ? 1 : 0;
  }
};

__global__ __launch_bounds__(kThreads) void noise_mlp_solo_kernel(
    const float* __restrict__ pts, int64_t P, int64_t T, const float* __restrict__ cond,
    int64_t nclouds, const char* __restrict__ blob, int nsp, const float* __restrict__ bias,
    float* __restrict__ out, const uint32_t* __restrict__ wflag, uint32_t wvalue,
    uint32_t* __restrict__ wcount, int32_t* __restrict__ werr, int64_t wpolls,
    uint32_t* __restrict__ sflag, uint32_t svalue, uint32_t* __restrict__ scount) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // the start signal: every launch ahead of this one on its stream has completed (its inputs are
  // final), published for another stream (pcst_noise_mlp_ex's start_flag) by the first
  // work-group; with scount, by the last work-group to begin (counted out on *scount, which is
  // zero again after it): every work-group of the launch then holds its CU, so work another
  // stream starts behind the flag only finds the CUs the launch leaves idle
  if (sflag && threadIdx.x == 0) {
    if (!scount) {
      if (blockIdx.x == 0) __hip_atomic_store(sflag, svalue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (__hip_atomic_fetch_add(scount, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               gridDim.x - 1) {
      __hip_atomic_store(scount, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sflag, svalue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const uint32_t ba = lds0 + kBiasLds + 16 * g;  // bias rows 4g..4g+3 of a 16-row block
  auto bar = [&]() { sp_barrier(); };
  const f32x4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
  int sp = 0;
  // piece i (1 KiB) of superpart s for this wave
  // (past the last superpart it re-reads the last one into the free slot: no branch in the stream)
  auto piece = [&](int s, int i) {
    const int off = wid * (kSP / NW) + i * 1024;
    const int src = s < nsp ? s : nsp - 1;
    __builtin_amdgcn_global_load_lds((const void*)(blob + (int64_t)src * kSP + off + lane * 16),
                                     (__attribute__((address_space(3))) void*)(smem + (s & 1) * kSP + off),
                                     16, 0, 0);
  };
  // the next superpart's 8 pieces of this wave, at fragments 1, 5, .., 29
  auto dm = [&](auto fc) {
    constexpr int f = decltype(fc)::value;
    if constexpr (f % 4 == 1 && f < 32) piece(sp + 1, f / 4);
  };
  auto none = [](auto) {};
  auto slot = [&]() { return lds0 + (uint32_t)((sp & 1) * kSP) + lane * 16; };

#pragma unroll
  for (int i = 0; i < 8; ++i) piece(0, i);
  float* sb = reinterpret_cast<float*>(smem + kBiasLds);
  for (int i = tid; i < kBiasFloats; i += NW * 64) sb[i] = bias[i];
  const int64_t p0 = (int64_t)blockIdx.x * kPts + wid * 16 * NCB;
  int64_t cl[NCB];
  float px[NCB], py[NCB], pz[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const int64_t pq = p0 + cb * 16 + (lane & 15);
    const int64_t pc = pq < P ? pq : (P - 1);
    px[cb] = pts[pc * 3 + 0];
    py[cb] = pts[pc * 3 + 1];
    pz[cb] = pts[pc * 3 + 2];
    cl[cb] = pc / T;
  }
  bar();  // superpart 0 and the bias table are in LDS

  // ---- h1 = relu(W0 p + b0): 128 features = 4 k-steps, both column blocks (VALU)
  bf16x8 h1[4 * NCB];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = 32 * s + 16 * (j >> 2) + 4 * g + (j & 3);
        float v = sb[kOffB0 + f];
        v = fmaf(sb[kOffW0 + f * 3 + 0], px[cb], v);
        v = fmaf(sb[kOffW0 + f * 3 + 1], py[cb], v);
        v = fmaf(sb[kOffW0 + f * 3 + 2], pz[cb], v);
        o[j] = (__bf16)fmaxf(v, 0.0f);
      }
      h1[s * NCB + cb] = o;
    }

  // ---- h2 = relu(W2 h1 + b2) (superpart 0): row block rb's bias is its accumulator's start
  bf16x8 xb[8 * NCB];  // a K = 256 operand [ks*2 + cb]: here h2, later bf16(x)
  {
    f32x4 acc[16 * NCB];
    f32x4 bq;
    auto xr = [&](auto fc) {
      constexpr int f = decltype(fc)::value;
      if constexpr (f % 4 == 1 && f < 60) bq = lds_f4(ba, (kOffB2 + ((f + 3) / 4) * 16) * 4);
    };
    auto mf = [&](auto fc, const bf16x8& a) {
      constexpr int f = decltype(fc)::value, rb = f / 4, ks = f % 4;
      if constexpr (ks == 0) {
        if constexpr (f == 0) {
          bq = lds_f4(ba, kOffB2 * 4);
          wait_f4<0>(bq);
        } else {
          wait_f4<extra_after<SchH2>(f - 3, f)>(bq);
        }
      }
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
        acc[rb * NCB + cb] = mfma16(a, h1[ks * NCB + cb], ks == 0 ? bq : acc[rb * NCB + cb]);
    };
    auto po = [&](auto fc) {
      constexpr int f = decltype(fc)::value, rb = f / 4;
      // operand k-step s from row blocks 2s, 2s+1, two fragments after the last one's MFMAs
      if constexpr (f % 4 == 1 && rb >= 1 && rb % 2 == 0) {
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          xb[(rb / 2 - 1) * NCB + cb] = relu_bf16(opk(acc[(rb - 2) * NCB + cb], acc[(rb - 1) * NCB + cb]));
      }
      if constexpr (f == 63) {
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) xb[7 * NCB + cb] = relu_bf16(opk(acc[14 * NCB + cb], acc[15 * NCB + cb]));
      }
    };
    run_sp<SchH2>(slot(), xr, mf, dm, po);
  }

  // ---- x = W4 h2 + cond[cloud] (superparts 1, 2); cond enters as the accumulator's start.  The
  // row addresses pass through an empty asm so the loads stay here, after superpart 0 (hoisted
  // into it they would overlap its accumulators and spill); the barrier's wait covers them.
  f32x4 x[16 * NCB];
  {
    const float* crow[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      crow[cb] = cond + cl[cb] * 256 + 4 * g;
      asm volatile("" : "+v"(crow[cb]));
    }
#pragma unroll
    for (int rb = 0; rb < 16; ++rb)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) x[rb * NCB + cb] = *reinterpret_cast<const f32x4*>(crow[cb] + rb * 16);
  }
  auto xhalf = [&](auto hc_) {
    constexpr int h = decltype(hc_)::value;
    bar();
    ++sp;
    auto mf = [&](auto fc, const bf16x8& a) {
      constexpr int f = decltype(fc)::value, rb = h * 8 + f / 8, ks = f % 8;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) x[rb * NCB + cb] = mfma16(a, xb[ks * NCB + cb], x[rb * NCB + cb]);
    };
    run_sp<SchX>(slot(), none, mf, dm, none);
  };
  sfor<0, 2>(xhalf);

  // ---- 6 residual blocks x += W2 relu(W1 x + b1) + b2, 8 superparts each.  The epilogue of hidden
  // chunk c (hb = relu(bf16(hc))) runs after W2(c-1)'s MFMAs are issued: it never waits for an MFMA,
  // and W1(c+1) (independent of hb) follows it.
  bf16x8 hb[NCB] = {};  // zero: layer 0's part 0 has no W2(15) (zero fragments)
  f32x4 hc[2 * NCB];
  f32x4 b1r;  // the bias of the W1 row half whose first fragment comes next
  auto w1 = [&](auto ic, const bf16x8& a) {  // fragment (r, ks) of a W1 chunk, ic = 8r + ks
    constexpr int i = decltype(ic)::value, r = i / 8, ks = i % 8;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) hc[r * NCB + cb] = mfma16(a, xb[ks * NCB + cb], ks == 0 ? b1r : hc[r * NCB + cb]);
  };
  auto w2 = [&](auto rc, const bf16x8& a) {  // row block rc of a W2 chunk column
    constexpr int rb = decltype(rc)::value;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) x[rb * NCB + cb] = mfma16(a, hb[cb], x[rb * NCB + cb]);
  };
  auto epi = [&]() {
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) hb[cb] = relu_bf16(opk(hc[cb], hc[NCB + cb]));
  };
  for (int layer = 0; layer < 6; ++layer) {
    // bias byte offsets of this layer (uniform); each read adds its own to ba, so no per-layer
    // lane address stays live across the layer (it would spill)
    const uint32_t b1o = (kOffB1 + layer * 512) * 4;   // chunk c, row half r: + (32c + 16r)*4
    const uint32_t b2o = (kOffBB2 + layer * 256) * 4;
    bar();
    ++sp;
    {  // parts 0, 1: W2(15) of the previous layer | xb = bf16(x), x += b2 | W1(0) || W1(1) | W2(0)
      f32x4 bq[2];
      auto xr = [&](auto fc) {
        constexpr int f = decltype(fc)::value;
        if constexpr (f == 14 || f == 22 || f == 30 || f == 38) b1r = lds_f4(ba + here(b1o), (f - 14) / 8 * 64);
        if constexpr (f >= 15 && f < 31) bq[(f - 15) % 2] = lds_f4(ba + here(b2o), (f - 15) * 64);
      };
      auto mf = [&](auto fc, const bf16x8& a) {
        constexpr int f = decltype(fc)::value;
        if constexpr (f < 16) {
          w2(std::integral_constant<int, f>{}, a);
        } else if constexpr (f < 48) {
          if constexpr (f % 8 == 0) wait_f4<extra_after<SchL0>(f - 2, f)>(b1r);
          w1(std::integral_constant<int, (f - 16) % 16>{}, a);
        } else {
          w2(std::integral_constant<int, f - 48>{}, a);
        }
      };
      auto po = [&](auto fc) {
        constexpr int f = decltype(fc)::value;
        // xb k-step s from x row blocks 2s, 2s+1 (final after W2(15) fragment 2s+1), two
        // fragments later; W1(0) reads k-step s at fragment 16 + s
        if constexpr (f >= 3 && f <= 17 && f % 2 == 1) {
          constexpr int s = (f - 3) / 2;
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb) xb[s * NCB + cb] = opk(x[(2 * s) * NCB + cb], x[(2 * s + 1) * NCB + cb]);
        }
        if constexpr (f >= 16 && f < 32) {  // x += b2 (x's W2 products of this layer come later)
          constexpr int rb = f - 16;
          wait_f4<extra_after<SchL0>(f - 1, f)>(bq[rb % 2]);
          for (int cb = 0; cb < NCB; ++cb) x[rb * NCB + cb] += bq[rb % 2];
        }
        if constexpr (f == 31 || f == 63) epi();  // chunk 0 / chunk 1
      };
      run_sp<SchL0>(slot(), xr, mf, dm, po);
    }
    for (int m = 1; m < 8; ++m) {  // parts 2m, 2m + 1: W1(2m) | W2(2m-1) || W1(2m+1) | W2(2m)
      bar();
      ++sp;
      const uint32_t bmo = b1o + m * 256;
      auto xr = [&](auto fc) {
        constexpr int f = decltype(fc)::value;
        if constexpr (f == 0 || f == 6) b1r = lds_f4(ba + here(bmo), (f / 6) * 64);
        if constexpr (f == 30 || f == 38) b1r = lds_f4(ba + here(bmo), 128 + (f - 30) / 8 * 64);
      };
      auto mf = [&](auto fc, const bf16x8& a) {
        constexpr int f = decltype(fc)::value;
        if constexpr (f % 32 < 16) {
          if constexpr (f == 0) wait_f4<extra_after<SchR>(0, 0)>(b1r);
          if constexpr (f == 8 || f == 32 || f == 40) wait_f4<extra_after<SchR>(f - 2, f)>(b1r);
          w1(std::integral_constant<int, f % 16>{}, a);
        } else {
          w2(std::integral_constant<int, f % 16>{}, a);
        }
      };
      auto po = [&](auto fc) {
        constexpr int f = decltype(fc)::value;
        if constexpr (f == 31 || f == 63) epi();  // chunk 2m / 2m + 1
      };
      run_sp<SchR>(slot(), xr, mf, dm, po);
    }
  }

  // ---- tail: W2(15) of layer 5, then the output MLP 256 -> 256 -> 128 -> 3
  f32x4 acc[16 * NCB];   // out0 (16 row blocks), then out1 (8)
  bf16x8 o1[8 * NCB];   // out0's output: out1's K = 256 operand
  bf16x8 o2[4 * NCB];    // out1's output: out2's K = 128 operand
  f32x4 acc2[NCB];
  f32x4 bq[2];
  auto tail = [&](auto kc) {
    constexpr int K = decltype(kc)::value;
    using S = SchT<K>;
    bar();
    ++sp;
    auto xr = [&](auto fc) {
      constexpr int t = 64 * K + decltype(fc)::value;
      if constexpr (t >= 16 && t < 144 && (t - 16) % 8 == 5)
        bq[((t - 16) / 8) % 2] = lds_f4(ba, (kOffO0 + ((t - 16) / 8) * 16) * 4);
      if constexpr (t >= 144 && t < 208 && (t - 144) % 8 == 5)
        bq[((t - 144) / 8) % 2] = lds_f4(ba, (kOffO2 + ((t - 144) / 8) * 16) * 4);
    };
    auto mf = [&](auto fc, const bf16x8& a) {
      constexpr int t = 64 * K + decltype(fc)::value;
      if constexpr (t < 16) {
        w2(std::integral_constant<int, t>{}, a);
      } else if constexpr (t < 144) {
        constexpr int rb = (t - 16) / 8, ks = (t - 16) % 8;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          acc[rb * NCB + cb] = mfma16(a, xb[ks * NCB + cb], ks == 0 ? zero : acc[rb * NCB + cb]);
      } else if constexpr (t < 208) {
        constexpr int rb = (t - 144) / 8, ks = (t - 144) % 8;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          acc[rb * NCB + cb] = mfma16(a, o1[ks * NCB + cb], ks == 0 ? zero : acc[rb * NCB + cb]);
      } else {
        constexpr int ks = t - 208;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) acc2[cb] = mfma16(a, o2[ks * NCB + cb], ks == 0 ? zero : acc2[cb]);
      }
    };
    auto po = [&](auto fc) {
      constexpr int f = decltype(fc)::value, t = 64 * K + f;
      if constexpr (t >= 3 && t <= 17 && t % 2 == 1) {  // xb = bf16(x), as in a layer's part 0
        constexpr int s = (t - 3) / 2;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) xb[s * NCB + cb] = opk(x[(2 * s) * NCB + cb], x[(2 * s + 1) * NCB + cb]);
      }
      if constexpr (t >= 16 && t < 144 && (t - 16) % 8 == 7) {  // out0 row block rb done
        constexpr int rb = (t - 16) / 8;
        wait_f4<extra_after<S>(f - 2, f)>(bq[rb % 2]);
        for (int cb = 0; cb < NCB; ++cb) acc[rb * NCB + cb] += bq[rb % 2];
        if constexpr (rb % 2 == 1) {
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb)
            o1[(rb / 2) * NCB + cb] = relu_bf16(opk(acc[(rb - 1) * NCB + cb], acc[rb * NCB + cb]));
        }
      }
      if constexpr (t >= 144 && t < 208 && (t - 144) % 8 == 7) {  // out1 row block rb done
        constexpr int rb = (t - 144) / 8;
        wait_f4<extra_after<S>(f - 2, f)>(bq[rb % 2]);
        for (int cb = 0; cb < NCB; ++cb) acc[rb * NCB + cb] += bq[rb % 2];
        if constexpr (rb % 2 == 1) {
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb)
            o2[(rb / 2) * NCB + cb] = relu_bf16(opk(acc[(rb - 1) * NCB + cb], acc[rb * NCB + cb]));
        }
      }
    };
    run_sp<S>(slot(), xr, mf, dm, po);
  };
  sfor<0, 4>(tail);
  const uint32_t ln = lane_id();  // (recomputed: not kept live through the kernel)
  if (ln < 16) {                   // lane group 0 holds rows 0..3
    const float o0 = sb[kOffO4 + 0], o1v = sb[kOffO4 + 1], o2v = sb[kOffO4 + 2];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      const int64_t q = (int64_t)here(blockIdx.x * kPts + wid * 16 * NCB + cb * 16) + ln;
      if (q < P) {
        out[q * 3 + 0] = acc2[cb][0] + o0;
        out[q * 3 + 1] = acc2[cb][1] + o1v;
        out[q * 3 + 2] = acc2[cb][2] + o2v;
      }
    }
  }
  if (wflag) last_group_wait(wflag, wvalue, wcount, werr, wpolls, wid == 0 && lane_id() == 0);
}

}  // namespace solo

// cond[c] = b4 + time_proj(emb(t_c)) + style_proj(style_c)   (diffusion_model.py:15-26, 56-58)
// freqs[64] is the reference's exp table computed on the host with torch's own CPU exp.
// Grid (clouds, 8): workgroup y computes outputs [32y, 32y + 32); its 8 row groups split the
// K ranges (16 of the 128 time features, 32 of the 256 style features each) and the partial
// sums meet in LDS.
constexpr int kCondSplit = 8;
__global__ __launch_bounds__(256) void cond_bias_kernel(
    const int64_t* __restrict__ t, const float* __restrict__ style, const float* __restrict__ freqs,
    const float* __restrict__ wt, const float* __restrict__ bt, const float* __restrict__ ws,
    const float* __restrict__ bs, const float* __restrict__ b4, float* __restrict__ cond) {
  const int c = blockIdx.x, i = threadIdx.x;
  const int o = blockIdx.y * 32 + (i & 31), g = i >> 5;
  __shared__ float emb[128];
  __shared__ float sty[256];
  __shared__ float pa[kCondSplit][32], pb[kCondSplit][32];
  const float tf = (float)t[c];
  if (i < 64) emb[i] = sinf(tf * freqs[i]);
  else if (i < 128) emb[i] = cosf(tf * freqs[i - 64]);
  sty[i] = style[c * 256 + i];
  __syncthreads();
  // wt / ws are the TRANSPOSED weights ([in][out]): 32 lanes read 128 contiguous bytes
  float a = 0.0f;
#pragma unroll
  for (int k = g * 16; k < g * 16 + 16; ++k) a = fmaf(wt[k * 256 + o], emb[k], a);
  float b = 0.0f;
#pragma unroll
  for (int k = g * 32; k < g * 32 + 32; ++k) b = fmaf(ws[k * 256 + o], sty[k], b);
  pa[g][i & 31] = a;
  pb[g][i & 31] = b;
  __syncthreads();
  if (i < 32) {
    float sa = bt[o], sb = bs[o];
#pragma unroll
    for (int q = 0; q < kCondSplit; ++q) {
      sa += pa[q][i];
      sb += pb[q][i];
    }
    cond[c * 256 + o] = (b4[o] + sa) + sb;
  }
}

template <class TR>
static int launch_noise_mlp(const float* pts, int64_t P, int64_t T, const float* cond,
                            int64_t nclouds, const void* blob, int64_t blob_bytes,
                            const float* bias, float* out, hipStream_t s) {
  constexpr int PTS = TR::THREADS / 64 * 32 * TR::NCB;
  const int nparts = (int)(blob_bytes / kPart);
  const size_t lds = Streamer<TR>::kSlots * kPart + (kBiasFloats + kCondSlots * 256) * sizeof(float);
  hipLaunchKernelGGL(noise_mlp_kernel<TR>, dim3((unsigned)cdiv(P, PTS)), dim3(TR::THREADS), lds, s,
                     pts, P, T, cond, nclouds, (const char*)blob, nparts, bias, out);
  return PCST_OK;
}

}  // namespace pcst

using namespace pcst;

// Bytes of the packed weight blob for a precision: 0 = f32 (parity), 1 = bf16 (solo superparts).
extern "C" int64_t pcst_noise_mlp_blob_bytes(int precision) {
  if (precision == 1) return (int64_t)solo::kNSP * solo::kSP;  // 55 superparts (packing.py BF16)
  if (precision != 0) return -1;
  // f32: every layer starts on a fresh 32 KiB part (see packing.py); a residual chunk takes two
  // parts (W1c, W2c)
  constexpr int64_t ks = 2, fpp = kPart / 256;
  auto parts = [&](int64_t nob, int64_t k) { return cdiv(nob * (k / ks), fpp); };
  const int64_t np = parts(8, 128) + parts(8, 256) + 6 * 16 * 2 + parts(8, 256) + parts(4, 256) +
                     parts(1, 128);
  return np * kPart;
}

extern "C" int pcst_noise_cond(const int64_t* t, const float* style, int64_t nclouds,
                               const float* freqs, const float* wt, const float* bt,
                               const float* ws, const float* bs, const float* b4, float* cond,
                               void* stream) {
  PCST_CHECK_ARG(nclouds >= 0, "noise_cond: bad shape");
  if (nclouds == 0) return PCST_OK;
  hipLaunchKernelGGL(cond_bias_kernel, dim3((unsigned)nclouds, 256 / 32), dim3(256), 0,
                     as_stream(stream), t,
                     style, freqs, wt, bt, ws, bs, b4, cond);
  PCST_LAUNCH_CHECK("noise_cond");
  return PCST_OK;
}

namespace {
int check_mlp_args(const char* name, int64_t P, int64_t points_per_cloud, int64_t nclouds,
                   const void* blob, int64_t blob_bytes, int precision) {
  PCST_CHECK_ARG(P >= 0 && points_per_cloud > 0 && nclouds > 0, "%s: bad shape", name);
  PCST_CHECK_ARG(P <= points_per_cloud * nclouds, "%s: P exceeds clouds*points", name);
  PCST_CHECK_ARG(precision == 0 || precision == 1, "%s: precision must be 0 (f32) or 1 (bf16)", name);
  PCST_CHECK_ARG(blob_bytes == pcst_noise_mlp_blob_bytes(precision), "%s: blob size %lld != %lld", name,
                 (long long)blob_bytes, (long long)pcst_noise_mlp_blob_bytes(precision));
  PCST_CHECK_ARG(((uintptr_t)blob & 15) == 0, "%s: blob must be 16-byte aligned", name);
  return PCST_OK;
}

void launch_solo(const float* pts, int64_t P, int64_t T, const float* cond, int64_t nclouds,
                 const void* blob, const float* bias, float* out, const uint32_t* wflag,
                 uint32_t wvalue, uint32_t* wcount, int32_t* werr, int64_t wpolls, uint32_t* sflag,
                 uint32_t svalue, uint32_t* scount, hipStream_t s) {
  hipLaunchKernelGGL(solo::noise_mlp_solo_kernel, dim3((unsigned)cdiv(P, solo::kPts)), dim3(solo::kThreads),
                     solo::kLds, s, pts, P, T, cond, nclouds, (const char*)blob, solo::kNSP, bias, out,
                     wflag, wvalue, wcount, werr, wpolls, sflag, svalue, scount);
}
}  // namespace

extern "C" int pcst_noise_mlp(const float* pts, int64_t P, int64_t points_per_cloud,
                              const float* cond, int64_t nclouds, const void* blob,
                              int64_t blob_bytes, const float* bias, int precision, float* out,
                              void* stream) {
  if (int rc = check_mlp_args("noise_mlp", P, points_per_cloud, nclouds, blob, blob_bytes, precision)) return rc;
  if (P == 0) return PCST_OK;
  hipStream_t s = as_stream(stream);
  if (precision == 1)
    launch_solo(pts, P, points_per_cloud, cond, nclouds, blob, bias, out, nullptr, 0u, nullptr,
                nullptr, 0, nullptr, 0u, nullptr, s);
  else
    launch_noise_mlp<TrF32>(pts, P, points_per_cloud, cond, nclouds, blob, blob_bytes, bias, out, s);
  PCST_LAUNCH_CHECK("noise_mlp");
  return PCST_OK;
}

namespace pcst {
__global__ void mlp_start_signal_kernel(uint32_t* flag, uint32_t value) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace pcst

extern "C" int pcst_noise_mlp_ex(const float* pts, int64_t P, int64_t points_per_cloud,
                                 const float* cond, int64_t nclouds, const void* blob,
                                 int64_t blob_bytes, const float* bias, int precision, float* out,
                                 uint32_t* start_flag, uint32_t start_value,
                                 uint32_t* start_counter, const uint32_t* wait_flag,
                                 uint32_t wait_value, uint32_t* wait_counter, int32_t* wait_err,
                                 int64_t max_polls, void* stream) {
  // every argument is checked before anything is launched: a start signal published for an
  // invalid call would release a side stream although no MLP ran
  if (int rc = check_mlp_args("noise_mlp_ex", P, points_per_cloud, nclouds, blob, blob_bytes, precision)) return rc;
  PCST_CHECK_ARG(!wait_flag || precision != 1 || P == 0 || wait_counter,
                 "noise_mlp_ex: a wait needs its counter");
  if (precision != 1 || P == 0) {  // the f32 kernel has no fused form: separate launches
    if (start_flag && !start_counter) {
      hipLaunchKernelGGL(mlp_start_signal_kernel, dim3(1), dim3(64), 0, as_stream(stream), start_flag,
                         start_value);
      PCST_LAUNCH_CHECK("noise_mlp_ex: start signal");
    }
    const int rc = pcst_noise_mlp(pts, P, points_per_cloud, cond, nclouds, blob, blob_bytes, bias,
                                  precision, out, stream);
    if (rc != PCST_OK) return rc;
    if (start_flag && start_counter) {  // every work-group has begun: published once it completed
      hipLaunchKernelGGL(mlp_start_signal_kernel, dim3(1), dim3(64), 0, as_stream(stream), start_flag,
                         start_value);
      PCST_LAUNCH_CHECK("noise_mlp_ex: start signal");
    }
    if (!wait_flag) return rc;
    return pcst_signal_wait(wait_flag, wait_value, wait_err, max_polls, stream);
  }
  launch_solo(pts, P, points_per_cloud, cond, nclouds, blob, bias, out, wait_flag, wait_value,
              wait_counter, wait_err, max_polls > 0 ? max_polls : (int64_t)kSignalPolls, start_flag,
              start_value, start_counter, as_stream(stream));
  PCST_LAUNCH_CHECK("noise_mlp_ex");
  return PCST_OK;
}
