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
// bf16 mode: 4 waves x 32 points per workgroup (1 wave/SIMD: 420 VGPR+AGPR per lane; a
// 512-thread variant would have 256 and spills), fp32 accumulate, fp32 residual.
// f32 mode (parity): exact-f32 MFMA, 4 waves x 32 points (1 wave/SIMD).
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

// Perf-experiment knobs, compiled only by tools/nm_variants.sh; the product build uses the
// defaults.  PCST_NM_EXPERIMENT bits: 1 = no weight DMA after the first two parts,
// 2 = no barrier between parts (both give wrong results; they time the overheads;
// tools/nm_quad.hip defines more for its experiment kernel),
// 4 = no LDS fragment reads in the pair16 kernel (A operands from registers), 16 = the same for
// the first group of 4 fragments of every run16 call only, 32 = no residual chunk hand-off,
// 8 = compiler-scheduled LDS fragment reads instead of the asm reads.
#ifndef PCST_NM_EXPERIMENT
#define PCST_NM_EXPERIMENT 0
#endif
#ifndef PCST_NM_NCB
#define PCST_NM_NCB 1
#endif
#ifndef PCST_NM_EPI_GROUP  // pair16 residual loop: the W2 fragment group after which the next
#define PCST_NM_EPI_GROUP 3    // hidden chunk's epilogue + hand-off run (0..3; 3 measured best)
#endif
#ifndef PCST_NM_EARLY  // pair16: issue weight parts 0 and 1 before the prologue loads (0: after)
#define PCST_NM_EARLY 1
#endif
#ifndef PCST_NM_RD  // pair16 kernel: fragment groups read ahead of their MFMAs
#define PCST_NM_RD 1
#endif
#ifndef PCST_NM_PAIRX  // pair kernel: partner = wave ^ PAIRX (4: the partner shares the SIMD)
#define PCST_NM_PAIRX 4
#endif

struct TrBF16 {
  static constexpr int KS = 16;          // K per MFMA
  static constexpr int FRAG = 1024;      // bytes per A fragment
  static constexpr int OPB = 2;          // operands per 32-row block
  static constexpr int THREADS = 256;
  static constexpr int NCB = PCST_NM_NCB;  // 32-point column blocks per wave (A-fragment reuse)
  static constexpr int G = 4;              // fragments per pipelined LDS read group
  static constexpr bool kAsmReads = !(PCST_NM_EXPERIMENT & 8);
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
  // registers 4gi..4gi+3 of a C block -> elements 4(gi&1).. of operand gi>>1
  __device__ static void to_op4(const float (&v)[4], Op* o, int gi) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[gi >> 1][4 * (gi & 1) + j] = (__bf16)v[j];
  }
};

struct TrF32 {
  static constexpr int KS = 2;
  static constexpr int FRAG = 256;
  static constexpr int OPB = 16;
  static constexpr int THREADS = 256;
  static constexpr int NCB = 1;
  static constexpr int G = 8;
  static constexpr bool kAsmReads = false;
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
    if ((PCST_NM_EXPERIMENT & 1) && q >= 2) return;
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
    if (!(PCST_NM_EXPERIMENT & 2)) __syncthreads();
    ++part;
    issue(part + 1);
  }
  // LDS byte address of fragment f of part q for this lane
  __device__ uint32_t frag_addr(int q, int f) const {
    return (uint32_t)(uintptr_t)(lds + (q % kSlots) * kPart + f * TR::FRAG +
                                 (threadIdx.x & 63) * (int)sizeof(typename TR::A));
  }
  __device__ typename TR::A frag_at(int q, int f) const {
    return *reinterpret_cast<const typename TR::A*>(
        lds + (q % kSlots) * kPart + f * TR::FRAG + (threadIdx.x & 63) * (int)sizeof(typename TR::A));
  }
  __device__ typename TR::A frag(int f) const { return frag_at(part, f); }
};

// bf16 fragment reads in inline asm.  With LDS DMA in flight the compiler stops counting LDS
// waits and drains lgkmcnt(0) before every use, which exposes the LDS latency once per read
// group; here the reads are issued a group ahead and waited for with a counted
// s_waitcnt lgkmcnt(G) that is tied (in/out operands) to the registers it guards, so no MFMA
// can be scheduled above it.  LDS operations complete in order, so a counted wait also
// covers any compiler-issued LDS access older than these reads.
template <int OFF>
__device__ __forceinline__ bf16x8 lds_read_b128(uint32_t addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
// one fragment read at byte offset `off` from `addr` (off is a compile-time constant after
// unrolling; it goes into the instruction's offset field when it fits)
__device__ __forceinline__ bf16x8 lds_read_one(uint32_t addr, int off) {
  bf16x8 v;
  if (__builtin_constant_p(off) && off >= 0 && off < 65536)
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
  else
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr + off));
  return v;
}
// f32x4 read from LDS in asm (bias rows in the hot loop): like the fragment reads, invisible to
// the compiler's lgkmcnt accounting, so no compiler-inserted lgkmcnt(0) drains the fragment
// read pipeline at their first use; covered by the counted waits (LDS ops complete in order)
__device__ __forceinline__ f32x4 lds_read_f4(const float* p) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)p) : "memory");
  return v;
}
template <int N>
__device__ __forceinline__ void lgkm_wait4(bf16x8& a, bf16x8& b, bf16x8& c, bf16x8& d) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N));
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
  if constexpr (TR::kAsmReads) {
    static_assert(G == 4, "asm read path is written for groups of 4 fragments");
    const uint32_t a0 = st.frag_addr(q, base);
    A cur[4], nxt[4];
    cur[0] = lds_read_b128<0 * TR::FRAG>(a0);
    cur[1] = lds_read_b128<1 * TR::FRAG>(a0);
    cur[2] = lds_read_b128<2 * TR::FRAG>(a0);
    cur[3] = lds_read_b128<3 * TR::FRAG>(a0);
#pragma unroll
    for (int g = 0; g < N; g += 4) {
      if (g + 4 < N) {
        nxt[0] = lds_read_b128<0>(a0 + (g + 4) * TR::FRAG);
        nxt[1] = lds_read_b128<TR::FRAG>(a0 + (g + 4) * TR::FRAG);
        nxt[2] = lds_read_b128<2 * TR::FRAG>(a0 + (g + 4) * TR::FRAG);
        nxt[3] = lds_read_b128<3 * TR::FRAG>(a0 + (g + 4) * TR::FRAG);
        lgkm_wait4<4>(cur[0], cur[1], cur[2], cur[3]);
      } else {
        lgkm_wait4<0>(cur[0], cur[1], cur[2], cur[3]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = g + j;
#pragma unroll
        for (int cb = 0; cb < TR::NCB; ++cb)
          acc[(i / KPER) * AST + cb * ACB] =
              TR::mfma(cur[j], in[cb * ICB + i % KPER], acc[(i / KPER) * AST + cb * ACB]);
      }
      hook(g / 4);  // VALU work that fills this group's MFMA shadow
      if (g + 4 < N) {
#pragma unroll
        for (int j = 0; j < 4; ++j) cur[j] = nxt[j];
      }
    }
  } else {
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
    if constexpr (W2_OWN_PART) {
      // f32 parity path: W1 chunk and W2 chunk each fill a part; no cross-chunk overlap
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
    } else {
      // bf16: part c = [W1 rows of chunk c | W2 columns of chunk c].  Iteration c runs W1 of
      // chunk c+1 (part c+1) then W2 of chunk c (part c) with chunk c+1's ReLU/convert
      // epilogue in the W2 MFMA shadow.
      Op hb[NCB * OPB];
      st.next();
      {
        f32x16 hc[NCB];
        const f32x16 bc = bias_block(b1, h);
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) hc[cb] = bc;
        run_seq<TR, NSX, NSX, NSX, 1, 1>(st, st.part, 0, xb, hc);
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) act_op<TR>(hc[cb], true, &hb[cb * OPB]);
      }
      for (int c = 0; c < 15; ++c) {
        st.next();
        f32x16 hc[NCB];
        const f32x16 bc = bias_block(b1 + (c + 1) * 32, h);
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) hc[cb] = bc;
        run_seq<TR, NSX, NSX, NSX, 1, 1>(st, st.part, 0, xb, hc);
        Op hn[NCB * OPB];
        // W2 has 16 fragments = 4 groups of 4; group gi converts registers 4gi..4gi+3 of
        // each hc[cb] (half of operand gi/2)
        auto epi = [&](int gi) {
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb) {
            float v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = fmaxf(hc[cb][4 * gi + k], 0.0f);
            TR::to_op4(v, &hn[cb * OPB], gi);
          }
        };
        run_seq<TR, 8 * OPB, OPB, OPB, 1, 8>(st, st.part - 1, NSX, hb, x, epi);
#pragma unroll
        for (int i = 0; i < NCB * OPB; ++i) hb[i] = hn[i];
      }
      run_seq<TR, 8 * OPB, OPB, OPB, 1, 8>(st, st.part, NSX, hb, x);
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

// ============================================================================================
// bf16 production kernel: wave PAIRS.  A 512-thread workgroup (8 waves, 2 per SIMD) owns 128
// points; waves w and w^4 form a pair that shares 32 points and splits every layer's OUTPUT
// features: role 0 (waves 0-3) computes output blocks [0, NOB/2), role 1 the rest.  Per wave
// that halves the live activations (residual stream 4 x 32 rows fp32 = 64 VGPRs, the full bf16
// B operand of the next layer 64 VGPRs), so two waves fit on a SIMD (<= 256 VGPRs) and each
// hides the other's LDS waits, epilogues and barrier skew behind its MFMAs; the SIMD's MFMA
// work per 128 points is unchanged.
//   * dense layers: after a layer each wave converts its own output blocks to bf16 operands and
//     puts them in its LDS exchange area (8 KiB per wave); after the next part barrier it reads
//     the partner's half, so both hold the full K operand;
//   * residual blocks, per pair of hidden chunks (it, 8 + it): W1 part -- role 0 computes hidden
//     chunk it, role 1 chunk 8 + it (K = 256, 16 MFMAs each); each writes its ReLU'd bf16
//     chunk into its PARTNER's area; W2 part -- each reads the partner's chunk and accumulates
//     both chunks into its own 4 residual blocks (16 MFMAs).
// Exchange areas: a wave writes its layer outputs into its own area and its hidden chunks into
// the partner's, and reads the opposite; with the part barriers in between, no exchange needs
// a barrier of its own (see DESIGN.md §3 for the ordering argument).
// Weights stream through a 2-slot ring of 32 KiB parts; the packing (packing.py, pair layout)
// puts each role's fragments for a part in one half of it.
constexpr int kPairThreads = 512;
constexpr int kXBytes = 8192;  // exchange area per wave (8 operands x 1 KiB)

struct Streamer2 {
  static constexpr int kSlots = 2;
  static constexpr int kWaves = kPairThreads / 64;
  static constexpr int kPerWave = kPart / 1024 / kWaves;  // 1 KiB pieces per wave per part
  const char* blob;
  char* lds;
  int part;
  int nparts;
  int wave;
  __device__ void issue(int q) {
    if (q >= nparts) return;
    if ((PCST_NM_EXPERIMENT & 1) && q >= 2) return;
    const int lane = threadIdx.x & 63;
    char* dst = lds + (q & 1) * kPart + wave * kPerWave * 1024;
    const char* src = blob + (int64_t)q * kPart + wave * kPerWave * 1024;
#pragma unroll
    for (int i = 0; i < kPerWave; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src + i * 1024 + lane * 16),
                                       (__attribute__((address_space(3))) void*)(dst + i * 1024),
                                       16, 0, 0);
  }
  // __syncthreads waits for this wave's DMA (vmcnt 0) before the barrier: after it, the part
  // issued one part earlier has landed for every wave, and every wave is done with the slot
  // the next DMA overwrites.
  __device__ void begin() {
    issue(0);
    __syncthreads();
    issue(1);
  }
  // both slots are free at kernel start: parts 0 and 1 in flight before the caller's own
  // prologue loads; the caller's next __syncthreads (vmcnt 0 first) then has both landed
  __device__ void begin_early() {
    issue(0);
    issue(1);
  }
  __device__ void next() {
    if (!(PCST_NM_EXPERIMENT & 2)) __syncthreads();
    ++part;
    issue(part + 1);
  }
  __device__ uint32_t frag_addr(int q, int f) const {
    return (uint32_t)(uintptr_t)(lds + (q & 1) * kPart + f * 1024 + (threadIdx.x & 63) * 16);
  }
  __device__ bf16x8 frag_at(int q, int f) const {
    return *reinterpret_cast<const bf16x8*>(lds + (q & 1) * kPart + f * 1024 + (threadIdx.x & 63) * 16);
  }
};

template <int N>
__device__ __forceinline__ void xput(char* X, int area, const bf16x8* ops) {
  bf16x8* d = reinterpret_cast<bf16x8*>(X + area * kXBytes) + (threadIdx.x & 63);
#pragma unroll
  for (int i = 0; i < N; ++i) d[i * 64] = ops[i];
}
// the same at operand offset `at` (1 KiB units) of the area
template <int N>
__device__ __forceinline__ void xput_at(char* X, int area, int at, const bf16x8* ops) {
  if constexpr ((PCST_NM_EXPERIMENT & 32) != 0) return;  // timing only: no chunk hand-off
  bf16x8* d = reinterpret_cast<bf16x8*>(X + area * kXBytes) + at * 64 + (threadIdx.x & 63);
#pragma unroll
  for (int i = 0; i < N; ++i) d[i * 64] = ops[i];
}
// asm reads (see lds_read_f4): the hand-off registers are waited for by the next counted wait
template <int N>
__device__ __forceinline__ void xget_at(const char* X, int area, int at, bf16x8* ops) {
  if constexpr ((PCST_NM_EXPERIMENT & 32) != 0) return;
  const uint32_t a = (uint32_t)(uintptr_t)(X + area * kXBytes + at * 1024 + (threadIdx.x & 63) * 16);
#pragma unroll
  for (int i = 0; i < N; ++i)
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ops[i]) : "v"(a), "i"(i * 1024) : "memory");
}
template <int N>
__device__ __forceinline__ void xget(const char* X, int area, bf16x8* ops) {
  const bf16x8* d = reinterpret_cast<const bf16x8*>(X + area * kXBytes) + (threadIdx.x & 63);
#pragma unroll
  for (int i = 0; i < N; ++i) ops[i] = d[i * 64];
}

// NOWN own output blocks of K = 16*NS, streamed as parts that hold OWNPP own blocks per role.
template <int NOWN, int NS, int DONE = 0>
__device__ __forceinline__ void dense_pair(Streamer2& st, int role, const bf16x8* in, f32x16* acc) {
  constexpr int FPP = kPart / TrBF16::FRAG;
  constexpr int OWNPP = FPP / NS / 2;
  static_assert(OWNPP >= 1 && FPP % (2 * NS) == 0, "part must hold whole blocks for both roles");
  constexpr int NOW = (NOWN - DONE) < OWNPP ? (NOWN - DONE) : OWNPP;
  run_seq<TrBF16, NOW * NS, NS, NS, 1, 8>(st, st.part, role * OWNPP * NS, in, acc + DONE);
  if constexpr (DONE + NOW < NOWN) {
    st.next();
    dense_pair<NOWN, NS, DONE + NOW>(st, role, in, acc);
  }
}

// One wave's program; ROLE is a template parameter so that every register-array index is a
// compile-time constant (a role-dependent index into a register array would go to scratch).
template <int ROLE>
__device__ __forceinline__ void pair_wave(const float* __restrict__ cond, const float* sb,
                                          const float* sc, char* X, Streamer2& st, int wid,
                                          int64_t c0, int slot, float px, float py, float pz,
                                          int64_t p, int64_t P, float* __restrict__ out) {
  using TR = TrBF16;
  using Op = bf16x8;
  constexpr int R = ROLE;
  const int h = (threadIdx.x & 63) >> 5;
  const int mate = wid ^ PCST_NM_PAIRX;

  // ---- h1 = relu(W0 p + b0), all 128 rows in both roles (VALU), operand form
  Op h1[8];
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
    TR::to_op(v, &h1[ob * 2]);
  }

  Op xb[16];   // the full K = 256 operand: blocks 0-3 at [0, 8), blocks 4-7 at [8, 16)
  // own operands (already in xb[8R..]) -> own area; after the next part barrier the
  // partner's half is read into xb[8(1-R)..]
  auto put_own = [&](const f32x16* acc, bool relu) {
#pragma unroll
    for (int j = 0; j < 4; ++j) act_op<TR>(acc[j], relu, &xb[8 * R + 2 * j]);
    xput<8>(X, wid, &xb[8 * R]);
  };
  auto get_mate = [&]() { xget<8>(X, mate, &xb[8 * (1 - R)]); };

  // ---- h2 = relu(W2 h1 + b2): own blocks 4R + j
  {
    f32x16 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = bias_block(sb + kOffB2 + (4 * R + j) * 32, h);
    dense_pair<4, 8>(st, R, h1, acc);
    put_own(acc, true);
  }
  // ---- x = W4 h2 + cond[cloud]  (cond holds b4)
  f32x16 x[4];
  {
    const bool in_lds = slot >= 0 && slot < kCondSlots;
    const float* cs = in_lds ? sc + slot * 256 : cond + (c0 + slot) * 256;
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = bias_block(cs + (4 * R + j) * 32, h);
  }
  st.next();
  get_mate();
  dense_pair<4, 16>(st, R, xb, x);
  put_own(x, false);

  // ---- 6 residual blocks
  for (int layer = 0; layer < 6; ++layer) {
    const float* b1 = sb + kOffB1 + layer * 512;
    const float* b2 = sb + kOffBB2 + layer * 256;
    st.next();
    get_mate();
    for (int it = 0; it < 8; ++it) {
      if (it) st.next();
      // W1: hidden chunk (it | 8 + it) of this role, K = 256
      f32x16 hc = bias_block(b1 + (it + 8 * R) * 32, h);
      run_seq<TR, 16, 16, 16, 1, 1>(st, st.part, R * 16, xb, &hc);
      Op hb[4];   // [chunk it op 0, op 1, chunk 8+it op 0, op 1]
      act_op<TR>(hc, true, &hb[2 * R]);
      xput<2>(X, mate, &hb[2 * R]);          // into the partner's area
      st.next();
      xget<2>(X, wid, &hb[2 * (1 - R)]);     // the partner's chunk, from this wave's area
      // W2: own residual blocks += W2[block, chunk it] h_it + W2[block, chunk 8+it] h_8+it
      run_seq<TR, 16, 4, 4, 1, 1>(st, st.part, R * 16, hb, x);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] += bias_block(b2 + (4 * R + j) * 32, h);
    put_own(x, false);
  }

  // ---- output MLP 256 -> 256 -> 128 -> 3
  {
    f32x16 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = bias_block(sb + kOffO0 + (4 * R + j) * 32, h);
    st.next();
    get_mate();
    dense_pair<4, 16>(st, R, xb, acc);
    put_own(acc, true);
  }
  Op o2[8];  // K = 128 operand: blocks 0-1 at [0, 4), blocks 2-3 at [4, 8)
  {
    f32x16 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j] = bias_block(sb + kOffO2 + (2 * R + j) * 32, h);
    st.next();
    get_mate();
    dense_pair<2, 16>(st, R, xb, acc);
#pragma unroll
    for (int j = 0; j < 2; ++j) act_op<TR>(acc[j], true, &o2[4 * R + 2 * j]);
    xput<4>(X, wid, &o2[4 * R]);
  }
  st.next();
  xget<4>(X, mate, &o2[4 * (1 - R)]);
  f32x16 acc0 = f32x16{};
  run_seq<TR, 8, 8, 8, 1, 1>(st, st.part, 0, o2, &acc0);   // both roles: the same 3 rows
  if (R == 0 && p < P && h == 0) {
    out[p * 3 + 0] = acc0[0] + sb[kOffO4 + 0];
    out[p * 3 + 1] = acc0[1] + sb[kOffO4 + 1];
    out[p * 3 + 2] = acc0[2] + sb[kOffO4 + 2];
  }
}

__global__ __launch_bounds__(kPairThreads) void noise_mlp_pair_kernel(
    const float* __restrict__ pts, int64_t P, int64_t T, const float* __restrict__ cond,
    int64_t nclouds, const char* __restrict__ blob, int nparts, const float* __restrict__ bias,
    float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* X = smem + Streamer2::kSlots * kPart;
  float* sb = reinterpret_cast<float*>(X + Streamer2::kWaves * kXBytes);
  float* sc = sb + kBiasFloats;  // kCondSlots x 256
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t p0 = (int64_t)blockIdx.x * 128;
  const int64_t c0 = p0 / T;
  for (int i = tid; i < kBiasFloats; i += kPairThreads) sb[i] = bias[i];
  for (int i = tid; i < kCondSlots * 256; i += kPairThreads) {
    const int64_t c = c0 + i / 256;
    sc[i] = c < nclouds ? cond[c * 256 + (i % 256)] : 0.0f;
  }
  constexpr int PX = PCST_NM_PAIRX;
  const int pair = (wid & (PX - 1)) | ((wid / (2 * PX)) * PX);  // wave index without the role bit
  const int64_t p = p0 + pair * 32 + (lane & 31);
  const int64_t pc = p < P ? p : (P - 1);
  const float px = pts[pc * 3 + 0], py = pts[pc * 3 + 1], pz = pts[pc * 3 + 2];
  const int slot = (int)(pc / T - c0);
  __syncthreads();
  Streamer2 st{blob, smem, 0, nparts, wid};
  st.begin();
  if ((wid & PX) == 0)
    pair_wave<0>(cond, sb, sc, X, st, wid, c0, slot, px, py, pz, p, P, out);
  else
    pair_wave<1>(cond, sb, sc, X, st, wid, c0, slot, px, py, pz, p, P, out);
}

// ============================================================================================
// bf16 pair kernel on v_mfma_f32_16x16x32_bf16 ("pair16", precision code 2).  Same work split,
// part stream and exchange protocol as noise_mlp_pair_kernel; only the MFMA shape differs.
// Under MFMA load the chip holds a higher clock on 16x16x32 than on 32x32x16 at equal cycles
// per FLOP (MI355X_MICROARCH.md, DVFS item 7), and each 1 KiB weight fragment (16 rows x 32 k)
// feeds two MFMAs, one per 16-point column block of the wave's 32 points.
//   C/D: lane l holds rows 4(l>>4)+i (i < 4) of column l&15;
//   A:   lane l holds W[row l&15][kslot 8(l>>4)+j];  B: lane l holds X[kslot 8(l>>4)+j][col l&15].
// The operand of k-step s and column block cb is assembled from the accumulators of row blocks
// 2s and 2s+1: op[j] = acc(2s + (j>>2), cb)[j&3], i.e. kslot (g, j) is feature
// 32s + 16(j>>2) + 4g + (j&3) -- the permutation packing.py (_kmap16) applies to every K.
// Register arrays: operands [ks*2 + cb], accumulators [rb*2 + cb] (rb = 16-row block).
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// N fragments from LDS part q starting at fragment base; fragment i is (row block i / NKS,
// k-step i % NKS) and feeds both column blocks.  Same counted-wait read pipeline as run_seq.
template <int N, int NKS, class Hook = NoHook>
__device__ __forceinline__ void run16(const Streamer2& st, int q, int base, const bf16x8* in,
                                      f32x4* acc, const Hook& hook = Hook()) {
  static_assert(N % 4 == 0, "groups of 4 fragments");
  if constexpr ((PCST_NM_EXPERIMENT & 4) != 0) {  // timing only: no LDS fragment reads
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int rb = i / NKS, ks = i % NKS;
      acc[rb * 2 + 0] = mfma16(in[(ks + 1) % NKS * 2], in[ks * 2 + 0], acc[rb * 2 + 0]);
      acc[rb * 2 + 1] = mfma16(in[(ks + 1) % NKS * 2], in[ks * 2 + 1], acc[rb * 2 + 1]);
    }
    return;
  }
  const uint32_t a0 = st.frag_addr(q, base);
  constexpr int NG = N / 4;
  // groups of 4 fragments read PCST_NM_RD groups ahead of their MFMAs (1: cur + nxt; 2: + nn)
  bf16x8 cur[4], nxt[4], nn[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if constexpr ((PCST_NM_EXPERIMENT & 16) != 0)   // timing only: first group from registers
      cur[j] = in[(j + 1) % NKS * 2];
    else
      cur[j] = lds_read_one(a0, j * 1024);
  }
  if constexpr (PCST_NM_RD >= 2 && NG > 1) {
#pragma unroll
    for (int j = 0; j < 4; ++j) nxt[j] = lds_read_one(a0, 4096 + j * 1024);
  }
#pragma unroll
  for (int gg = 0; gg < NG; ++gg) {
    const int g = gg * 4;
    if constexpr (PCST_NM_RD >= 2) {
      if (gg + 2 < NG) {
#pragma unroll
        for (int j = 0; j < 4; ++j) nn[j] = lds_read_one(a0, (g + 8) * 1024 + j * 1024);
        lgkm_wait4<8>(cur[0], cur[1], cur[2], cur[3]);
      } else if (gg + 1 < NG) {
        lgkm_wait4<4>(cur[0], cur[1], cur[2], cur[3]);
      } else {
        lgkm_wait4<0>(cur[0], cur[1], cur[2], cur[3]);
      }
    } else {
      if (gg + 1 < NG) {
#pragma unroll
        for (int j = 0; j < 4; ++j) nxt[j] = lds_read_one(a0, (g + 4) * 1024 + j * 1024);
        lgkm_wait4<4>(cur[0], cur[1], cur[2], cur[3]);
      } else {
        lgkm_wait4<0>(cur[0], cur[1], cur[2], cur[3]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = g + j, rb = i / NKS, ks = i % NKS;
      acc[rb * 2 + 0] = mfma16(cur[j], in[ks * 2 + 0], acc[rb * 2 + 0]);
      acc[rb * 2 + 1] = mfma16(cur[j], in[ks * 2 + 1], acc[rb * 2 + 1]);
    }
    hook(gg);  // VALU / LDS-store work placed in this group's MFMA shadow
    if (gg + 1 < NG) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cur[j] = nxt[j];
        if constexpr (PCST_NM_RD >= 2) nxt[j] = nn[j];
      }
    }
  }
}

// NOWN own row blocks of K = 32*NKS, streamed as parts that hold OWNPP own blocks per role.
template <int NOWN, int NKS, int DONE = 0>
__device__ __forceinline__ void dense16(Streamer2& st, int role, const bf16x8* in, f32x4* acc) {
  constexpr int FPP = kPart / 1024;
  constexpr int OWNPP = FPP / NKS / 2;
  static_assert(OWNPP >= 1 && FPP % (2 * NKS) == 0, "part must hold whole blocks for both roles");
  constexpr int NOW = (NOWN - DONE) < OWNPP ? (NOWN - DONE) : OWNPP;
  run16<NOW * NKS, NKS>(st, st.part, role * OWNPP * NKS, in, acc + 2 * DONE);
  if constexpr (DONE + NOW < NOWN) {
    st.next();
    dense16<NOWN, NKS, DONE + NOW>(st, role, in, acc);
  }
}

// the 4 bias values of a 16-row block in accumulator order
__device__ __forceinline__ f32x4 bias4(const float* b, int g) {
  f32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = b[4 * g + i];
  return v;
}

// accumulators of row blocks (2t, 2t+1) x column block cb -> operand of local k-step t
__device__ __forceinline__ bf16x8 op16(const f32x4& lo, const f32x4& hi, bool relu) {
  bf16x8 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[i] = (__bf16)(relu ? fmaxf(lo[i], 0.0f) : lo[i]);
    o[4 + i] = (__bf16)(relu ? fmaxf(hi[i], 0.0f) : hi[i]);
  }
  return o;
}
// NRB accumulator row blocks [rb*2 + cb] -> NRB/2 k-steps of operands [t*2 + cb]
template <int NRB>
__device__ __forceinline__ void ops16(const f32x4* acc, bool relu, bf16x8* out) {
#pragma unroll
  for (int t = 0; t < NRB / 2; ++t)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) out[t * 2 + cb] = op16(acc[(2 * t) * 2 + cb], acc[(2 * t + 1) * 2 + cb], relu);
}

template <int ROLE>
__device__ __forceinline__ void pair16_wave(const float* __restrict__ cond, const float* sb,
                                            const float* sc, char* X, Streamer2& st, int wid,
                                            int64_t c0, const int (&slot)[2], const float (&px)[2],
                                            const float (&py)[2], const float (&pz)[2],
                                            const int64_t (&p)[2], int64_t P, float* __restrict__ out) {
  using Op = bf16x8;
  constexpr int R = ROLE;
  const int g = (threadIdx.x & 63) >> 4;
  const int mate = wid ^ PCST_NM_PAIRX;

  // ---- h1 = relu(W0 p + b0): 128 features = 4 k-steps, both column blocks (VALU)
  Op h1[8];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      Op o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = 32 * s + 16 * (j >> 2) + 4 * g + (j & 3);
        float v = sb[kOffB0 + f];
        v = fmaf(sb[kOffW0 + f * 3 + 0], px[cb], v);
        v = fmaf(sb[kOffW0 + f * 3 + 1], py[cb], v);
        v = fmaf(sb[kOffW0 + f * 3 + 2], pz[cb], v);
        o[j] = (__bf16)fmaxf(v, 0.0f);
      }
      h1[s * 2 + cb] = o;
    }

  Op xb[16];  // the full K = 256 operand, [ks*2 + cb]; own k-steps 4R..4R+3 at [8R, 8R+8)
  auto put_own = [&](const f32x4* acc, bool relu) {
    ops16<8>(acc, relu, &xb[8 * R]);
    xput<8>(X, wid, &xb[8 * R]);
  };
  auto get_mate = [&]() { xget<8>(X, mate, &xb[8 * (1 - R)]); };

  // ---- h2 = relu(W2 h1 + b2): own row blocks 8R + rb
  {
    f32x4 acc[16];
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) acc[rb * 2] = acc[rb * 2 + 1] = bias4(sb + kOffB2 + (8 * R + rb) * 16, g);
    dense16<8, 4>(st, R, h1, acc);
    put_own(acc, true);
  }
  // ---- x = W4 h2 + cond[cloud]  (cond holds b4)
  f32x4 x[16];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const bool in_lds = slot[cb] >= 0 && slot[cb] < kCondSlots;
    const float* cs = in_lds ? sc + slot[cb] * 256 : cond + (c0 + slot[cb]) * 256;
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) x[rb * 2 + cb] = bias4(cs + (8 * R + rb) * 16, g);
  }
  st.next();
  get_mate();
  dense16<8, 8>(st, R, xb, x);
  put_own(x, false);

  // ---- 6 residual blocks; per pair of hidden chunks (it, 8 + it): W1 part (own chunk it + 8R,
  // 2 row blocks x 8 k-steps), W2 part (own 8 row blocks x k-steps {chunk it, chunk 8 + it}).
  // Software-pipelined (parts packed W1(0), W1(1), W2(0), W1(2), W2(1), ...): W1 of chunk it + 1
  // runs before W2 of chunk it, so the partner's chunk it -- written before the barrier that
  // opens W1(it + 1) -- is read at the start of that part and is in registers when W2(it)
  // starts, and chunk it + 1's ReLU/bf16 epilogue and hand-off run after the W2 MFMAs are
  // issued.  The hand-off alternates between two 2 KiB slots of the partner's area (chunk c in
  // slot c & 1): a wave writes chunk it + 1 while its partner may still read chunk it.
  for (int layer = 0; layer < 6; ++layer) {
    const float* b1 = sb + kOffB1 + layer * 512;
    const float* b2 = sb + kOffBB2 + layer * 256;
    st.next();
    get_mate();
    Op hb[4];  // [chunk it: cb 0, cb 1 | chunk 8 + it: cb 0, cb 1]
    {
      f32x4 hc[4];
      hc[0] = hc[1] = bias4(b1 + (8 * R) * 32, g);
      hc[2] = hc[3] = bias4(b1 + (8 * R) * 32 + 16, g);
      run16<16, 8>(st, st.part, R * 16, xb, hc);
      ops16<2>(hc, true, &hb[2 * R]);
      xput_at<2>(X, mate, 0, &hb[2 * R]);
    }
    for (int it = 0; it < 8; ++it) {
      f32x4 hn[4];
      if (it < 7) {
        st.next();                                           // part W1(it + 1)
        xget_at<2>(X, wid, (it & 1) * 2, &hb[2 * (1 - R)]);  // the partner's chunk it
        hn[0] = hn[1] = lds_read_f4(b1 + (it + 1 + 8 * R) * 32 + 4 * g);
        hn[2] = hn[3] = lds_read_f4(b1 + (it + 1 + 8 * R) * 32 + 16 + 4 * g);
        run16<16, 8>(st, st.part, R * 16, xb, hn);
        st.next();                                           // part W2(it)
      } else {
        st.next();                                           // part W2(7)
        xget_at<2>(X, wid, (it & 1) * 2, &hb[2 * (1 - R)]);
      }
      if (it < 7) {
        // chunk it + 1's epilogue and hand-off in the MFMA shadow of W2's fragment group
        // PCST_NM_EPI_GROUP (after the last: measured 1-4 % faster than after the first or
        // second, where the VALU and LDS stores compete with the fragment reads)
        Op hbn[2];
        auto epi = [&](int gg) {
          if (gg == PCST_NM_EPI_GROUP) {
            ops16<2>(hn, true, hbn);
            xput_at<2>(X, mate, ((it + 1) & 1) * 2, hbn);
          }
        };
        run16<16, 2>(st, st.part, R * 16, hb, x, epi);
        hb[2 * R] = hbn[0];
        hb[2 * R + 1] = hbn[1];
      } else {
        run16<16, 2>(st, st.part, R * 16, hb, x);
      }
    }
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      const f32x4 b = bias4(b2 + (8 * R + rb) * 16, g);
      x[rb * 2] += b;
      x[rb * 2 + 1] += b;
    }
    put_own(x, false);
  }

  // ---- output MLP 256 -> 256 -> 128 -> 3
  {
    f32x4 acc[16];
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) acc[rb * 2] = acc[rb * 2 + 1] = bias4(sb + kOffO0 + (8 * R + rb) * 16, g);
    st.next();
    get_mate();
    dense16<8, 8>(st, R, xb, acc);
    put_own(acc, true);
  }
  Op o2[8];  // K = 128 operand [ks*2 + cb]; own k-steps 2R, 2R+1 at [4R, 4R+4)
  {
    f32x4 acc[8];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) acc[rb * 2] = acc[rb * 2 + 1] = bias4(sb + kOffO2 + (4 * R + rb) * 16, g);
    st.next();
    get_mate();
    dense16<4, 8>(st, R, xb, acc);
    ops16<4>(acc, true, &o2[4 * R]);
    xput<4>(X, wid, &o2[4 * R]);
  }
  st.next();
  xget<4>(X, mate, &o2[4 * (1 - R)]);
  f32x4 acc0[2] = {f32x4{}, f32x4{}};
  run16<4, 4>(st, st.part, 0, o2, acc0);  // both roles: the same 3 rows
  if (R == 0 && g == 0) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
      if (p[cb] < P) {
        out[p[cb] * 3 + 0] = acc0[cb][0] + sb[kOffO4 + 0];
        out[p[cb] * 3 + 1] = acc0[cb][1] + sb[kOffO4 + 1];
        out[p[cb] * 3 + 2] = acc0[cb][2] + sb[kOffO4 + 2];
      }
  }
}

// The MLP's last work-group waits for a device flag (pcst_noise_mlp_then_wait): every work-group
// counts itself out (agent scope) after its rows are written; the last one resets the counter and
// polls *flag >= value (bounded: a timeout sets *err), so the launch completes only after the
// flag's producer on another stream.  No work-group waits while another has yet to start, so the
// producer always finds free CUs.
constexpr int kMlpWaitPolls = 1 << 26;
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

__global__ __launch_bounds__(kPairThreads) void noise_mlp_pair16_kernel(
    const float* __restrict__ pts, int64_t P, int64_t T, const float* __restrict__ cond,
    int64_t nclouds, const char* __restrict__ blob, int nparts, const float* __restrict__ bias,
    float* __restrict__ out, const uint32_t* __restrict__ wflag, uint32_t wvalue,
    uint32_t* __restrict__ wcount, int32_t* __restrict__ werr, int64_t wpolls,
    uint32_t* __restrict__ sflag, uint32_t svalue) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // start signal (pcst_noise_mlp_ex): the launch has begun, so every kernel queued before it on
  // this stream has completed (and released its writes at its end): one agent-scope store
  // publishes that to a waiter on another stream without a signal launch of its own
  if (sflag && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(sflag, svalue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  char* X = smem + Streamer2::kSlots * kPart;
  float* sb = reinterpret_cast<float*>(X + Streamer2::kWaves * kXBytes);
  float* sc = sb + kBiasFloats;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t p0 = (int64_t)blockIdx.x * 128;
  const int64_t c0 = p0 / T;
  Streamer2 st{blob, smem, 0, nparts, wid};
  if (PCST_NM_EARLY) st.begin_early();  // the first two weight parts under the prologue loads
  for (int i = tid; i < kBiasFloats; i += kPairThreads) sb[i] = bias[i];
  for (int i = tid; i < kCondSlots * 256; i += kPairThreads) {
    const int64_t c = c0 + i / 256;
    sc[i] = c < nclouds ? cond[c * 256 + (i % 256)] : 0.0f;
  }
  constexpr int PX = PCST_NM_PAIRX;
  const int pair = (wid & (PX - 1)) | ((wid / (2 * PX)) * PX);
  int64_t p[2];
  int slot[2];
  float px[2], py[2], pz[2];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    p[cb] = p0 + pair * 32 + cb * 16 + (lane & 15);
    const int64_t pc = p[cb] < P ? p[cb] : (P - 1);
    px[cb] = pts[pc * 3 + 0];
    py[cb] = pts[pc * 3 + 1];
    pz[cb] = pts[pc * 3 + 2];
    slot[cb] = (int)(pc / T - c0);
  }
  __syncthreads();
  if (!PCST_NM_EARLY) st.begin();
  if ((wid & PX) == 0)
    pair16_wave<0>(cond, sb, sc, X, st, wid, c0, slot, px, py, pz, p, P, out);
  else
    pair16_wave<1>(cond, sb, sc, X, st, wid, c0, slot, px, py, pz, p, P, out);
  if (wflag) last_group_wait(wflag, wvalue, wcount, werr, wpolls, threadIdx.x == 0);
}

// ============================================================================================
// bf16 "solo" kernel on v_mfma_f32_16x16x32_bf16 (precision code 3).  Every wave owns 32 points
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

#ifndef PCST_SOLO_NCB
#define PCST_SOLO_NCB 2
#endif
constexpr int kNCB = PCST_SOLO_NCB;    // column blocks per wave of the product instantiation
constexpr int kPts = 256;               // points per work-group
constexpr int kSP = 65536;              // superpart bytes
constexpr int kNF = kSP / 1024;         // fragments per superpart
#ifndef PCST_SOLO_KD
#define PCST_SOLO_KD 2
#endif
#ifndef PCST_SOLO_PRIO
#define PCST_SOLO_PRIO 0
#endif
#ifndef PCST_SOLO_STAMPS  // experiment builds (tools/solo_bench.hip): per-wave clock stamps
#define PCST_SOLO_STAMPS 0
#endif
#ifndef PCST_SOLO_EXP  // timing-only experiment builds (wrong results): 1 no DMA after superpart 1,
#define PCST_SOLO_EXP 0  // 2 no s_barrier, 4 fragments from registers (no LDS fragment reads)
#endif
constexpr int kD = PCST_SOLO_KD;        // fragment reads in flight ahead of their MFMAs
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

// PCST_SOLO_PRIO 2 (experiment): waves 4-7 lead the first half of a superpart, waves 0-3 the second
__device__ __forceinline__ void prio_start() {
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 4) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}
__device__ __forceinline__ void prio_flip() {
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 4) __builtin_amdgcn_s_setprio(0);
  else __builtin_amdgcn_s_setprio(1);
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
  if constexpr ((PCST_SOLO_EXP & 4) != 0) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int i = 0; i <= kD; ++i) w[i] = w[i % NPRO];
  }
  auto it = [&](auto fc) {
    constexpr int f = decltype(fc)::value;
    xr(fc);
    if constexpr ((PCST_SOLO_EXP & 4) == 0) {
      if constexpr (f + kD < S::NF) w[(f + kD) % (kD + 1)] = lds_read_one(a, (f + kD) * 1024);
      wait_frag<frag_after<S>(f)>(w[f % (kD + 1)]);
    }
    mf(fc, w[f % (kD + 1)]);
    dm(fc);
    po(fc);
    if constexpr (PCST_SOLO_PRIO == 2 && f == 31) prio_flip();
  };
  if constexpr (PCST_SOLO_PRIO == 2) prio_start();
  sfor<0, S::NF>(it);
}

// every wave: its own DMAs have landed and it is done with the current slot; then the barrier
__device__ __forceinline__ void sp_barrier() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if (!(PCST_SOLO_EXP & 2)) __builtin_amdgcn_s_barrier();
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

#ifndef PCST_SOLO_DMA  // 0: the next superpart's pieces at fragments 1, 5, .., 29; 1: at 1..8
#define PCST_SOLO_DMA 0
#endif

template <int NCB>  // 16-point column blocks per wave: 2 (8 waves, 2 per SIMD) or 4 (4 waves, 1 per SIMD)
__global__ __launch_bounds__(16 / NCB * 64) void noise_mlp_solo_kernel(
    const float* __restrict__ pts, int64_t P, int64_t T, const float* __restrict__ cond,
    int64_t nclouds, const char* __restrict__ blob, int nsp, const float* __restrict__ bias,
    float* __restrict__ out, const uint32_t* __restrict__ wflag, uint32_t wvalue,
    uint32_t* __restrict__ wcount, int32_t* __restrict__ werr, int64_t wpolls,
    uint32_t* __restrict__ sflag, uint32_t svalue) {
  constexpr int NW = 16 / NCB;  // waves per work-group
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (sflag && blockIdx.x == 0 && threadIdx.x == 0)  // see noise_mlp_pair16_kernel
    __hip_atomic_store(sflag, svalue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (PCST_SOLO_PRIO && wid >= 4) __builtin_amdgcn_s_setprio(1);
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const uint32_t ba = lds0 + kBiasLds + 16 * g;  // bias rows 4g..4g+3 of a 16-row block
  long long st_t0 = 0, st_r0 = 0, st_dma = 0, st_bar = 0, st_head = 0, st_res = 0;
  if (PCST_SOLO_STAMPS) {
    st_t0 = __builtin_amdgcn_s_memtime();
    st_r0 = __builtin_amdgcn_s_memrealtime();
  }
  // every wave: its own DMAs have landed and it is done with the current slot; then the barrier
  int st_nb = 0;  // stamps mode 2: each barrier's arrival time (cycles since the kernel start)
  auto bar = [&]() {
    if (PCST_SOLO_STAMPS == 2 && lane == 0) {
      out[P * 3 + ((int64_t)blockIdx.x * 8 + wid) * 64 + st_nb] = (float)(__builtin_amdgcn_s_memtime() - st_t0);
      ++st_nb;
    }
    if (PCST_SOLO_STAMPS == 1) {
      const long long t0 = __builtin_amdgcn_s_memtime();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const long long t1 = __builtin_amdgcn_s_memtime();
      sp_barrier();
      const long long t2 = __builtin_amdgcn_s_memtime();
      st_dma += t1 - t0;
      st_bar += t2 - t1;
    } else {
      sp_barrier();
    }
  };
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
  auto piece2 = [&](int s, int i) {  // PCST_SOLO_PRIO 3: 16 pieces per wave of waves 0-3
    const int off = wid * 16384 + i * 1024;
    const int src = s < nsp ? s : nsp - 1;
    __builtin_amdgcn_global_load_lds((const void*)(blob + (int64_t)src * kSP + off + lane * 16),
                                     (__attribute__((address_space(3))) void*)(smem + (s & 1) * kSP + off),
                                     16, 0, 0);
  };
  // the next superpart's 8 pieces
  auto dm = [&](auto fc) {
    constexpr int f = decltype(fc)::value;
    if ((PCST_SOLO_EXP & 1) && sp >= 1) return;
    if constexpr (PCST_SOLO_PRIO == 3) {  // experiment: the older waves (0-3) carry the DMA
      if constexpr (f % 2 == 1 && f < 32) {
        if (wid < 4) {
          piece2(sp + 1, f / 2);
        }
      }
      return;
    }
    if constexpr (PCST_SOLO_DMA == 0 && NW == 8 && f % 4 == 1 && f < 32) piece(sp + 1, f / 4);
    if constexpr (PCST_SOLO_DMA == 0 && NW == 4 && f % 2 == 1 && f < 32) piece(sp + 1, f / 2);
    if constexpr (PCST_SOLO_DMA == 1 && f >= 1 && f <= 8) piece(sp + 1, f - 1);
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
  if (PCST_SOLO_STAMPS) st_head = __builtin_amdgcn_s_memtime();

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
  if (PCST_SOLO_STAMPS) st_res = __builtin_amdgcn_s_memtime();

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
  if (PCST_SOLO_STAMPS == 2 && lane == 0)
    out[P * 3 + ((int64_t)blockIdx.x * 8 + wid) * 64 + 63] = (float)(__builtin_amdgcn_s_memtime() - st_t0);
  if (PCST_SOLO_STAMPS == 1 && lane == 0) {  // {cycles, DMA wait, barrier, 100 MHz ticks, head, residual, tail, 1}
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float* st = out + P * 3 + ((int64_t)blockIdx.x * 8 + wid) * 8;
    st[0] = (float)(t1 - st_t0);
    st[1] = (float)st_dma;
    st[2] = (float)st_bar;
    st[3] = (float)(r1 - st_r0);
    st[4] = (float)(st_head - st_t0);
    st[5] = (float)(st_res - st_head);
    st[6] = (float)(t1 - st_res);
    st[7] = 1.0f;
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

// Bytes of the packed weight blob for a precision: 0 = f32 (parity), 1 = bf16.
extern "C" int64_t pcst_noise_mlp_blob_bytes(int precision) {
  if (precision == 3) return (int64_t)solo::kNSP * solo::kSP;  // 55 superparts (packing.py SOLO16)
  // every layer starts on a fresh 32 KiB part (see packing.py); residual chunks take one part
  // (bf16: W1c | W2c) or two (f32: W1c, W2c).  The two bf16 layouts (1: 32x32x16 fragments,
  // 2: 16x16x32 fragments) hold the same fragments per part, so their blobs have one size.
  if (precision == 2) precision = 1;
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
  hipLaunchKernelGGL(cond_bias_kernel, dim3((unsigned)nclouds, 256 / 32), dim3(256), 0,
                     as_stream(stream), t,
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
  PCST_CHECK_ARG(precision >= 0 && precision <= 3,
                 "noise_mlp: precision must be 0 (f32), 1 (bf16 32x32x16), 2 (bf16 pair16) or 3 (bf16 solo)");
  PCST_CHECK_ARG(blob_bytes == pcst_noise_mlp_blob_bytes(precision), "noise_mlp: blob size %lld != %lld",
                 (long long)blob_bytes, (long long)pcst_noise_mlp_blob_bytes(precision));
  PCST_CHECK_ARG(((uintptr_t)blob & 15) == 0, "noise_mlp: blob must be 16-byte aligned");
  if (P == 0) return PCST_OK;
  hipStream_t s = as_stream(stream);
  if (precision == 3) {
    hipLaunchKernelGGL(solo::noise_mlp_solo_kernel<solo::kNCB>, dim3((unsigned)cdiv(P, solo::kPts)), dim3(16 / solo::kNCB * 64),
                       solo::kLds, s, pts, P, points_per_cloud, cond, nclouds, (const char*)blob,
                       solo::kNSP, bias, out, (const uint32_t*)nullptr, 0u, (uint32_t*)nullptr,
                       (int32_t*)nullptr, (int64_t)0, (uint32_t*)nullptr, 0u);
  } else if (precision == 2) {
    const size_t lds = Streamer2::kSlots * kPart + Streamer2::kWaves * kXBytes +
                       (kBiasFloats + kCondSlots * 256) * sizeof(float);
    hipLaunchKernelGGL(noise_mlp_pair16_kernel, dim3((unsigned)cdiv(P, 128)), dim3(kPairThreads),
                       lds, s, pts, P, points_per_cloud, cond, nclouds, (const char*)blob,
                       (int)(blob_bytes / kPart), bias, out, (const uint32_t*)nullptr, 0u,
                       (uint32_t*)nullptr, (int32_t*)nullptr, (int64_t)0, (uint32_t*)nullptr, 0u);
  } else if (precision == 1) {
    const size_t lds = Streamer2::kSlots * kPart + Streamer2::kWaves * kXBytes +
                       (kBiasFloats + kCondSlots * 256) * sizeof(float);
    hipLaunchKernelGGL(noise_mlp_pair_kernel, dim3((unsigned)cdiv(P, 128)), dim3(kPairThreads),
                       lds, s, pts, P, points_per_cloud, cond, nclouds, (const char*)blob,
                       (int)(blob_bytes / kPart), bias, out);
  } else
    launch_noise_mlp<TrF32>(pts, P, points_per_cloud, cond, nclouds, blob, blob_bytes, bias, out, s);
  PCST_LAUNCH_CHECK("noise_mlp");
  return PCST_OK;
}

extern "C" int pcst_noise_mlp_then_wait(const float* pts, int64_t P, int64_t points_per_cloud,
                                        const float* cond, int64_t nclouds, const void* blob,
                                        int64_t blob_bytes, const float* bias, float* out,
                                        const uint32_t* flag, uint32_t value, uint32_t* counter,
                                        int32_t* err, int64_t max_polls, void* stream) {
  PCST_CHECK_ARG(P > 0 && points_per_cloud > 0 && nclouds > 0, "noise_mlp_then_wait: bad shape");
  PCST_CHECK_ARG(P <= points_per_cloud * nclouds, "noise_mlp_then_wait: P exceeds clouds*points");
  PCST_CHECK_ARG(blob_bytes == pcst_noise_mlp_blob_bytes(2), "noise_mlp_then_wait: blob size %lld != %lld",
                 (long long)blob_bytes, (long long)pcst_noise_mlp_blob_bytes(2));
  PCST_CHECK_ARG(((uintptr_t)blob & 15) == 0, "noise_mlp_then_wait: blob must be 16-byte aligned");
  PCST_CHECK_ARG(flag && counter, "noise_mlp_then_wait: null flag or counter");
  const size_t lds = Streamer2::kSlots * kPart + Streamer2::kWaves * kXBytes +
                     (kBiasFloats + kCondSlots * 256) * sizeof(float);
  hipLaunchKernelGGL(noise_mlp_pair16_kernel, dim3((unsigned)cdiv(P, 128)), dim3(kPairThreads), lds,
                     as_stream(stream), pts, P, points_per_cloud, cond, nclouds, (const char*)blob,
                     (int)(blob_bytes / kPart), bias, out, flag, value, counter, err,
                     max_polls > 0 ? max_polls : (int64_t)kMlpWaitPolls, (uint32_t*)nullptr, 0u);
  PCST_LAUNCH_CHECK("noise_mlp_then_wait");
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
                                 const uint32_t* wait_flag, uint32_t wait_value,
                                 uint32_t* wait_counter, int32_t* wait_err, int64_t max_polls,
                                 void* stream) {
  if ((precision != 2 && precision != 3) || P == 0) {  // no fused form: separate launches
    if (start_flag) {
      hipLaunchKernelGGL(mlp_start_signal_kernel, dim3(1), dim3(64), 0, as_stream(stream), start_flag,
                         start_value);
      PCST_LAUNCH_CHECK("noise_mlp_ex: start signal");
    }
    const int rc = pcst_noise_mlp(pts, P, points_per_cloud, cond, nclouds, blob, blob_bytes, bias,
                                  precision, out, stream);
    if (rc != PCST_OK || !wait_flag) return rc;
    return pcst_signal_wait(wait_flag, wait_value, wait_err, max_polls, stream);
  }
  PCST_CHECK_ARG(P > 0 && points_per_cloud > 0 && nclouds > 0, "noise_mlp_ex: bad shape");
  PCST_CHECK_ARG(P <= points_per_cloud * nclouds, "noise_mlp_ex: P exceeds clouds*points");
  PCST_CHECK_ARG(blob_bytes == pcst_noise_mlp_blob_bytes(precision), "noise_mlp_ex: blob size %lld != %lld",
                 (long long)blob_bytes, (long long)pcst_noise_mlp_blob_bytes(precision));
  PCST_CHECK_ARG(((uintptr_t)blob & 15) == 0, "noise_mlp_ex: blob must be 16-byte aligned");
  PCST_CHECK_ARG(!wait_flag || wait_counter, "noise_mlp_ex: a wait needs its counter");
  if (precision == 3) {
    hipLaunchKernelGGL(solo::noise_mlp_solo_kernel<solo::kNCB>, dim3((unsigned)cdiv(P, solo::kPts)), dim3(16 / solo::kNCB * 64),
                       solo::kLds, as_stream(stream), pts, P, points_per_cloud, cond, nclouds,
                       (const char*)blob, solo::kNSP, bias, out, wait_flag, wait_value, wait_counter,
                       wait_err, max_polls > 0 ? max_polls : (int64_t)kMlpWaitPolls, start_flag,
                       start_value);
    PCST_LAUNCH_CHECK("noise_mlp_ex");
    return PCST_OK;
  }
  const size_t lds = Streamer2::kSlots * kPart + Streamer2::kWaves * kXBytes +
                     (kBiasFloats + kCondSlots * 256) * sizeof(float);
  hipLaunchKernelGGL(noise_mlp_pair16_kernel, dim3((unsigned)cdiv(P, 128)), dim3(kPairThreads), lds,
                     as_stream(stream), pts, P, points_per_cloud, cond, nclouds, (const char*)blob,
                     (int)(blob_bytes / kPart), bias, out, wait_flag, wait_value, wait_counter,
                     wait_err, max_polls > 0 ? max_polls : (int64_t)kMlpWaitPolls, start_flag,
                     start_value);
  PCST_LAUNCH_CHECK("noise_mlp_ex");
  return PCST_OK;
}
