// Timing harness for the bf16 noise-MLP kernels (perf experiments only, not product code).
// Built by tools/solo_variants.sh once per knob setting (PCST_SOLO_KD / PCST_SOLO_PRIO /
// PCST_SOLO_STAMPS, see csrc/noise_mlp.hip solo::); each binary times the bench launch (2 x 30000
// points) and the 32-cloud launch (64 x 30000) for precisions 2 (pair16) and 3 (solo), alternating,
// with HIP events on random bf16 weights, and with PCST_SOLO_STAMPS prints the per-wave clock
// stamps of the solo kernel.
#include "../pointcloud_style_transfer_amd/csrc/noise_mlp.hip"

#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));  \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

namespace pcst {
void set_error(const char* fmt, ...) { (void)fmt; }
}  // namespace pcst
extern "C" int pcst_signal_wait(const uint32_t*, uint32_t, int32_t*, int64_t, void*) { return 0; }

static float rnd(uint32_t& s) {
  s = s * 1664525u + 1013904223u;
  return (float)((s >> 8) & 0xffff) / 65536.0f - 0.5f;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 40;
  const int64_t T = 30000;
  const int64_t Cmax = 64, Pmax = T * Cmax;
  uint32_t s = 12345;
  std::vector<float> h_pts(Pmax * 3), h_cond(Cmax * 256), h_bias(kBiasFloats);
  for (auto& v : h_pts) v = 2.0f * rnd(s);
  for (auto& v : h_cond) v = 0.1f * rnd(s);
  for (auto& v : h_bias) v = 0.05f * rnd(s);
  float *pts, *cond, *bias, *out;
  CK(hipMalloc(&pts, Pmax * 12));
  CK(hipMalloc(&cond, Cmax * 1024));
  CK(hipMalloc(&bias, kBiasFloats * 4));
  const int64_t stamp_floats = (Pmax / 256 + 1) * 8 * 64;
  CK(hipMalloc(&out, Pmax * 12 + stamp_floats * 4));
  CK(hipMemcpy(pts, h_pts.data(), Pmax * 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(cond, h_cond.data(), Cmax * 1024, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, h_bias.data(), kBiasFloats * 4, hipMemcpyHostToDevice));
  void* blob[4] = {};
  int64_t bb[4] = {};
  for (int prec : {2, 3}) {
    bb[prec] = pcst_noise_mlp_blob_bytes(prec);
    std::vector<uint16_t> h(bb[prec] / 2);
    for (auto& v : h) {
      float f = 0.06f * rnd(s);
      uint32_t u;
      std::memcpy(&u, &f, 4);
      v = (uint16_t)(u >> 16);
    }
    CK(hipMalloc(&blob[prec], bb[prec]));
    CK(hipMemcpy(blob[prec], h.data(), bb[prec], hipMemcpyHostToDevice));
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // argv[2]: clouds (2 or 64; default both), argv[3]: precision (2 or 3; default both)
  const int only_c = argc > 2 ? atoi(argv[2]) : 0, only_p = argc > 3 ? atoi(argv[3]) : 0;
  for (int64_t C : {2, 64}) {
    if (only_c && C != only_c) continue;
    const int64_t P = T * C;
    const int n = C == 2 ? iters : iters / 8 + 2;
    for (int rep = 0; rep < 2; ++rep)
      for (int prec : {2, 3}) {
        if (only_p && prec != only_p) continue;
        for (int i = 0; i < 3; ++i)
          if (pcst_noise_mlp(pts, P, T, cond, C, blob[prec], bb[prec], bias, prec, out, st)) return 2;
        CK(hipMemset(out + P * 3, 0, stamp_floats * 4));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < n; ++i) pcst_noise_mlp(pts, P, T, cond, C, blob[prec], bb[prec], bias, prec, out, st);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / n;
        const double tf = 3540480.0 * P / (us * 1e-6) / 1e12;
        printf("ncb=%d kd=%d prio=%d dma=%d exp=%d prec=%d clouds=%lld  %.1f us/launch  %.1f TFLOP/s  frac %.4f\n", PCST_SOLO_NCB, PCST_SOLO_KD,
               PCST_SOLO_PRIO, PCST_SOLO_DMA, PCST_SOLO_EXP, prec, (long long)C, us, tf, tf / 2500.0);
        if (PCST_SOLO_STAMPS == 2 && prec == 3 && rep == 1) {
          // per barrier k: arrival spread over the 8 waves and |wave w - wave w+4| (one SIMD), mean
          // over work-groups; then each superpart's duration (first arrival to first arrival)
          const int64_t nwg = (P + 255) / 256;
          std::vector<float> h(nwg * 8 * 64);
          CK(hipMemcpy(h.data(), out + P * 3, h.size() * 4, hipMemcpyDeviceToHost));
          printf("  barrier  spread  simd-pair  sp-cycles\n");
          for (int k = 0; k < 56; ++k) {
            double spread = 0, pair = 0, dur = 0;
            for (int64_t wg = 0; wg < nwg; ++wg) {
              const float* a = &h[wg * 512];
              float mn = 1e30f, mx = -1e30f, mn2 = 1e30f;
              for (int w = 0; w < 8; ++w) {
                mn = fminf(mn, a[w * 64 + k]);
                mx = fmaxf(mx, a[w * 64 + k]);
                if (k + 1 < 56) mn2 = fminf(mn2, a[w * 64 + (k + 1 < 55 ? k + 1 : 63)]);
              }
              spread += mx - mn;
              for (int w = 0; w < 4; ++w) pair += fabsf(a[w * 64 + k] - a[(w + 4) * 64 + k]) / 4.0;
              dur += mn2 - mx;
            }
            if (k < 55 && (k < 6 || k % 8 == 3 || k > 50))
              printf("  %3d  %8.0f  %8.0f  %8.0f\n", k, spread / nwg, pair / nwg, dur / nwg);
          }
        }
        if (PCST_SOLO_STAMPS == 1 && prec == 3) {
          const int64_t nst = (P + 255) / 256 * 8 * 8;
          std::vector<float> h(nst);
          CK(hipMemcpy(h.data(), out + P * 3, nst * 4, hipMemcpyDeviceToHost));
          double c = 0, dm = 0, b = 0, rt = 0, hd = 0, rs = 0, tl = 0, k = 0;
          for (int64_t i = 0; i + 7 < nst; i += 8)
            if (h[i + 7] == 1.0f) {
              c += h[i]; dm += h[i + 1]; b += h[i + 2]; rt += h[i + 3]; hd += h[i + 4]; rs += h[i + 5]; tl += h[i + 6];
              k += 1;
            }
          if (k > 0)
            printf("  stamps: %.0f waves, %.0f cycles (MFMA-bound at 2 waves per SIMD: 221440), DMA wait %.0f, barrier %.0f "
                   "(%.1f%%), clock %.3f GHz; head %.0f, residual %.0f (%.0f per superpart; MFMA-bound 4096), tail %.0f\n",
                   k, c / k, dm / k, b / k, 100.0 * (b + dm) / c, c / rt * 0.1, hd / k, rs / k, rs / k / 48.0, tl / k);
        }
      }
  }
  return 0;
}
