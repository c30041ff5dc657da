// Timing harness for the fused noise-MLP kernel (perf experiments only, not product code).
// Built by tools/nm_variants.sh once per knob setting (PCST_NM_EXPERIMENT / PCST_NM_NCB, see
// csrc/noise_mlp.hip); each binary times the bench workload -- 60000 points (2 x 30000 CFG
// rows), bf16 -- with HIP events and prints one line.  Weights are random: the timing of
// an MFMA kernel does not depend on operand values beyond DVFS effects.
#ifdef NM_SRC
#include NM_SRC
#else
#include "../pointcloud_style_transfer_amd/csrc/noise_mlp.hip"
#endif
#ifndef PCST_NM_QUAD
#define PCST_NM_QUAD 0
#endif
#if PCST_NM_QUAD
#include "nm_quad.hip"
#endif
#ifndef PCST_NM_EXPERIMENT
#define PCST_NM_EXPERIMENT -1
#endif
#ifndef PCST_NM_NCB
#define PCST_NM_NCB -1
#endif

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

static int run(const float* pts, int64_t P, int64_t T, const float* cond, int64_t C, const void* blob,
               int64_t blob_bytes, const float* bias, int prec, float* out, hipStream_t st) {
#if PCST_NM_QUAD
  if (prec == 1) return pcst::launch_quad(pts, P, T, cond, C, blob, blob_bytes, bias, out, st);
#endif
  return pcst_noise_mlp(pts, P, T, cond, C, blob, blob_bytes, bias, prec, out, st);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 50;
  const int prec = argc > 2 ? atoi(argv[2]) : 1;
  const int64_t T = 30000, C = argc > 3 ? atoi(argv[3]) : 2, P = T * C;  // CFG rows of 30000
  const int64_t blob_bytes = pcst_noise_mlp_blob_bytes(prec);
  std::vector<float> h_pts(P * 3), h_cond(C * 256), h_bias(kBiasFloats);
  std::vector<uint16_t> h_blob(blob_bytes / 2);
  uint32_t s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (float)((s >> 8) & 0xffff) / 65536.0f - 0.5f; };
  for (auto& v : h_pts) v = 2.0f * rnd();
  for (auto& v : h_cond) v = 0.1f * rnd();
  for (auto& v : h_bias) v = 0.05f * rnd();
  for (auto& v : h_blob) {
    float f = 0.06f * rnd();
    uint32_t u;
    std::memcpy(&u, &f, 4);
    v = (uint16_t)(u >> 16);
  }
  float *pts, *cond, *bias, *out;
  void* blob;
  CK(hipMalloc(&pts, P * 12));
  CK(hipMalloc(&cond, C * 1024));
  CK(hipMalloc(&bias, kBiasFloats * 4));
  const int64_t stamp_floats = ((P + 255) / 256) * 4 * 8;  // quad diagnostic stamps past the outputs
  CK(hipMalloc(&out, P * 12 + stamp_floats * 4));
  CK(hipMemset(out, 0, P * 12 + stamp_floats * 4));
  CK(hipMalloc(&blob, blob_bytes));
  CK(hipMemcpy(pts, h_pts.data(), P * 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(cond, h_cond.data(), C * 1024, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, h_bias.data(), kBiasFloats * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(blob, h_blob.data(), blob_bytes, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (int i = 0; i < 5; ++i)
    if (run(pts, P, T, cond, C, blob, blob_bytes, bias, prec, out, st)) return 2;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < iters; ++i) run(pts, P, T, cond, C, blob, blob_bytes, bias, prec, out, st);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = 1e3 * ms / iters;
  const double tf = 3540480.0 * P / (us * 1e-6) / 1e12;
  std::vector<float> h_out(P * 3), h_st(stamp_floats);
  CK(hipMemcpy(h_out.data(), out, P * 12, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h_st.data(), out + P * 3, stamp_floats * 4, hipMemcpyDeviceToHost));
  double cs = 0;
  for (float v : h_out) cs += v;
  if (PCST_NM_EXPERIMENT & 16) {  // quad diagnostic: per-wave {cycles, barrier cycles, 100 MHz ticks, 1}
    double c = 0, b = 0, rt = 0, n = 0, pro = 0, res = 0, lend = 0;
    for (int64_t i = 0; i + 7 < stamp_floats; i += 8)
      if (h_st[i + 7] == 1.0f) {
        c += h_st[i]; b += h_st[i + 1]; rt += h_st[i + 2]; pro += h_st[i + 3];
        res += h_st[i + 4]; lend += h_st[i + 5]; n += 1;
      }
    if (n > 0)
      printf("waves %.0f: %.0f cycles, barrier %.0f (%.1f%%), clock %.3f GHz; prologue+dense %.0f, "
             "residual %.0f (layer ends %.0f), output %.0f\n", n, c / n, b / n, 100.0 * b / c,
             c / rt * 0.1, pro / n, res / n, lend / n, (c - pro - res) / n);
  }
  printf("quad=%d experiment=%d ncb=%d prec=%d rows=%lld  %.1f us/launch  %.1f TFLOP/s  (%.1f%% of 2500)  checksum=%.6e\n",
         PCST_NM_QUAD, PCST_NM_EXPERIMENT, PCST_NM_NCB, prec, (long long)C, us, tf, tf / 25.0, cs);
  return 0;
}
