// Timing harness for the bf16 noise-MLP kernel (perf experiments only, not product code): times
// the bench launch (2 x 30000 points) and the 32-cloud launch (64 x 30000) of precision 1 (the
// solo kernel) with HIP events on random bf16 weights.  Build: hipcc -O3 --offload-arch=gfx950
// -mno-amdgpu-ieee -fno-honor-nans -I include -I pointcloud_style_transfer_amd/csrc
// tools/solo_bench.hip -o tools/solo_bench; run: tools/solo_bench [iters] [clouds]
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
  CK(hipMalloc(&out, Pmax * 12));
  CK(hipMemcpy(pts, h_pts.data(), Pmax * 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(cond, h_cond.data(), Cmax * 1024, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, h_bias.data(), kBiasFloats * 4, hipMemcpyHostToDevice));
  const int prec = 1;
  const int64_t bb = pcst_noise_mlp_blob_bytes(prec);
  void* blob = nullptr;
  {
    std::vector<uint16_t> h(bb / 2);
    for (auto& v : h) {
      float f = 0.06f * rnd(s);
      uint32_t u;
      std::memcpy(&u, &f, 4);
      v = (uint16_t)(u >> 16);
    }
    CK(hipMalloc(&blob, bb));
    CK(hipMemcpy(blob, h.data(), bb, hipMemcpyHostToDevice));
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int only_c = argc > 2 ? atoi(argv[2]) : 0;  // clouds (2 or 64; default both)
  for (int64_t C : {2, 64}) {
    if (only_c && C != only_c) continue;
    const int64_t P = T * C;
    const int n = C == 2 ? iters : iters / 8 + 2;
    for (int rep = 0; rep < 2; ++rep) {
      for (int i = 0; i < 3; ++i)
        if (pcst_noise_mlp(pts, P, T, cond, C, blob, bb, bias, prec, out, st)) return 2;
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < n; ++i) pcst_noise_mlp(pts, P, T, cond, C, blob, bb, bias, prec, out, st);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1e3 * ms / n;
      const double tf = 3540480.0 * P / (us * 1e-6) / 1e12;
      printf("clouds=%lld  %.1f us/launch  %.1f TFLOP/s  frac %.4f\n", (long long)C, us, tf, tf / 2500.0);
    }
  }
  return 0;
}
