// Which XCC / SE / CU a CU-mask bit of hipExtStreamCreateWithCUMask selects (experiments only):
// for a few one-bit masks, 64 one-wave work-groups record HW_ID and XCC_ID; prints the distinct
// (xcc, se, sh, cu) seen per mask bit.
// Measured (round 5, MI355X, 256 CUs): bit b selects one CU of XCC b % 8, shader engine (b / 8) % 4,
// CU slot b / 32 of that engine; an XCC left with no bit set in the mask keeps ALL its CUs.  Within
// an XCC the dispatcher deals work-groups round-robin over the enabled shader engines regardless
// of free capacity, so a 235-work-group kernel (7-8 per engine) cannot give up even one CU per
// engine without a second round: the CU-masked step / kNN-build split was measured slower
// (MLP 0.157 -> 0.273 ms) and is not in the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void who(unsigned* out) {
  if (threadIdx.x == 0) {
    out[blockIdx.x * 2 + 0] = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID
    out[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_getreg(20 | (31 << 11));   // HW_REG_XCC_ID
  }
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount;
  printf("CUs %d\n", ncu);
  unsigned* d;
  hipMalloc(&d, 4096 * 8);
  std::vector<int> bits = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 15, 16, 31, 32, 33, 63, 64, 128, 240, 247, 248, 255};
  for (int b : bits) {
    if (b >= ncu) continue;
    unsigned mask[32] = {};
    mask[b / 32] = 1u << (b % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (ncu + 31) / 32 * 32, mask) != hipSuccess) { printf("mask %d failed\n", b); continue; }
    hipLaunchKernelGGL(who, dim3(64), dim3(64), 0, s, d);
    hipStreamSynchronize(s);
    std::vector<unsigned> h(128);
    hipMemcpy(h.data(), d, 128 * 4, hipMemcpyDeviceToHost);
    std::set<std::tuple<int, int, int, int>> seen;
    for (int i = 0; i < 64; ++i) {
      const unsigned hw = h[2 * i], xcc = h[2 * i + 1] & 0xf;
      seen.insert({(int)xcc, (int)((hw >> 13) & 7), (int)((hw >> 12) & 1), (int)((hw >> 8) & 15)});
    }
    printf("bit %3d ->", b);
    for (auto& t : seen) printf(" (xcc %d se %d sh %d cu %d)", std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t));
    printf("\n");
    hipStreamDestroy(s);
  }
  // the full device, no mask: distinct (xcc, se, sh, cu) over 4096 work-groups
  hipLaunchKernelGGL(who, dim3(4096), dim3(64), 0, 0, d);
  hipDeviceSynchronize();
  std::vector<unsigned> h(8192);
  hipMemcpy(h.data(), d, 8192 * 4, hipMemcpyDeviceToHost);
  std::set<std::tuple<int, int, int, int>> all;
  for (int i = 0; i < 4096; ++i)
    all.insert({(int)(h[2 * i + 1] & 0xf), (int)((h[2 * i] >> 13) & 7), (int)((h[2 * i] >> 12) & 1), (int)((h[2 * i] >> 8) & 15)});
  std::set<int> se_per_xcc[16], cu_vals;
  for (auto& t : all) { se_per_xcc[std::get<0>(t)].insert(std::get<1>(t) * 2 + std::get<2>(t)); cu_vals.insert(std::get<3>(t)); }
  printf("unmasked: %zu distinct (xcc,se,sh,cu); xcc0 se/sh:", all.size());
  for (int v : se_per_xcc[0]) printf(" %d", v);
  printf("; cu ids:");
  for (int v : cu_vals) printf(" %d", v);
  printf("\n");
  return 0;
}
