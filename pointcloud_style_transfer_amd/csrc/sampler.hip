// Fused classifier-free-guidance + DDIM update of DiffusionProcess.guided_sample_loop
// (models/diffusion_model.py:248-260) and of ddim_sample_loop (:283-290).
//   eps = eps_u + s*(eps_c - eps_u)                          (CFG only)
//   x0  = (x - sqrt(1-a_t)*eps) / (sqrt(a_t) + 1e-8)
//   x0  = x0 + 0.1*(source - x0)                             (guided only)
//   x0  = tanh(x0/1.8)*1.8
//   x'  = sqrt(a_prev)*x0 + sqrt(1-a_prev)*eps
// The four per-step scalars are computed on the host in fp32 exactly as the reference's 0-d
// tensor ops do.  The new x is also written into both halves of the next step's CFG batch
// (torch.cat([x]*2), :240), so no separate concatenation pass exists.
#include "common.h"

namespace pcst {

__global__ void cfg_ddim_kernel(const float* __restrict__ x, const float* __restrict__ eps_c,
                                const float* __restrict__ eps_u, const float* __restrict__ src,
                                int64_t n, float scale, float c1, float c2, float c3, float c4,
                                const float* __restrict__ coef, float* __restrict__ x_out,
                                float* __restrict__ x_cat) {
  if (coef) {  // device coefficients: hipGraph-replayable
    c1 = coef[0];
    c2 = coef[1];
    c3 = coef[2];
    c4 = coef[3];
  }
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const float xn = cfg_ddim_value(x[e], eps_c[e], eps_u ? eps_u + e : nullptr,
                                    src ? src + e : nullptr, scale, c1, c2, c3, c4);
    x_out[e] = xn;
    if (x_cat) {
      x_cat[e] = xn;
      x_cat[n + e] = xn;
    }
  }
}

}  // namespace pcst

using namespace pcst;

extern "C" int pcst_cfg_ddim_step(const float* x, const float* eps_c, const float* eps_u,
                                  const float* source, int64_t n, float guidance_scale,
                                  float sqrt_1m_at, float sqrt_at_eps, float sqrt_aprev,
                                  float sqrt_1m_aprev, float* x_out, float* x_cat, void* stream) {
  PCST_CHECK_ARG(n >= 0, "cfg_ddim_step: bad size");
  if (n == 0) return PCST_OK;
  PCST_CHECK_ARG(x && eps_c && x_out, "cfg_ddim_step: null pointer");
  const int64_t g = std::min<int64_t>(cdiv(n, 256), 4096);
  hipLaunchKernelGGL(cfg_ddim_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), x, eps_c,
                     eps_u, source, n, guidance_scale, sqrt_1m_at, sqrt_at_eps, sqrt_aprev,
                     sqrt_1m_aprev, (const float*)nullptr, x_out, x_cat);
  PCST_LAUNCH_CHECK("cfg_ddim_step");
  return PCST_OK;
}

extern "C" int pcst_cfg_ddim_step_dcoef(const float* x, const float* eps_c, const float* eps_u,
                                        const float* source, int64_t n, float guidance_scale,
                                        const float* coef_dev, float* x_out, float* x_cat,
                                        void* stream) {
  PCST_CHECK_ARG(n >= 0, "cfg_ddim_step_dcoef: bad size");
  if (n == 0) return PCST_OK;
  PCST_CHECK_ARG(x && eps_c && x_out && coef_dev, "cfg_ddim_step_dcoef: null pointer");
  const int64_t g = std::min<int64_t>(cdiv(n, 256), 4096);
  hipLaunchKernelGGL(cfg_ddim_kernel, dim3((unsigned)g), dim3(256), 0, as_stream(stream), x, eps_c,
                     eps_u, source, n, guidance_scale, 0.f, 1.f, 0.f, 0.f, coef_dev, x_out, x_cat);
  PCST_LAUNCH_CHECK("cfg_ddim_step_dcoef");
  return PCST_OK;
}

// ---- kernel-side stream signal (pcst.h: pcst_signal_write / pcst_signal_wait) -------------
namespace pcst {
// one lane: the stream's earlier kernels have completed and released at their end; the fence
// makes this kernel's view current before the flag (vector store, agent scope) is published
__global__ void signal_write_kernel(uint32_t* flag, uint32_t value) {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// one lane polls (agent-scope loads, L2-served, with s_sleep between polls) until the flag
// reaches `value`, at most max_polls times (default kSignalPolls, ~10 s); then an agent-scope
// acquire.  A wait that gives up sets *err: the caller must read it (the stream goes on).
__global__ void signal_wait_kernel(const uint32_t* flag, uint32_t value, int32_t* err,
                                   int64_t max_polls) {
  if (threadIdx.x == 0) {
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
}  // namespace pcst

extern "C" int pcst_signal_write(uint32_t* flag, uint32_t value, void* stream) {
  PCST_CHECK_ARG(flag != nullptr, "signal_write: null flag");
  hipLaunchKernelGGL(pcst::signal_write_kernel, dim3(1), dim3(64), 0, pcst::as_stream(stream), flag,
                     value);
  PCST_LAUNCH_CHECK("signal_write");
  return PCST_OK;
}

extern "C" int pcst_signal_wait(const uint32_t* flag, uint32_t value, int32_t* err, int64_t max_polls,
                                void* stream) {
  PCST_CHECK_ARG(flag != nullptr, "signal_wait: null flag");
  hipLaunchKernelGGL(pcst::signal_wait_kernel, dim3(1), dim3(64), 0, pcst::as_stream(stream), flag,
                     value, err, max_polls > 0 ? max_polls : (int64_t)pcst::kSignalPolls);
  PCST_LAUNCH_CHECK("signal_wait");
  return PCST_OK;
}
