// Microbenchmark: what a cross-stream dependency costs on the queue that carries it.
//   hipcc --offload-arch=gfx950 -O2 tools/sync_probe.hip -o tools/_scratch/sync_probe && ./sync_probe
// A chain of K dependent ~5 us kernels on stream A, with one of these between kernel K/2 and the
// next, repeated; prints the mean time per chain:
//   none       nothing (the baseline)
//   rec        hipEventRecord (hipEventDisableTiming | hipEventDisableSystemFence) on A
//   rec+wait   the same event waited on by stream B (which runs one tiny kernel after it)
//   waitB      A waits (hipStreamWaitEvent) on an event B recorded long before (already done)
//   wval       A waits on hipStreamWaitValue32 for a value a kernel on B wrote long before
//   wrval      hipStreamWriteValue32 on A
// A development tool (tools/ only).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void spin_kernel(float* buf, int iters) {
  float v = buf[threadIdx.x];
  for (int i = 0; i < iters; ++i) v = v * 1.0000001f + 0.5f;
  buf[blockIdx.x * 256 + threadIdx.x] = v;
}

__global__ void flag_kernel(unsigned* flag, unsigned v) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one lane polls the flag (agent scope, with s_sleep) until it reaches v or a bounded number of
// polls elapsed (then it gives up: the probe's hang guard)
__global__ void spin_wait_kernel(const unsigned* flag, unsigned v) {
  if (threadIdx.x == 0) {
    for (int i = 0; i < (1 << 24); ++i) {
      if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= v) break;
      __builtin_amdgcn_s_sleep(2);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
}

int main() {
  float* buf;
  CK(hipMalloc(&buf, 256 * 256 * sizeof(float)));
  CK(hipMemset(buf, 0, 256 * 256 * sizeof(float)));
  unsigned* sig = nullptr;
  unsigned* wv = nullptr;
  CK(hipExtMallocWithFlags((void**)&sig, 8, hipMallocSignalMemory));
  CK(hipMemset(sig, 0, 8));
  CK(hipMalloc(&wv, 64));
  CK(hipMemset(wv, 0, 64));
  hipStream_t A, B;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  hipEvent_t ev, evB;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventDisableSystemFence));
  CK(hipEventCreateWithFlags(&evB, hipEventDisableTiming | hipEventDisableSystemFence));
  const int K = 16, reps = 200, iters = 2000;
  const char* names[] = {"none", "rec", "rec+wait", "waitB", "wval", "wrval", "flag+wvalB",
                         "wrval+wvalB", "rec+waitonly", "Bkernel", "flag+wvalB+k", "flag+spinB",
                         "flag+spinB+k"};
  unsigned counter = 0;
  for (int mode = 0; mode < 13; ++mode) {
    for (int pass = 0; pass < 2; ++pass) {
      CK(hipDeviceSynchronize());
      auto t0 = std::chrono::high_resolution_clock::now();
      for (int r = 0; r < reps; ++r) {
        if (mode == 3) {  // B records an event long before A needs it
          CK(hipEventRecord(evB, B));
        }
        if (mode == 4) {
          ++counter;  // B's kernel writes the value long before A waits on it
          hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, B, sig, counter);
        }
        for (int k = 0; k < K; ++k) {
          hipLaunchKernelGGL(spin_kernel, dim3(256), dim3(256), 0, A, buf, iters);
          if (k == K / 2) {
            if (mode == 1 || mode == 2) CK(hipEventRecord(ev, A));
            if (mode == 2) {
              CK(hipStreamWaitEvent(B, ev, 0));
              hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(256), 0, B, buf, 10);
            }
            if (mode == 3) CK(hipStreamWaitEvent(A, evB, 0));
            if (mode == 4) CK(hipStreamWaitValue32(A, sig, counter, hipStreamWaitValueGte, 0xffffffffu));
            if (mode == 5) CK(hipStreamWriteValue32(A, wv, r, 0));
            if (mode == 6 || mode == 10) {  // a kernel on A writes the flag; B waits on its value
              ++counter;
              hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, A, sig, counter);
              CK(hipStreamWaitValue32(B, sig, counter, hipStreamWaitValueGte, 0xffffffffu));
              if (mode == 10) hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(256), 0, B, buf, 10);
            }
            if (mode == 7) {  // hipStreamWriteValue32 on A, B waits on it
              ++counter;
              CK(hipStreamWriteValue32(A, sig, counter, 0));
              CK(hipStreamWaitValue32(B, sig, counter, hipStreamWaitValueGte, 0xffffffffu));
              hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(256), 0, B, buf, 10);
            }
            if (mode == 8) {
              CK(hipEventRecord(ev, A));
              CK(hipStreamWaitEvent(B, ev, 0));
            }
            if (mode == 11 || mode == 12) {  // a kernel on A writes the flag; a kernel on B spins
              ++counter;
              hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, A, wv, counter);
              hipLaunchKernelGGL(spin_wait_kernel, dim3(1), dim3(64), 0, B, wv, counter);
              if (mode == 12) hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(256), 0, B, buf, 10);
            }
            if (mode == 9) hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(256), 0, B, buf, 10);
          }
        }
      }
      CK(hipDeviceSynchronize());
      auto t1 = std::chrono::high_resolution_clock::now();
      const double us = std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
      if (pass == 1) printf("%-9s %8.2f us per chain of %d kernels\n", names[mode], us, K);
    }
  }
  return 0;
}
