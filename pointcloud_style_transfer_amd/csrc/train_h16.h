// The 16-bit-operand training GEMMs (train_mlp.hip, train_gemm.hip) are compiled twice: as
// themselves for bf16 (namespace pcst::bf16m) and through train_*_f16.hip for fp16
// (pcst::f16m).  The C entry points, defined in the bf16 build, dispatch on their `f16` argument.
#pragma once
#include <stddef.h>
#include <stdint.h>

#if defined(PCST_H16_F16) && PCST_H16_F16
#define PCST_H16_NS f16m
#else
#define PCST_H16_NS bf16m
#endif

namespace pcst {
constexpr int kCastMax = 64;  // tensors per pcst_cast16_batch call
#define PCST_H16_DECLS                                                                              \
  int gemm_ex_impl(const void* A, int a_bf16, int64_t M, int64_t K, const void* B, int b_bf16,     \
                   int64_t O, const float* bias, int relu, int epilogue, const void* aux,          \
                   uint64_t seed, float drop_p, int64_t group_rows, void* C, uint16_t* C2,         \
                   void* stream);                                                                  \
  int dropout_grad_impl(const float* g, int64_t n, uint64_t seed, float drop_p, uint16_t* out,     \
                        void* stream);                                                             \
  int resblock_fwd_impl(const uint16_t* x, int64_t M, const uint16_t* w1, const float* b1,         \
                        const uint16_t* w2, const float* b2, uint64_t seed, float drop_p,          \
                        uint16_t* h, uint16_t* xo, uint32_t* hbits, void* stream);                 \
  int cast16_batch_impl(const float* const* src, uint16_t* const* dst, const int32_t* rows,         \
                        const int32_t* cols, const int32_t* trans, int n, void* stream);           \
  int resblock_bwd_impl(const uint16_t* dd, int64_t M, const uint16_t* w2t, const uint16_t* w1t,   \
                        const uint16_t* h, const uint16_t* g, uint64_t seed, float drop_p,         \
                        uint16_t* dz, uint16_t* g_out, uint16_t* dd_out, const uint32_t* hbits,    \
                        void* stream);                                                             \
  int wgrad_ex_workspace_impl(int64_t M, int64_t I, int64_t O, size_t* bytes);                     \
  int wgrad_ex_impl(const void* dZ, int dz_bf16, const void* X, int x_bf16, int64_t M, int64_t I, \
                    int64_t O, float* dW, float* db, void* workspace, void* stream);               \
  int gemm_nt_impl(const float* A, int64_t M, int64_t K, const float* B, int64_t O,               \
                   const float* scale, const float* shift, int relu, float* C, void* stream);      \
  int wgrad16_workspace_impl(int64_t M, int64_t I, int64_t O, size_t* bytes);                      \
  int wgrad16_impl(const float* dZ, const float* X, int64_t M, int64_t I, int64_t O, float* dW,    \
                   float* db, void* workspace, void* stream);
namespace bf16m {
PCST_H16_DECLS
}
namespace f16m {
PCST_H16_DECLS
}
#undef PCST_H16_DECLS
}  // namespace pcst
