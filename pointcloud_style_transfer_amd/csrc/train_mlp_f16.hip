// fp16 build of csrc/train_mlp.hip (the autocast dtype of the reference's CUDA trainer): the same
// kernels on v_mfma_f32_32x32x16_f16 with fp16 operand storage, in namespace pcst::f16m.
#define PCST_H16_F16 1
#include "train_mlp.hip"
