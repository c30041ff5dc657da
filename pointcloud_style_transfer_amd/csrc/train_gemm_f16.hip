// fp16 build of csrc/train_gemm.hip (namespace pcst::f16m), see train_mlp_f16.hip.
#define PCST_H16_F16 1
#include "train_gemm.hip"
