#!/bin/bash
# Resource usage (VGPR/SGPR/LDS/spills) of the kernels in one built object: tools/kres.sh build/knn.o
set -e
O=$(realpath "$1"); T=$(mktemp -d)
cd "$T"
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=fat.bin "$O"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=fat.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=dev.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes dev.co | grep -E "^ +\.name:|\.vgpr_count|\.sgpr_count|group_segment_fixed|spill_count|agpr_count" \
  | paste - - - - - - - | sed 's/  */ /g' | awk '{print}'
rm -rf "$T"
