#!/bin/bash
# VGPR / scratch / spill counts of the kernels in a built object of libafm.so (the code object
# metadata), e.g. tools/kernel_resources.sh factors PartT
set -e
R=$(cd $(dirname $0)/.. && pwd)
obj=$R/alpha-multi-factor-models_amd/build/$1.hip.o
T=$(mktemp -d)
B=/opt/rocm/lib/llvm/bin
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin $obj
$B/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$T/fat.bin \
    --output=$T/dev.o --unbundle
$B/llvm-readelf --notes $T/dev.o | grep -E "^ +\.name:|\.vgpr_count:|\.private_segment_fixed_size:|\.vgpr_spill_count:" |
    paste - - - - | sed 's/  */ /g' | grep -E "${2:-.}"
rm -rf $T
