#!/bin/bash
# VGPRs, spills and scratch of every kernel in a built object (default: the main kernel object), from the gfx950
# code object's metadata notes.  usage: tools/co_resources.sh [build/xxx.o] [name filter regex]
set -eu
obj=${1:-$(dirname "$0")/../lua-multigrid-poisson_amd/csrc/build/mgp_kernels.o}
tmp=$(mktemp -d)
trap 'rm -rf $tmp' EXIT
objcopy -O binary --only-section=.hip_fatbin "$obj" $tmp/fat.bin
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$tmp/fat.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$tmp/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $tmp/k.co |
  grep -E "^ +\.name:|private_segment_fixed_size|\.vgpr_count|vgpr_spill_count" | paste - - - - |
  sed -E 's/ +/ /g;s/_ZN3mgp12_GLOBAL__N_1[0-9]+//' | grep -E "${2:-.}" || true
