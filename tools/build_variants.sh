#!/bin/bash
# Build library variants with extra -D flags into var/<name>/libmgpoisson.so (shipped to the GPU
# box with the tree, git-ignored).  usage: tools/build_variants.sh name1 "-DFOO=1" name2 "-DBAR=2" ...
set -eu
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p var/$name
  make -s -C lua-multigrid-poisson_amd/csrc BUILD=../../var/$name/build OUT=../../var/$name/libmgpoisson.so EXTRA="$flags" &
done
wait
ls -la var/*/libmgpoisson.so
