#!/bin/bash
# Build A/B variants of libzpix_amd.so into build/variants/<name>.so.
# Usage: tools/build_variants.sh name1 "-DFLAG=1 ..." name2 "..."
set -eu
ROOTDIR=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOTDIR/zpix_amd/variants"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  make -s -j8 -C "$ROOTDIR/zpix_amd/csrc" OBJDIR="$ROOTDIR/build/obj_$name" OUT="$ROOTDIR/zpix_amd/variants/$name.so" \
      CXXFLAGS="-O3 -std=c++17 -fPIC -fwrapv -Wall -Wextra -Wno-unused-parameter -I$ROOTDIR/include $flags" 2>&1 | grep -v hip-link || true
done
