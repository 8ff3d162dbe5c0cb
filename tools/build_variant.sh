#!/bin/bash
# Builds libzpix_amd.so with extra compile definitions into zpix_amd/variants/<name>.so
# (kernel A/B experiments; run with ZPX_LIB_PATH=zpix_amd/variants/<name>.so).
# Usage: bash tools/build_variant.sh <name> "-DFOO=1 -DBAR=2"
set -eu
NAME=$1; DEFS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/zpix_amd/variants"
make -s -j8 -C "$ROOT/zpix_amd/csrc" OUT="$ROOT/zpix_amd/variants/$NAME.so" OBJDIR="$ROOT/build/obj_$NAME" \
    CXXFLAGS="-O3 -std=c++17 -fPIC -fwrapv -Wall -Wextra -Wno-unused-parameter -I$ROOT/include $DEFS"
