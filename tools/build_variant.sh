#!/bin/bash
# Builds libzpix_amd.so with extra -D flags into abso/<name>.so (kernel A/B
# experiments; the shipped library is zpix_amd/libzpix_amd.so).
# Usage: bash tools/build_variant.sh <name> "<-DFLAG=V ...>"
set -eu -o pipefail
NAME=$1; DEFS=${2:-}
ROOTDIR=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOTDIR/abso"
make -s -j8 -C "$ROOTDIR/zpix_amd/csrc" OUT="$ROOTDIR/abso/$NAME.so" OBJDIR="$ROOTDIR/build/var_$NAME" \
    CXXFLAGS="-O3 -std=c++17 -fPIC -fwrapv -Wall -Wextra -Wno-unused-parameter -I../../include $DEFS"
