#!/bin/bash
# A/B of PNG kernel builds on the GPU box: each build (a libzpix_amd.so
# variant under abso/<name>.so) times the named probe shapes, rounds
# alternating.  Usage: bash tools/png_ab.sh <tag> "<variants>" "<shapes>" [rounds]
set -eu -o pipefail
TAG=$1; VARS=$2; SHAPES=$3; ROUNDS=${4:-2}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
for r in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    echo "== round $r variant $v" | tee -a "$OUT/ab.log"
    ZPX_LIB_PATH=$ROOTDIR/abso/$v.so timeout -k 10 240 python -u tools/png_probe.py 4096 $SHAPES 2>&1 | tee -a "$OUT/ab.log"
  done
done
