#!/bin/bash
# Generic PNG A/B on the GPU box: alternating rounds of tools/png_probe.py over
# library builds abso/<variant>.so (stream layout).  Usage:
#   bash tools/gpu_ab.sh <tag> <rounds> "<shapes>" <variant> ...
set -eu -o pipefail
TAG=$1; ROUNDS=$2; SHAPES=$3; shift 3
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
export TMPDIR=/tmp ZPX_PROBE_LAYOUT=${ZPX_PROBE_LAYOUT:-stream}
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    echo "== round $r $v" | tee -a "$OUT/ab.log"
    ZPX_LIB_PATH=$ROOTDIR/abso/$v.so timeout -k 10 240 python -u tools/png_probe.py 4096 $SHAPES 2>&1 | grep -v amdgpu.ids | tee -a "$OUT/ab.log"
  done
done
echo ab done
