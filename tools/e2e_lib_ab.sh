#!/bin/bash
# End-to-end batch (configs[3], tools/e2e_ab.py) with library builds
# alternating: abso/<name>.so per variant, one batch each per round.
# Usage: bash tools/e2e_lib_ab.sh <tag> "<variants>" [rounds] [threads]
set -eu -o pipefail
TAG=$1; VARS=$2; ROUNDS=${3:-3}; TH=${4:-16}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    echo "== $v round $r" >> "$OUT/ab.txt"
    ZPX_LIB_PATH=$ROOTDIR/abso/$v.so timeout -k 10 200 python -u tools/e2e_ab.py 2 $TH batch_makespan 1 1 2>&1 \
        | grep -v amdgpu.ids >> "$OUT/ab.txt"
  done
done
cat "$OUT/ab.txt"
