#!/bin/bash
# A/B of library builds on the GPU box: each abso/<name>.so runs bench.py
# with the given arguments, rounds alternating; prints the kernel ms of every
# line (tools/bench_lines.py).  Timing-only variants: ZPX_BENCH_TIMING_ONLY=1
# skips the headline's parity gate.
# Usage: bash tools/ab.sh <tag> "<variants>" "<bench args>" [rounds]
set -eu -o pipefail
TAG=$1; VARS=$2; BARGS=$3; ROUNDS=${4:-2}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
for r in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    ZPX_LIB_PATH=$ROOTDIR/abso/$v.so timeout -k 10 300 python -u bench.py $BARGS > "$OUT/$v.$r.json" 2> "$OUT/$v.$r.err" \
        || { echo "$v failed"; tail -5 "$OUT/$v.$r.err"; exit 1; }
    echo "$v $(python3 tools/bench_lines.py "$OUT/$v.$r.json")"
  done
done
