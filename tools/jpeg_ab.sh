#!/bin/bash
# A/B of JPEG kernel builds on the GPU box (timing-only variants allowed:
# the bench's parity check is skipped with ZPX_BENCH_TIMING_ONLY=1): each build
# under abso/<name>.so runs the JPEG lines of bench.py, rounds alternating.
# Usage: bash tools/jpeg_ab.sh <tag> "<variants>" [rounds]
# (C5=1: also the configs[4] progressive 4:4:4 JPEG line)
set -eu -o pipefail
TAG=$1; VARS=$2; ROUNDS=${3:-2}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
for r in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    C5ARGS="--no-config5"; [ "${C5:-0}" = 1 ] && C5ARGS="--no-adam7"
    ZPX_BENCH_TIMING_ONLY=1 ZPX_LIB_PATH=$ROOTDIR/abso/$v.so timeout -k 10 300 python -u bench.py --no-png $C5ARGS \
        --no-strip --no-e2e --no-cpu-baseline --steps 10 > "$OUT/$v.$r.json" 2> "$OUT/$v.$r.err"
    python3 -c "
import json; d=json.loads(open('$OUT/$v.$r.json').read().strip().splitlines()[-1])
c5 = d.get('config5', {}).get('jpeg_progressive_444', {}).get('kernel_ms_per_launch')
print('$v', d['roofline']['kernel_ms_per_launch'], d['int16_transport']['kernel_ms_per_launch'], c5)"
  done
done
