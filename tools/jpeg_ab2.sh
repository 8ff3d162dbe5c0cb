#!/bin/bash
# A/B of JPEG kernel builds (abso/<name>.so, tools/build_variant.sh): every
# JPEG line of bench.py -- headline, int16, planar int8 / int16, pieces rgba /
# planes, 4:1:1 and 4094-wide -- per build, rounds alternating; prints the
# kernel ms per launch of each line.  Usage: bash tools/jpeg_ab2.sh <tag> "<variants>" [rounds]
set -eu -o pipefail
TAG=$1; VARS=$2; ROUNDS=${3:-2}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
for r in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    C5ARGS="--no-config5"; [ "${C5:-0}" = 1 ] && C5ARGS="--no-adam7"
    ZPX_BENCH_TIMING_ONLY=${TIMING_ONLY:-0} ZPX_LIB_PATH=$ROOTDIR/abso/$v.so timeout -k 10 300 python -u bench.py --no-png $C5ARGS \
        --no-e2e --no-cpu-baseline --steps 10 > "$OUT/$v.$r.json" 2> "$OUT/$v.$r.err"
    python3 -c "
import json; d=json.loads(open('$OUT/$v.$r.json').read().strip().splitlines()[-1])
g=lambda *k: (lambda x: x)(__import__('functools').reduce(lambda a,b: (a or {}).get(b), k, d))
c5 = g('config5', 'jpeg_progressive_444', 'kernel_ms_per_launch')
print('$v', 'head', d['roofline']['kernel_ms_per_launch'], 'i16', d['int16_transport']['kernel_ms_per_launch'],
      'pl8', g('planar','int8','kernel_ms_per_launch'), 'pl16', g('planar','int16','kernel_ms_per_launch'),
      'pz.rgba', g('pieces','rgba','kernel_ms_per_launch'), 'pz.planes', g('pieces','planes','kernel_ms_per_launch'),
      '411', g('odd_width','ratio411','kernel_ms_per_launch'), 'odd', g('odd_width','kernel_ms_per_launch'), 'c5', c5, flush=True)"
  done
done
