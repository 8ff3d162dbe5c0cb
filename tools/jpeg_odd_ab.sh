#!/bin/bash
# A/B of JPEG builds on the odd-width bench line (abso/<name>.so), rounds alternating.
set -eu -o pipefail
TAG=$1; VARS=$2; ROUNDS=${3:-2}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOTDIR"
for r in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    ZPX_LIB_PATH=$ROOTDIR/abso/$v.so timeout -k 10 240 python -u bench.py --no-png --no-config5 --no-e2e \
        --no-cpu-baseline --steps 10 > "$OUT/$v.$r.json" 2> "$OUT/$v.$r.err"
    python3 -c "
import json; d=json.loads(open('$OUT/$v.$r.json').read().strip().splitlines()[-1])
print('$v', d['roofline']['kernel_ms_per_launch'], d['odd_width']['kernel_ms_per_launch'])"
  done
done
