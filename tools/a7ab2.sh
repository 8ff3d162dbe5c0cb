#!/bin/bash
# Adam7 RGBA16 (64 x 4K, from the stream) per library build, rounds
# alternating, rocprof per launch: bash tools/a7ab2.sh <tag> "<variants>" [rounds]
set -eu -o pipefail
TAG=$1; VARS=$2; ROUNDS=${3:-2}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp; export TMPDIR=/tmp
for r in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    ZPX_PROBE_LAYOUT=stream ZPX_LIB_PATH=$ROOTDIR/abso/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
        -d "$OUT/$v.$r" -o run -- python3 "$ROOTDIR/tools/png_probe.py" 4096 rgba16_adam7 > "$OUT/$v.$r.log" 2>&1
    echo "$v $r $(grep ms/launch "$OUT/$v.$r.log")"
    python3 "$ROOTDIR/tools/trace_stats.py" "$OUT/$v.$r/run_kernel_trace.csv" | grep pair_kernel | cut -c1-110
  done
done
