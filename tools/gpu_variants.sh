#!/bin/bash
# Bench each zpix_amd/variants/*.so (JPEG only, no CPU leg) in one GPU call.
# Usage: gpurun -- 'bash tools/gpu_variants.sh <tag> [bench args]'
set -eu -o pipefail
TAG=${1:-var}; shift || true
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
for so in zpix_amd/variants/*.so; do
  n=$(basename "$so" .so)
  TONLY=""; case $n in *copy*) TONLY=1;; esac
  ZPX_BENCH_TIMING_ONLY=$TONLY ZPX_LIB_PATH=$ROOTDIR/$so timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" \
      || { echo "bench $n failed rc=$?"; tail -20 "$OUT/$n.err"; exit 1; }
  python3 -c "import json,sys; r=json.load(open(sys.argv[1])); p=r.get('png',{}); print(sys.argv[2], 'JPEG', r.get('value'), r.get('roofline',{}).get('frac'), r.get('roofline',{}).get('kernel_ms_per_launch'), 'PNG', p.get('value'), p.get('roofline',{}).get('kernel_ms_per_launch'))" "$OUT/$n.json" "$n"
done
