#!/bin/bash
# PNG bench at several persistent-grid sizes (ZPX_PNG_WAVES_PER_CU).
# Usage: gpurun -- 'bash tools/gpu_png_occ.sh <tag> [waves ...]'
set -eu -o pipefail
TAG=${1:-occ}; shift || true
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
for w in "${@:-8 16}"; do
  for so in zpix_amd/libzpix_amd.so zpix_amd/variants/*.so; do
    [ -e "$so" ] || continue
    n=$(basename "$so" .so)_w$w
    ZPX_PNG_WAVES_PER_CU=$w ZPX_LIB_PATH=$ROOTDIR/$so timeout -k 10 200 python -u bench.py --png-only --no-cpu-baseline \
        > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "bench $n failed rc=$?"; tail -20 "$OUT/$n.err"; exit 1; }
    python3 -c "import json,sys; r=json.load(open(sys.argv[1])); p=r.get('png',r); print(sys.argv[2], 'PNG', p.get('value'), p.get('roofline',{}).get('frac'), p.get('roofline',{}).get('kernel_ms_per_launch'))" "$OUT/$n.json" "$n"
  done
done
echo done
