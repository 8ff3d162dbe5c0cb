#!/bin/bash
# A/B bench runs without the parity suite (variants already parity-tested or
# timing-only): bench.py per "name|lib|ENV=VAL ..." spec; prints the JPEG,
# int16, progressive 4:4:4, PNG and Adam7 kernel times.
# Usage: gpurun -- 'bash tools/gpu_ab_bench.sh <tag> "<bench args>" "a|zpix_amd/libzpix_amd.so|" ...'
set -eu -o pipefail
TAG=$1; BARGS=$2; shift 2
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
for spec in "$@"; do
  IFS='|' read -r n lib envs <<< "$spec"
  env $envs ZPX_LIB_PATH=$ROOTDIR/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline $BARGS > "$OUT/$n.json" 2> "$OUT/$n.err" \
      || { echo "bench $n failed rc=$?"; tail -20 "$OUT/$n.err"; exit 1; }
  python3 -c "
import json,sys; r=json.load(open(sys.argv[1])); c=r.get('config5',{})
g=lambda d,*k: (lambda x: x)(__import__('functools').reduce(lambda a,b: (a or {}).get(b), k, d))
print(sys.argv[2], 'jpeg', g(r,'roofline','kernel_ms_per_launch'), 'int16', g(r,'int16_transport','kernel_ms_per_launch'),
      'prog444', g(c,'jpeg_progressive_444','kernel_ms_per_launch'), 'png', g(r,'png','roofline','kernel_ms_per_launch'),
      'adam7', g(c,'png_adam7_rgba16','kernel_ms_per_launch'))" "$OUT/$n.json" "$n"
done
echo done
