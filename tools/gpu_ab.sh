#!/bin/bash
# A/B kernel runs in one GPU call: the gpu parity suite on the main build, then
# bench.py for each "name|lib|ENV=VAL ..." spec (lib relative to the repo root).
# Usage: gpurun -- 'bash tools/gpu_ab.sh <tag> "<bench args>" "a|zpix_amd/libzpix_amd.so|" "b|zpix_amd/libzpix_amd.so|X=1"'
set -eu -o pipefail
TAG=$1; BARGS=$2; shift 2
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest -m gpu failed rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for spec in "$@"; do
  IFS='|' read -r n lib envs <<< "$spec"
  env $envs ZPX_LIB_PATH=$ROOTDIR/$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline $BARGS > "$OUT/$n.json" 2> "$OUT/$n.err" \
      || { echo "bench $n failed rc=$?"; tail -20 "$OUT/$n.err"; exit 1; }
  python3 -c "
import json,sys; r=json.load(open(sys.argv[1])); p=r.get('png',{})
print(sys.argv[2], 'JPEG', r.get('value'), r.get('roofline',{}).get('frac'), r.get('roofline',{}).get('kernel_ms_per_launch'), 'PNG', p.get('value'), p.get('roofline',{}).get('kernel_ms_per_launch'))" "$OUT/$n.json" "$n"
done
echo done
