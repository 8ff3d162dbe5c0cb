#!/bin/bash
# Quick GPU iteration: JPEG+PNG gpu parity tests, then bench without the CPU leg.
# Usage: gpurun --timeout 600 -- 'bash tools/gpu_quick.sh <tag> [bench args...]'
set -eu -o pipefail
TAG=${1:-quick}; shift || true
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest -m gpu failed rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 240 python -u bench.py --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed rc=$?"; tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print('JPEG', r.get('value'), r.get('roofline',{}).get('frac'), r.get('roofline',{}).get('kernel_ms_per_launch')); p=r.get('png',{}); print('PNG', p.get('value'), p.get('roofline',{}).get('frac'), p.get('roofline',{}).get('kernel_ms_per_launch'))" "$OUT/bench.json"
