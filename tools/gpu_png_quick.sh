#!/bin/bash
# PNG iteration: PNG + batch gpu parity tests, then the PNG bench lines.
# Usage: gpurun --timeout 600 -- 'bash tools/gpu_png_quick.sh <tag> [bench args...]'
set -eu -o pipefail
TAG=${1:-pngq}; shift || true
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
timeout -k 10 300 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_batch.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 240 python -u bench.py --png-only --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed rc=$?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
