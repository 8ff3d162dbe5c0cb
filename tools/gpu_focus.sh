#!/bin/bash
# One short gpurun call: a pytest -k selection, then (optional) the same
# selection under rocprofv3 --kernel-trace --stats (kernel names and times of
# what it ran, e.g. RCCL's kernels).
# Usage: gpurun -- 'bash tools/gpu_focus.sh <tag> "<pytest -k expr>" [prof]'
set -eu -o pipefail
TAG=$1; KEXPR=$2; PROF=${3:-}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$KEXPR" \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
if [ -n "$PROF" ]; then
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python3 -m pytest "$ROOTDIR/tests" -m gpu -x -q --timeout 120 --timeout-method thread -k "$KEXPR" \
      > "$OUT/prof_pytest.log" 2>&1 || { echo "rocprof failed rc=$?"; tail -30 "$OUT/prof_pytest.log"; exit 1; }
  find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
  cut -c1-160 "$OUT/kernel_stats.csv" | head -30
fi
echo gpu_focus done
