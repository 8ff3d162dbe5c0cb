#!/bin/bash
# One short gpurun call: a pytest selection (-k expression, or "none"), then
# bench.py with the given arguments, then (optional) rocprofv3 kernel stats
# of the same bench command.
# Usage: gpurun -- 'bash tools/gpu_quick.sh <tag> "<pytest -k expr|none>" "<bench args>" [prof]'
set -eu -o pipefail
TAG=$1; KEXPR=$2; BARGS=$3; PROF=${4:-}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
export TMPDIR=/tmp
if [ "$KEXPR" != none ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$KEXPR" \
      > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
fi
timeout -k 10 300 python -u bench.py $BARGS > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed rc=$?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ -n "$PROF" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python3 "$ROOTDIR/bench.py" $BARGS > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" \
      || { echo "rocprof failed rc=$?"; tail -30 "$OUT/prof_bench.err"; exit 1; }
  find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
  find "$OUT/prof" -name '*kernel_trace.csv' -exec python3 "$ROOTDIR/tools/trace_stats.py" {} \; > "$OUT/kernel_by_launch.csv"
  cut -c1-220 "$OUT/kernel_by_launch.csv" | head -12
fi
echo gpu_quick done
