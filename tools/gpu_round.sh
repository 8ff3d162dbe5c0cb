#!/bin/bash
# One gpurun call: GPU parity suite, smoke, bench, rocprofv3 kernel stats.
# Usage (from this container):
#   gpurun --timeout 1100 -- 'bash tools/gpu_round.sh <tag> [tests|notests]'
# Every GPU step has its own time limit; the first failure ends the script.
set -eu -o pipefail
TAG=${1:-run}
MODE=${2:-tests}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
export TMPDIR=/tmp
if [ "$MODE" = tests ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest -m gpu failed rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
  timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1 \
      || { echo "smoke failed rc=$?"; tail -30 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed rc=$?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOTDIR/bench.py" --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" \
    || { echo "rocprof failed rc=$?"; tail -30 "$OUT/prof_bench.err"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/prof" -name '*kernel_trace.csv' -exec python3 "$ROOTDIR/tools/trace_stats.py" {} \; > "$OUT/kernel_by_launch.csv"
cut -c1-200 "$OUT/kernel_by_launch.csv" | sed -n 1,8p
echo gpu_round done
