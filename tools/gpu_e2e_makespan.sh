#!/bin/bash
# e2e batch pipeline: batch_makespan 0 vs 1 at 12-16 host threads (round 6),
# after the batch GPU tests.  gpurun -- 'bash tools/gpu_e2e_makespan.sh <tag>'
set -eu -o pipefail
TAG=${1:-e2e}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_batch.log" 2>&1 \
    || { echo "batch tests failed"; tail -20 "$OUT/pytest_batch.log"; exit 1; }
tail -1 "$OUT/pytest_batch.log"
for th in 12 14 15 16 10; do
  echo "== threads $th" | tee -a "$OUT/ab.txt"
  timeout -k 10 240 python -u tools/e2e_ab.py 3 $th batch_makespan 0 1 >> "$OUT/ab.txt" 2>&1 \
      || { echo "e2e_ab failed"; tail -20 "$OUT/ab.txt"; exit 1; }
done
cat "$OUT/ab.txt"
