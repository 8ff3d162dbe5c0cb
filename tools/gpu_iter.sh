#!/bin/bash
# One gpurun iteration: selected GPU tests, then a bench run with chosen flags.
# Usage: gpurun -- 'bash tools/gpu_iter.sh <tag> "<pytest files/-k>" "<bench flags>"'
set -eu -o pipefail
TAG=${1:-iter}
TESTS=${2:-}
BFLAGS=${3:-}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
fi
if [ "$BFLAGS" != "none" ]; then
  timeout -k 10 300 python -u bench.py $BFLAGS > "$OUT/bench.json" 2> "$OUT/bench.err" \
      || { echo "bench failed rc=$?"; tail -30 "$OUT/bench.err"; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('jpeg', d['ms_per_step'], d['roofline']['frac'])
p=d.get('png');
if p: print('png', p['ms_per_step'], p['roofline']['kernel_ms_per_launch'], p['roofline']['frac'])
c=d.get('config5',{})
for k,v in c.items(): print(k, v.get('kernel_ms_per_launch'), v['roofline']['frac'])
s=d.get('odd_width')
if s: print('odd_width', s['kernel_ms_per_launch'], s['roofline']['frac'], 'strip', s['strip_kernel']['kernel_ms_per_launch'], s['strip_kernel']['roofline']['frac'])
"
fi
echo iter done
