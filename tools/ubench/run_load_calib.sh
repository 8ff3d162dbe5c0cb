#!/bin/bash
# FETCH_SIZE calibration of the PNG stream instance's load shape
# (png_load_pattern modes 1 / 3 / 5): time of each mode, then one
# rocprofv3 --pmc FETCH_SIZE pass per mode (own process, KILL timeout).
# Usage (GPU box, repo root): bash tools/ubench/run_load_calib.sh <tag>
set -eu -o pipefail
TAG=$1
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B=$ROOTDIR/tools/ubench/png_load_pattern
for m in 1 3 8 6 7 5 0; do timeout -k 5 60 "$B" $m 8 | tee -a "$OUT/calib.log"; done
cd /tmp
for m in 3 8; do
  for p in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    q=$(echo $p | cut -c1-5)
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $p --output-format csv \
        -d "$OUT/m$m$q" -o run -- "$B" $m 8 > "$OUT/m$m$q.out" 2> "$OUT/m$m$q.err" || { echo "pmc mode $m $q failed"; tail -5 "$OUT/m$m$q.err"; exit 1; }
    find "$OUT/m$m$q" -name '*counter_collection.csv' -exec cp {} "$OUT/m$m.$q.csv" \;
  done
done
echo calib done
