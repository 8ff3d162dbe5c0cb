#!/bin/bash
# PNG stream instance A/B: load bursts of 1 vs 2 groups (abso/lg1.so,
# abso/lg2.so): parity subset, times of the stream-layout probe shapes,
# FETCH_SIZE of each.  Usage (GPU box): bash tools/gpu_lg_ab.sh <tag>
set -eu -o pipefail
TAG=$1
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_png.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "png" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
export ZPX_PROBE_LAYOUT=stream
for r in 1 2; do
  for v in lg1 lg2; do
    echo "== round $r $v" | tee -a "$OUT/ab.log"
    ZPX_LIB_PATH=$ROOTDIR/abso/$v.so timeout -k 10 240 python -u tools/png_probe.py 4096 rgb8_flat rgba16_flat rgba16_adam7 2>&1 | grep -v amdgpu.ids | tee -a "$OUT/ab.log"
  done
done
cd /tmp
for v in lg1 lg2; do
  ZPX_LIB_PATH=$ROOTDIR/abso/$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_$v" -o run -- \
      python3 "$ROOTDIR/tools/png_probe.py" 4096 rgb8_flat rgba16_adam7 > "$OUT/pmc_$v.out" 2> "$OUT/pmc_$v.err" || { echo "pmc $v failed"; tail -5 "$OUT/pmc_$v.err"; exit 1; }
  find "$OUT/pmc_$v" -name '*counter_collection.csv' -exec cp {} "$OUT/pmc_$v.csv" \;
done
echo lg ab done
