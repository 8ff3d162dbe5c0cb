#!/bin/bash
# PNG kernel iteration: gpu parity suite on the main build, then PNG-only bench
# of the main build and every zpix_amd/variants/*.so.
# Usage: gpurun --timeout 900 -- 'bash tools/gpu_png_variants.sh <tag> [bench args]'
set -eu -o pipefail
TAG=${1:-pngvar}; shift || true
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOTDIR"
timeout -k 10 300 python -u -m pytest tests/test_gpu_png.py tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest -m gpu failed rc=$?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
run() {
  local n=$1 so=$2; shift 2
  ZPX_LIB_PATH=$so timeout -k 10 200 python -u bench.py --png-only --no-cpu-baseline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" \
      || { echo "bench $n failed rc=$?"; tail -20 "$OUT/$n.err"; exit 1; }
  python3 -c "import json,sys; r=json.load(open(sys.argv[1])); p=r.get('png',r); print(sys.argv[2], 'PNG', p.get('value'), p.get('roofline',{}).get('frac'), p.get('roofline',{}).get('kernel_ms_per_launch'))" "$OUT/$n.json" "$n"
}
run main "$ROOTDIR/zpix_amd/libzpix_amd.so" "$@"
for so in zpix_amd/variants/*.so; do
  [ -e "$so" ] || continue
  run "$(basename "$so" .so)" "$ROOTDIR/$so" "$@"
done
echo done
