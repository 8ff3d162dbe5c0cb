#!/bin/bash
# PNG A/B with traffic: for the main library and each variant, a png-only
# bench line, then FETCH_SIZE and WRITE_SIZE passes (each its own rocprofv3
# run, --kernel-trace only next to --pmc).
# Usage: gpurun -- 'bash tools/gpu_png_pmc.sh <tag>'
set -eu -o pipefail
TAG=${1:-pngpmc}
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp ZPX_BENCH_NO_INT16=1
ARGS="--png-only --steps 3 --warmup 1 --distinct 1 --no-cpu-baseline --no-config5 --no-e2e"
for so in "$ROOTDIR"/zpix_amd/libzpix_amd.so "$ROOTDIR"/zpix_amd/variants/*.so; do
  [ -e "$so" ] || continue
  n=$(basename "$so" .so)
  cd "$ROOTDIR"
  ZPX_LIB_PATH=$so timeout -k 10 200 python -u bench.py --png-only --no-cpu-baseline > "$OUT/$n.json" 2> "$OUT/$n.err" \
      || { echo "bench $n failed rc=$?"; tail -20 "$OUT/$n.err"; exit 1; }
  python3 -c "import json,sys; r=json.load(open(sys.argv[1])); p=r.get('png',r); print(sys.argv[2], 'PNG', p.get('value'), p.get('roofline',{}).get('frac'), p.get('roofline',{}).get('kernel_ms_per_launch'))" "$OUT/$n.json" "$n"
  cd /tmp
  mkdir -p "$OUT/pmc_$n"
  for c in FETCH_SIZE WRITE_SIZE; do
    ZPX_LIB_PATH=$so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/pmc_$n/$c" -o run -- \
        python3 "$ROOTDIR/bench.py" $ARGS > "$OUT/pmc_$n/$c.json" 2> "$OUT/pmc_$n/$c.err" || { echo "pmc $n $c failed rc=$?"; exit 1; }
  done
  python3 "$ROOTDIR/tools/pmc_summary.py" "$OUT/pmc_$n" > "$OUT/pmc_$n.json" 2>/dev/null || true
  grep -A3 png_unfilter "$OUT/pmc_$n.json" | head -4 || true
done
echo done
