#!/bin/bash
# PMC passes of the PNG bench line (png-only bench, one rocprofv3 run per
# pass, --kernel-trace only next to --pmc), plus the counter list.
# Usage: gpurun -- 'bash tools/gpu_png_pmc2.sh <tag> [extra pass counters...]'
set -eu -o pipefail
TAG=${1:-pngpmc2}; shift || true
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--png-only --steps 3 --warmup 1 --distinct 1 --no-cpu-baseline"
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
pass() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$ROOTDIR/bench.py" $ARGS > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "pass $name failed rc=$?"; tail -5 "$OUT/$name.err"; exit 1; }
}
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
for extra in "$@"; do pass "x_$(echo $extra | tr ',' '_')" $(echo $extra | tr ',' ' '); done
python3 "$ROOTDIR/tools/pmc_summary.py" "$OUT" > "$OUT/summary.json"
cat "$OUT/summary.json"
