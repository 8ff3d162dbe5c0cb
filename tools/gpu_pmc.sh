#!/bin/bash
# PMC passes of a bench.py line (one rocprofv3 run per pass, --kernel-trace
# only next to --pmc; slot limits per pass respected), then the per-kernel
# summary (tools/pmc_summary.py).
# Usage: gpurun -- 'bash tools/gpu_pmc.sh <tag> "<bench args>" [extra pass counters (comma-separated)...]'
set -eu -o pipefail
TAG=${1:-pmc}; ARGS=${2:-"--no-png --no-config5 --no-e2e --steps 3 --warmup 1 --no-cpu-baseline"}; shift 2 || true
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export ZPX_BENCH_NO_INT16=${ZPX_BENCH_NO_INT16:-1}
cd /tmp
pass() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$ROOTDIR/bench.py" $ARGS > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "pass $name failed rc=$?"; tail -5 "$OUT/$name.err"; exit 1; }
}
# ZPX_PMC_SQ=0: the traffic passes only (FETCH_SIZE, WRITE_SIZE)
if [ "${ZPX_PMC_SQ:-1}" != 0 ]; then
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE
fi
pass fetch FETCH_SIZE
pass write WRITE_SIZE
for extra in "$@"; do pass "x_$(echo $extra | tr ',' '_')" $(echo $extra | tr ',' ' '); done
python3 "$ROOTDIR/tools/pmc_summary.py" "$OUT" "$OUT/traffic.json" > "$OUT/summary.json"
cat "$OUT/summary.json"
