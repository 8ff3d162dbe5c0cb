#!/bin/bash
# PMC passes (one rocprofv3 run per pass, --kernel-trace next to --pmc only,
# per-block slot limits respected) of an arbitrary python command, then the
# per-kernel summary.  Usage (on the GPU box, from the repo root):
#   bash tools/gpu_pmc_cmd.sh <tag> <python script> [args...]
set -eu -o pipefail
TAG=$1; shift
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SCRIPT=$ROOTDIR/$1; shift
cd /tmp
pass() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$SCRIPT" $ARGS > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "pass $name failed rc=$?"; tail -5 "$OUT/$name.err"; exit 1; }
}
ARGS="$*"
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass tcc TCC_HIT_sum TCC_MISS_sum
python3 "$ROOTDIR/tools/pmc_summary.py" "$OUT" "$OUT/traffic.json" > "$OUT/summary.json"
cat "$OUT/summary.json"
