#!/bin/bash
# SQ counter passes of the PNG probe (one shape, slab layout) for library
# variants abso/<v>.so: why a variant is faster or slower.
# Usage (GPU box): bash tools/gpu_pmc_variants.sh <tag> "<variants>" <shape>
set -eu -o pipefail
TAG=$1; VARS=$2; SHAPE=$3
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for v in $VARS; do
  i=0
  for p in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    ZPX_LIB_PATH=$ROOTDIR/abso/$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $p --output-format csv -d "$OUT/${v}_p$i" -o run -- \
        python3 "$ROOTDIR/tools/png_probe.py" 4096 $SHAPE > "$OUT/${v}_p$i.out" 2> "$OUT/${v}_p$i.err" || { echo "pass $v $i failed"; tail -5 "$OUT/${v}_p$i.err"; exit 1; }
    find "$OUT/${v}_p$i" -name '*counter_collection.csv' -exec cp {} "$OUT/${v}_p$i.csv" \;
  done
done
echo pmc variants done
