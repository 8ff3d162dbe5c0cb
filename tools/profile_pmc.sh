#!/bin/bash
# PMC passes for the bench kernels (run on the GPU box from the repo root).
# Each pass is its own rocprofv3 run with --kernel-trace only (no sys/runtime
# trace next to --pmc).  Output: gpurun_out/pmc/<pass>/...
set -u
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOTDIR/gpurun_out/pmc
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --distinct 1 --no-cpu-baseline --no-config5 --no-e2e"}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export ZPX_BENCH_NO_INT16=1 # one kernel instance per pass (mean per dispatch)
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
      python3 $ROOTDIR/bench.py $ARGS > $OUT/$name.json 2> $OUT/$name.err || { echo "pass $name failed rc=$?"; exit 1; }
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES
run sq2 SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
echo pmc done
