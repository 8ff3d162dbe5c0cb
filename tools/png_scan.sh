#!/bin/bash
# PNG kernel study: kernel time vs batch size, then PMC passes (one counter set per run).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/scan1
for n in 1 4 16 64; do
  timeout -k 10 200 python -u bench.py --png-only --no-cpu-baseline --images $n --distinct 1 > gpurun_out/scan1/i$n.json 2> gpurun_out/scan1/i$n.err || { echo fail $n; tail gpurun_out/scan1/i$n.err; exit 1; }
  python3 -c "import json,sys; r=json.load(open(sys.argv[1])); p=r.get('png',r); print(sys.argv[2], p.get('value'), p.get('roofline',{}).get('kernel_ms_per_launch'))" gpurun_out/scan1/i$n.json $n
done
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/scan1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $OUT/p1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --png-only --no-cpu-baseline --steps 3 --warmup 1 --distinct 1 > $OUT/p1.json 2> $OUT/p1.err || echo pmc1 fail
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --png-only --no-cpu-baseline --steps 3 --warmup 1 --distinct 1 > $OUT/p2.json 2> $OUT/p2.err || echo pmc2 fail
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/p3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --png-only --no-cpu-baseline --steps 3 --warmup 1 --distinct 1 > $OUT/p3.json 2> $OUT/p3.err || echo pmc3 fail
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/p4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --png-only --no-cpu-baseline --steps 3 --warmup 1 --distinct 1 > $OUT/p4.json 2> $OUT/p4.err || echo pmc4 fail
cd $GRAFT_REPO_ROOT && python3 tools/pmc_summary.py gpurun_out/scan1
