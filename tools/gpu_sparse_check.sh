set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/sp; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sp/pytest.log 2>&1 || { tail -20 gpurun_out/sp/pytest.log; exit 1; }
tail -1 gpurun_out/sp/pytest.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sp/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-png --no-config5 --no-strip --no-cpu-baseline --steps 5 > $GRAFT_REPO_ROOT/gpurun_out/sp/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/sp/bench.err
grep -h sparse $GRAFT_REPO_ROOT/gpurun_out/sp/prof/run_kernel_stats.csv | cut -c1-160
