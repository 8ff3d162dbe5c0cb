set -e
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/a7ab; cd /tmp; export TMPDIR=/tmp
for v in ${VARIANTS:-base nosc}; do
  ZPX_LIB_PATH=$GRAFT_REPO_ROOT/abso/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/a7ab/$v -o run -- python3 $GRAFT_REPO_ROOT/tools/png_probe.py 4096 rgba16_adam7 > $GRAFT_REPO_ROOT/gpurun_out/a7ab/$v.log 2>&1
  grep ms/launch $GRAFT_REPO_ROOT/gpurun_out/a7ab/$v.log
  python3 $GRAFT_REPO_ROOT/tools/trace_stats.py $GRAFT_REPO_ROOT/gpurun_out/a7ab/$v/run_kernel_trace.csv | grep pair_kernel | cut -c1-120
done
