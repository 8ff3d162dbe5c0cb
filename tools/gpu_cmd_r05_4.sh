set -eu -o pipefail
mkdir -p gpurun_out/r05_a7
for r in 1 2; do for v in base a7p7; do
  echo "== round $r $v" | tee -a gpurun_out/r05_a7/ab.log
  ZPX_PROBE_LAYOUT=stream ZPX_LIB_PATH=$PWD/abso/$v.so timeout -k 10 200 python -u tools/png_probe.py 4096 rgba16_adam7 rgba8_adam7 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05_a7/ab.log
done; done
