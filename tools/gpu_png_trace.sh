#!/bin/bash
# Band timeline of the paired-row PNG kernel (trace variant build).
set -eu -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/trace
for n in ${@:-64}; do
  ZPX_LIB_PATH=zpix_amd/variants/trace.so timeout -k 10 120 python -u tools/png_trace.py --images $n > gpurun_out/trace/n$n.txt 2>&1
  cat gpurun_out/trace/n$n.txt
done
