#!/bin/bash
# PNG bench line at several grid sizes (ZPX_PNG_WAVES_PER_CU) of the paired kernel.
set -eu -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/occ2
for w in ${@:-4 6 7 8}; do
  ZPX_PNG_WAVES_PER_CU=$w timeout -k 10 120 python -u bench.py --png-only --no-cpu-baseline > gpurun_out/occ2/w$w.json 2> gpurun_out/occ2/w$w.err
  python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print('waves/CU', sys.argv[2], r['roofline']['kernel_ms_per_launch'])" gpurun_out/occ2/w$w.json $w
done
