set -eu -o pipefail
mkdir -p gpurun_out/r05_e2e
timeout -k 10 300 python -u tools/e2e_ab.py 3 16 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05_e2e/ab.log
