set -eu -o pipefail
mkdir -p gpurun_out/r05_e2e
for t in 16 15 14; do
  echo "== threads $t" | tee -a gpurun_out/r05_e2e/ab4.log
  cat /sys/fs/cgroup/cpu.stat | tee -a gpurun_out/r05_e2e/ab4.log
  timeout -k 10 300 python -u tools/e2e_ab.py 2 $t 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05_e2e/ab4.log
  cat /sys/fs/cgroup/cpu.stat | tee -a gpurun_out/r05_e2e/ab4.log
done
