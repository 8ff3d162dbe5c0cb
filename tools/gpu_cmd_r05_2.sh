set -eu -o pipefail
timeout -k 10 300 bash tools/ubench/run_load_calib.sh r05_calib2
bash tools/gpu_quick.sh r05_b1 none "" prof
