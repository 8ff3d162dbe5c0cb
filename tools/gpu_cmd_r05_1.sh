set -eu -o pipefail
bash tools/gpu_focus.sh r05_f1 "epoch_cycle or sharded or recreated or batch" prof
timeout -k 10 400 bash tools/png_ab.sh r05_ab1 "base fl4w1 fl4w2" "rgb8_flat rgba16_flat" 2
timeout -k 10 300 bash tools/ubench/run_load_calib.sh r05_calib
