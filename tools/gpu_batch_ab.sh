#!/bin/bash
# One gpurun call: the pieces-transport tests + a short bench, then two
# kernel A/Bs (PNG flush shape, 4:4:4 waves per EU).
set -eu -o pipefail
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOTDIR"
bash tools/gpu_quick.sh pz1 "test_gpu_pieces or test_gpu_batch or test_gpu_jpeg_fused or planar" \
    "--steps 5 --warmup 2 --no-png --no-e2e --no-cpu-baseline --no-config5 --no-strip --no-planar"
export ZPX_BENCH_TIMING_ONLY=1 ZPX_BENCH_NO_INT16=1
bash tools/ab.sh pnga "base fl4w2" "--png-only --steps 8 --warmup 2 --no-cpu-baseline" 2
bash tools/ab.sh jpa "base w444" "--no-png --no-e2e --no-cpu-baseline --no-strip --no-planar --no-pieces --no-adam7 --steps 8 --warmup 2" 2
echo batch_ab done
