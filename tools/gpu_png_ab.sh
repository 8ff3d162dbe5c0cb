#!/bin/bash
# One gpurun call: the PNG GPU tests, then an A/B of abso/old.so vs
# abso/new.so on the PNG lines (tc8 from the slab and from the stream,
# Adam7 RGBA16).
set -eu -o pipefail
ROOTDIR=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOTDIR"
bash tools/gpu_quick.sh pngt "png or slab or batch or rgba" "--png-only --steps 4 --warmup 1 --no-cpu-baseline"
export ZPX_BENCH_TIMING_ONLY=1 ZPX_BENCH_NO_INT16=1
bash tools/ab.sh pngab "old new" "--png-only --steps 10 --warmup 2 --no-cpu-baseline" 3
bash tools/ab.sh a7ab "old new" "--no-png --no-e2e --no-cpu-baseline --no-strip --no-planar --no-pieces --steps 6 --warmup 2" 2
echo png_ab done
