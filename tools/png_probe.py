"""PNG kernel probe (diagnostic): ms per launch of 64 x WxH images for several
depth / interlace shapes, to split the Adam7 cost from the per-byte cost.
Usage: python tools/png_probe.py [size] [shape ...]   (ZPX_LIB_PATH selects a library build)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import torch  # noqa: E402

from tools import synthetic as S  # noqa: E402
from zpix_amd import device, png  # noqa: E402


def timed(pb, n=8):
    s = torch.cuda.Stream()  # non-null: the plan launches on it and the events see it
    pb.launch(s.cuda_stream)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(n):
        pb.launch(s.cuda_stream)
    b.record(s)
    torch.cuda.synchronize()
    pb.status(s.cuda_stream)
    return a.elapsed_time(b) / n


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    shapes = [("rgba16_adam7", 16, 6, 1), ("rgba16_flat", 16, 6, 0), ("rgba8_adam7", 8, 6, 1),
              ("rgba8_flat", 8, 6, 0), ("rgb8_flat", 8, 2, 0)]
    pick = sys.argv[2:]
    for name, depth, ct, il in shapes:
        if pick and name not in pick:
            continue
        t0 = time.perf_counter()
        d = S.png_generic(7, size, size, depth, ct, interlace=il, filters=(1, 2, 3, 4))
        st = png.Stream(d)
        # ZPX_PROBE_LAYOUT: "auto" (host-built slab where the pair kernel takes it) or "stream"
        # ZPX_PROBE_N: images per plan (default 64)
        n = int(os.environ.get("ZPX_PROBE_N", "64"))
        pb = device.PngBatch([st], slots=[0] * n, layout=os.environ.get("ZPX_PROBE_LAYOUT", "auto"))
        ms = timed(pb)
        print(f"{name:14s} {ms:8.3f} ms/launch  {ms * 64 / n:8.3f} ms per 64 images  "
              f"{pb.bytes / ms / 1e6:8.1f} GB/s algorithmic  (prep {time.perf_counter() - t0:.1f}s)", flush=True)
        del pb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
