"""Batch pipeline debug aid: one JPEG fixture through the plan path, then the
batch path (host dst, device dst), printing as it goes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import test_gpu_batch as T  # noqa: E402
import zpix_amd  # noqa: E402
from zpix_amd import batch  # noqa: E402

mode = sys.argv[1]
i = int(sys.argv[2])
data = T.mixed_buffers()[i]
print("item", i, T.FIXTURES[i] if i < len(T.FIXTURES) else "synthetic", len(data), flush=True)
t0 = time.time()
if mode == "plan":
    out = zpix_amd.jpeg.decode_rgba(data) if data[:2] == b"\xff\xd8" else zpix_amd.png.decode(data).rgba_pixels()
    print("plan ok", out.shape, f"{time.time() - t0:.2f}s", flush=True)
else:
    res = batch.decode_rgba([data], host_threads=1, depth=1, on_host=(mode == "host"))
    print(mode, res[0].status, res[0].width, res[0].height, f"{time.time() - t0:.2f}s", flush=True)
