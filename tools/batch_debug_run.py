"""Batch pipeline debug aid: runs zpx_batch_decode_rgba on one item at a time
(item index from argv) and prints its status."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import test_gpu_batch as T  # noqa: E402
from zpix_amd import batch  # noqa: E402

bufs = T.mixed_buffers()
lo, hi = int(sys.argv[1]), int(sys.argv[2])
for i in range(lo, min(hi, len(bufs))):
    t0 = time.time()
    res = batch.decode_rgba([bufs[i]], host_threads=1, depth=1)
    print(i, T.FIXTURES[i] if i < len(T.FIXTURES) else "synthetic", res[0].status, res[0].format,
          res[0].width, res[0].height, f"{time.time() - t0:.2f}s", flush=True)
