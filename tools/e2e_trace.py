"""Timeline of one end-to-end batch (the bench's 64 alternating 4K JPEG /
tc8 PNG images, 16 host threads) from the pipeline's trace lines
(ZPX_BATCH_TRACE=1, set here): run after a whole-batch warm-up; prints the
per-worker busy spans and the dispatcher's events relative to the batch start.
Usage: python tools/e2e_trace.py [threads] [depth] > timeline.txt 2> trace.log"""
import os
import sys
import time

os.environ["ZPX_BATCH_TRACE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import torch  # noqa: E402

from tools import synthetic as S  # noqa: E402
from zpix_amd import batch  # noqa: E402


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    depth = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    W = H = 4096
    uniq = {True: S.jpeg_420(0, W, H, 75), False: S.png_tc8_mixed(1, W, H)}
    bufs = [uniq[i % 2 == 0] for i in range(64)]
    arena = torch.empty(64 * W * H * 4, dtype=torch.uint8, device="cuda")
    dst = [arena[i * W * H * 4:(i + 1) * W * H * 4].view(H, W, 4) for i in range(64)]
    batch.decode_rgba(bufs, host_threads=threads, dst=dst)  # warm-up
    torch.cuda.synchronize()
    sys.stderr.flush()
    print(f"MARK {time.monotonic() * 1e3:.3f}", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    res, st = batch.decode_rgba(bufs, host_threads=threads, depth=depth, dst=dst, with_stats=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"wall {dt:.3f} s  host {st.host_s:.2f} s (jpeg {st.host_jpeg_s:.2f}, png {st.host_png_s:.2f})", flush=True)


if __name__ == "__main__":
    main()
