"""A/B of an end-to-end batch pipeline test switch (configs[3] on one GPU,
the bench's 64 alternating 4K JPEG / tc8 PNG images): option <name> at value
A against value B (default "batch_lookahead" 0 -- the costliest of the next
2 x threads items first -- against 1, item order), rounds alternating, after
one full-batch warm-up (pinned pools at their steady state).  Prints the
decode wall and the host CPU per stage.
Usage: python tools/e2e_ab.py [rounds] [threads] [name A B]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import torch  # noqa: E402

from tools import synthetic as S  # noqa: E402
from zpix_amd import _lib, batch  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    name = sys.argv[3].encode() if len(sys.argv) > 3 else b"batch_lookahead"
    modes = (int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (0, 1)
    W = H = 4096
    uniq = {True: S.jpeg_420(0, W, H, 75), False: S.png_tc8_mixed(1, W, H)}
    bufs = [uniq[i % 2 == 0] for i in range(64)]
    arena = torch.empty(64 * W * H * 4, dtype=torch.uint8, device="cuda")
    dst = [arena[i * W * H * 4:(i + 1) * W * H * 4].view(H, W, 4) for i in range(64)]
    L = _lib.lib()
    batch.decode_rgba(bufs, host_threads=threads, dst=dst)  # warm-up: the whole batch
    torch.cuda.synchronize()
    for r in range(rounds):
        for mode in modes:
            prev = L.zpx_debug_option(name, mode)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res, st = batch.decode_rgba(bufs, host_threads=threads, dst=dst, with_stats=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            L.zpx_debug_option(name, prev)
            assert all(x.status == "Ok" for x in res)
            print(f"round {r} {name.decode()}={mode}: wall {dt:.3f} s (run loop {st.wall_s:.3f})  "
                  f"{64 * W * H / dt / 1e6:7.1f} MPix/s  host {st.host_s:.2f} s (jpeg {st.host_jpeg_s:.2f}, "
                  f"png {st.host_png_s:.2f})", flush=True)


if __name__ == "__main__":
    main()
