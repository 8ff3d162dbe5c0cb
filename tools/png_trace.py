"""Per-band timeline of the paired-row PNG kernel (diagnostic build).

Run with a library built with -DZPX_PNG_TRACE=1 (tools/build_variants.sh
trace "-DZPX_PNG_TRACE=1"), e.g. on the GPU box:
  ZPX_LIB_PATH=zpix_amd/variants/trace.so python tools/png_trace.py --images 64
Prints: the launch's wall time from the band records, how many bands run
at once over time, band durations, the per-image lag between consecutive
bands, and how many waves / CUs held bands.
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=64)
    ap.add_argument("--size", type=int, default=4096)
    a = ap.parse_args()
    import numpy as np
    import torch

    from tools import synthetic as S
    from zpix_amd import _lib, device, png

    data = S.png_tc8_mixed(0, a.size, a.size)
    st = png.Stream(data)
    pb = device.PngBatch([st], slots=[0] * a.images)
    for _ in range(3):
        pb.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    L = _lib.lib()
    nb = a.images * ((a.size + 127) // 128)
    buf = (C.c_uint64 * (4 * nb))()
    L.zpx_debug_png_trace.argtypes = [C.c_void_p, C.c_size_t]
    assert L.zpx_debug_png_trace(buf, 4 * nb) == 0
    t = np.frombuffer(buf, np.uint64).reshape(nb, 4).astype(np.int64)
    t0 = t[:, 0].min()
    start = (t[:, 0] - t0) / 100.0  # us (100 MHz)
    end = (t[:, 1] - t0) / 100.0
    dur = end - start
    print(f"bands {nb}: wall {end.max():.1f} us; band duration mean {dur.mean():.1f} min {dur.min():.1f} max {dur.max():.1f}")
    hw = t[:, 2]
    hwid = hw & 0xffffffff
    xcc = (hw >> 32) & 0xf
    cu = (hwid >> 8) & 0xf
    sh = (hwid >> 12) & 1
    se = (hwid >> 13) & 0x7
    simd = (hwid >> 4) & 0x3
    wave = hwid & 0xf
    cus = set(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist()))
    slots = set(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist(), simd.tolist(), wave.tolist()))
    print(f"distinct CUs {len(cus)}, distinct wave slots {len(slots)}")
    ts = np.linspace(0, end.max(), 21)
    conc = [int(((start <= x) & (end > x)).sum()) for x in ts]
    print("bands running at t (us):", " ".join(f"{x:.0f}:{c}" for x, c in zip(ts, conc)))
    per_img = (a.size + 127) // 128
    # tickets are band-major: ticket = band * images + image
    st2 = start.reshape(per_img, a.images)
    lag = np.diff(st2, axis=0)
    print(f"start lag band b vs b-1 of one image: mean {lag.mean():.1f} us, max {lag.max():.1f}")
    steps = t[:, 3] >> 32
    skew = t[:, 3] & 0xffffffff
    print(f"steps mean {steps.mean():.1f}, max skew mean {skew.mean():.1f} max {skew.max()}")
    print(f"per-step time (duration / steps): {np.mean(dur / steps) * 1e3:.0f} ns")
    print("first 8 bands of image 0 (start, end us):",
          [(round(float(start[b * a.images]), 1), round(float(end[b * a.images]), 1)) for b in range(8)])


if __name__ == "__main__":
    main()
