"""Probe: planar (jpeg.load) output vs the oracle on the fixtures, reporting
where the first mismatches are (plane, block) -- a debugging aid."""
import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import oracle_py as O  # noqa: E402
from conftest import golden  # noqa: E402
from zpix_amd import _lib  # noqa: E402
from zpix_amd import jpeg as J  # noqa: E402

for strip in (0, 1):
    _lib.lib().zpx_debug_option(b"jpeg_strip", strip)
    for p in sorted(glob.glob(golden("testdata", "*.jpeg"))):
        data = open(p, "rb").read()
        try:
            want = O.jpeg_decode(data)
        except O.OracleError:
            continue
        got = J.decode(data)
        co = J.Coefficients(data)
        f = co.frame
        ok = np.array_equal(got.pixels, want.pixels)
        line = f"strip={strip} {os.path.basename(p)} bits={f.coeff_bits} ok={ok}"
        if not ok and want.kind == "YCbCr":
            g, w = got.pixels, want.pixels
            for name, off, stride, end in (("Y", 0, want.y_stride, want.cb_off), ("Cb", want.cb_off, want.c_stride, want.cr_off),
                                           ("Cr", want.cr_off, want.c_stride, len(w))):
                d = np.nonzero(g[off:end] != w[off:end])[0]
                if len(d):
                    ys, xs = d // stride, d % stride
                    blocks = sorted({(int(y) // 8, int(x) // 8) for y, x in zip(ys, xs)})
                    line += f" {name}: {len(d)} bytes, blocks {blocks[:6]}... ({len(blocks)}) first (y,x)=({ys[0]},{xs[0]}) got {g[off + d[0]]} want {w[off + d[0]]}"
        print(line, flush=True)
