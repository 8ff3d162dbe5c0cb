"""Band slab layout (png_slab.cpp, ZPX_PNG_LAYOUT_SLAB) against a Python
model of it, on the host: the bytes the paired-row kernel reads at group g
for row r are the row's bytes from chunk 8 g - skew(r) on, zeros outside
(readImagePass's unfilter walk, src/png/decoder.zig:806-842).  The kernel on
the slab is checked by every -m gpu PNG test (PngBatch and the decode paths
upload slabs)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

from tools import synthetic as S  # noqa: E402
from zpix_amd import png  # noqa: E402

# depth code (zpx_png_depth) -> (bytes per pixel, chunk bytes)
GEOM = {4: (1, 16), 6: (3, 12), 11: (4, 16), 12: (2, 16), 14: (6, 12), 15: (8, 16)}
A7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def passes(w, h, bpp, interlace):
    """(pass width, rows, row bytes, stream offset) of every non-empty pass."""
    out, off = [], 0
    for xo, yo, xf, yf in (A7 if interlace else [(0, 0, 1, 1)]):
        pw = (max(w - xo, 0) + xf - 1) // xf
        ph = (max(h - yo, 0) + yf - 1) // yf
        if pw == 0 or ph == 0:
            continue
        rb = pw * bpp
        out.append((pw, ph, rb, off))
        off += ph * (rb + 1)
    return out


def skews(ft, rows):
    last, sk = 0, []
    for r in range(128):
        if r == 0 or r >= rows or ft[r] < 2:
            last = r
        sk.append(r - last)
    return sk, max(s for r, s in enumerate(sk) if r < rows)


def check_slab(st, slab=None):
    """The slab (the host's, st.slab(), unless given: e.g. the device-built
    one, tests/test_gpu_png.py) holds exactly the bytes the kernel reads."""
    f = st.frame
    bpp, cb = GEOM[f.depth]
    c, nq = cb // bpp, 8 * cb // 16
    stream = st.filtered()
    if slab is None:
        slab = st.slab()
    assert slab is not None
    ps = passes(f.width, f.height, bpp, f.interlace)
    nb = sum((p[1] + 127) // 128 for p in ps)
    offs = np.frombuffer(slab[:8 * nb].tobytes(), dtype=np.uint64)
    b = 0
    for pw, ph, rb, off in ps:
        nchunks = (pw + c - 1) // c
        for base in range(0, ph, 128):
            rows = min(128, ph - base)
            reg = slab[int(offs[b]):]
            assert int(offs[b]) % 256 == 0
            ft = [int(stream[off + (base + r) * (rb + 1)]) for r in range(rows)] + [0] * (128 - rows)
            assert list(reg[:128]) == ft
            sk, mx = skews(ft, rows)
            ngroups = (nchunks + mx + 7) // 8
            # per group and lane: the group windows of rows 2 lane and
            # 2 lane + 1 interleaved two bytes at a time (a0 a1 b0 b1 a2 a3
            # b2 b3 ...), as 2 NQ pieces: piece h NQ + q at tile h, piece q
            pieces = np.asarray(reg[128:128 + ngroups * 2 * nq * 1024]).reshape(ngroups, 2, nq, 64, 16)
            pad = 8 * cb * ngroups + 8 * cb * 128
            win = np.zeros((128, ngroups, 16 * nq), np.uint8)
            for r in range(128):
                row = (np.asarray(stream[off + (base + r) * (rb + 1) + 1: off + (base + r) * (rb + 1) + 1 + rb])
                       if r < rows else np.zeros(0, np.uint8))
                ext = np.zeros(pad + len(row) + pad, np.uint8)
                ext[pad:pad + len(row)] = row
                for g in range(ngroups):
                    s0 = pad + (8 * g - sk[r]) * cb
                    win[r, g] = ext[s0:s0 + 16 * nq]
            for lane in range(64):
                a = win[2 * lane].reshape(ngroups, 8 * nq, 2)
                bb = win[2 * lane + 1].reshape(ngroups, 8 * nq, 2)
                inter = np.concatenate([a, bb], axis=2).reshape(ngroups, 2, nq, 16)
                assert np.array_equal(pieces[:, :, :, lane], inter), (b, lane)
            b += 1
    assert b == nb


@pytest.mark.parametrize("depth,ct,w,h,il", [
    (8, 2, 70, 300, 0),     # TC8: 12-byte chunks, a partial last band
    (8, 6, 33, 130, 0),     # TCA8
    (16, 6, 21, 40, 1),     # TCA16 Adam7: every pass, empty-free
    (16, 2, 17, 17, 1),     # TC16 Adam7, tiny passes
    (8, 0, 100, 129, 0),    # G8
    (16, 0, 64, 64, 0),     # G16
])
def test_slab_layout_matches_model(depth, ct, w, h, il):
    d = S.png_generic(3, w, h, depth, ct, interlace=il, filters=(0, 1, 2, 3, 4))
    st = png.Stream(d)
    check_slab(st)


def test_slab_refused_where_pair_kernel_does_not_take_it():
    # paletted and sub-byte depths stay on the one-row kernel (stream layout)
    d = S.png_generic(5, 40, 20, 4, 0)
    assert png.Stream(d).slab() is None
