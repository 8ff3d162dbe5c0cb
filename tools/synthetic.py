"""Seeded synthetic inputs for parity tests and bench.py.

content: uint8 RGB = clip(128 + 100*sin(x/97+c)*cos(y/131-c) + N(0,12)), c = 0,1,2,
with numpy.random.default_rng(seed), seed = image index.

- jpeg_420(seed, w, h, quality=75): baseline 4:2:0 JFIF (Pillow, subsampling=2)
- jpeg_progressive_444(seed, w, h): progressive 4:4:4 (Pillow)
- png_tc8_mixed(seed, w, h): truecolor-8 PNG, per-row filter drawn from {1,2,3,4}
  (own encoder: numpy forward filter, zlib level 6, 64 KiB IDAT chunks, CRCs)
- png_rgba16_adam7(seed, w, h): Adam7-interlaced RGBA16 PNG (own encoder;
  Pillow cannot write interlaced PNG), per-row filters from {0..4}
"""
from __future__ import annotations

import io
import struct
import zlib

import numpy as np

ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def content(seed: int, w: int, h: int, channels: int = 3) -> np.ndarray:
    rng = np.random.default_rng(seed)
    x = np.arange(w, dtype=np.float32)[None, :]
    y = np.arange(h, dtype=np.float32)[:, None]
    out = np.empty((h, w, channels), np.uint8)
    for c in range(channels):
        v = 128 + 100 * np.sin(x / 97 + c) * np.cos(y / 131 - c) + rng.normal(0, 12, (h, w)).astype(np.float32)
        out[..., c] = np.clip(v, 0, 255).astype(np.uint8)
    return out


def jpeg_420(seed: int, w: int, h: int, quality: int = 75) -> bytes:
    from PIL import Image

    b = io.BytesIO()
    Image.fromarray(content(seed, w, h)).save(b, "JPEG", quality=quality, subsampling=2)
    return b.getvalue()


def jpeg_subsampled(seed: int, w: int, h: int, subsampling: int, quality: int = 75, progressive=False) -> bytes:
    from PIL import Image

    b = io.BytesIO()
    Image.fromarray(content(seed, w, h)).save(b, "JPEG", quality=quality, subsampling=subsampling,
                                             progressive=progressive)
    return b.getvalue()


def jpeg_progressive_444(seed: int, w: int, h: int, quality: int = 75) -> bytes:
    return jpeg_subsampled(seed, w, h, 0, quality, progressive=True)


def jpeg_gray(seed: int, w: int, h: int, quality: int = 75, progressive=False) -> bytes:
    from PIL import Image

    b = io.BytesIO()
    Image.fromarray(content(seed, w, h, 1)[..., 0]).save(b, "JPEG", quality=quality, progressive=progressive)
    return b.getvalue()


# ---------------------------------------------------------------- PNG encoder
def _chunk(tag: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def filter_rows(raw: np.ndarray, bpp: int, ftypes: np.ndarray) -> np.ndarray:
    """Forward PNG filtering of raw rows (H, row_bytes) with per-row types.
    Uses only the raw (unfiltered) bytes, so every row is vectorised."""
    h, n = raw.shape
    r = raw.astype(np.int16)
    up = np.zeros_like(r)
    up[1:] = r[:-1]
    left = np.zeros_like(r)
    left[:, bpp:] = r[:, :-bpp]
    ul = np.zeros_like(r)
    ul[1:, bpp:] = r[:-1, :-bpp]
    p = left + up - ul
    pa, pb, pc = np.abs(p - left), np.abs(p - up), np.abs(p - ul)
    paeth = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, up, ul))
    preds = [np.zeros_like(r), left, up, (left + up) >> 1, paeth]
    out = np.empty((h, n + 1), np.uint8)
    out[:, 0] = ftypes
    for t in range(5):
        rows = ftypes == t
        if rows.any():
            out[rows, 1:] = ((r[rows] - preds[t][rows]) & 0xFF).astype(np.uint8)
    return out


def encode_png(w: int, h: int, depth: int, color_type: int, filtered: bytes, interlace: int = 0,
               level: int = 6, idat_chunk: int = 65536, extra_chunks: list | None = None) -> bytes:
    z = zlib.compress(filtered, level)
    out = [b"\x89PNG\r\n\x1a\n", _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, color_type, 0, 0, interlace))]
    for tag, data in extra_chunks or []:
        out.append(_chunk(tag, data))
    for i in range(0, len(z), idat_chunk):
        out.append(_chunk(b"IDAT", z[i:i + idat_chunk]))
    out.append(_chunk(b"IEND", b""))
    return b"".join(out)


def png_filtered_tc8(seed: int, w: int, h: int, filters=(1, 2, 3, 4)) -> tuple[np.ndarray, np.ndarray]:
    """(raw RGB rows (H, 3W), filtered stream (H, 1+3W)) of the bench PNG."""
    rgb = content(seed, w, h)
    raw = rgb.reshape(h, w * 3)
    ft = np.random.default_rng(seed).choice(np.array(filters, np.uint8), size=h)
    return raw, filter_rows(raw, 3, ft)


def png_tc8_mixed(seed: int, w: int, h: int, filters=(1, 2, 3, 4)) -> bytes:
    _, f = png_filtered_tc8(seed, w, h, filters)
    return encode_png(w, h, 8, 2, f.tobytes())


def png_generic(seed: int, w: int, h: int, depth: int, color_type: int, interlace: int = 0,
                filters=(0, 1, 2, 3, 4), trns: bytes | None = None, palette: bytes | None = None) -> bytes:
    """Random content PNG of any depth / colour type, per-row random filters."""
    rng = np.random.default_rng(seed)
    chans = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[color_type]
    bits = depth * chans
    bpp = max(1, bits // 8)

    def rows_for(pw, ph, salt):
        row_bytes = (bits * pw + 7) // 8
        if depth >= 8:
            smooth = content(seed * 31 + salt, pw, ph, chans).astype(np.uint16)
            if depth == 16:
                vals = (smooth << 8) | rng.integers(0, 256, smooth.shape, dtype=np.uint16)
                raw = vals.astype(">u2").view(np.uint8).reshape(ph, row_bytes)
            else:
                raw = smooth.astype(np.uint8).reshape(ph, row_bytes)
            if color_type == 3:
                raw = (raw % (len(palette) // 3 if palette else 256)).astype(np.uint8)
        else:
            maxv = (1 << depth) - 1
            if color_type == 3 and palette:
                maxv = min(maxv, len(palette) // 3 - 1)
            px = rng.integers(0, maxv + 1, (ph, pw), dtype=np.uint8)
            per = 8 // depth
            pad = (-pw) % per
            px = np.concatenate([px, np.zeros((ph, pad), np.uint8)], 1).reshape(ph, -1, per)
            raw = np.zeros((ph, px.shape[1]), np.uint8)
            for j in range(per):
                raw |= (px[:, :, j] << (8 - depth * (j + 1))).astype(np.uint8)
        ft = rng.choice(np.array(filters, np.uint8), size=ph)
        return filter_rows(raw, bpp, ft)

    if interlace:
        parts = []
        for p, (xo, yo, xf, yf) in enumerate(ADAM7):
            pw = (max(w - xo, 0) + xf - 1) // xf
            ph = (max(h - yo, 0) + yf - 1) // yf
            if pw == 0 or ph == 0:
                continue
            parts.append(rows_for(pw, ph, p).tobytes())
        stream = b"".join(parts)
    else:
        stream = rows_for(w, h, 0).tobytes()
    extra = []
    if palette is not None:
        extra.append((b"PLTE", palette))
    if trns is not None:
        extra.append((b"tRNS", trns))
    return encode_png(w, h, depth, color_type, stream, interlace, extra_chunks=extra)


def png_rgba16_adam7(seed: int, w: int, h: int) -> bytes:
    return png_generic(seed, w, h, 16, 6, interlace=1)


def bmp_bytes(seed: int, w: int, h: int, bpp: int, top_down: bool = False, header: int = 40,
              ncol: int = 0, bitfields: bool = False) -> tuple[bytes, np.ndarray]:
    """An uncompressed BMP (the layouts src/bmp/decoder.zig:42-307 accepts) with
    random pixel data; returns (file bytes, raw row data as stored)."""
    rng = np.random.default_rng(seed)
    if bpp <= 8:
        ppb = 8 // bpp
        row = ((w + ppb - 1) // ppb + 3) & ~3
        ncol_eff = ncol or (1 << bpp)
        pal = rng.integers(0, 256, (ncol_eff, 4), dtype=np.uint8).tobytes()
    else:
        row = (w * 3 + 3) & ~3 if bpp == 24 else w * 4
        ncol_eff, pal = 0, b""
    rows = rng.integers(0, 256, (h, row), dtype=np.uint8)
    info = bytearray(header)
    struct.pack_into("<IiiHHI", info, 0, header, w, -h if top_down else h, 1, bpp, 3 if bitfields else 0)
    struct.pack_into("<I", info, 32, ncol)
    if header > 40:
        struct.pack_into("<IIII", info, 40, 0xFF0000, 0x00FF00, 0x0000FF, 0xFF000000)
    off = 14 + header + len(pal)
    data = rows.tobytes()
    fh = b"BM" + struct.pack("<IHHI", off + len(data), 0, 0, off)
    return fh + bytes(info) + pal + data, rows
