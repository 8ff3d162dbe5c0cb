"""qoi module mirror (src/qoi/root.zig): decode / load / load_from_buffer /
probe_* and encode (src/qoi/encoder.zig).  Decoding is a serial host loop;
encoding runs on the GPU (a segmented scan, byte-identical to the serial
encoder)."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib, context
from .image import Image


@dataclass
class Desc:
    """qoi.Desc (src/qoi/encoder.zig:20-25)."""

    width: int
    height: int
    channels: int  # 3 = RGB, 4 = RGBA
    colorspace: int = 0  # 0 = sRGB with linear alpha, 1 = all channels linear

    def _c(self) -> "_lib.zpx_qoi_desc":
        d = _lib.zpx_qoi_desc()
        d.width, d.height, d.channels, d.colorspace = self.width, self.height, self.channels, self.colorspace
        return d


def decode(data: bytes, ctx: context.Context | None = None) -> Image:
    """qoi.decode (src/qoi/decoder.zig:20-130): an .RGBA image."""
    raw = _lib.zpx_image()
    _lib.check(_lib.lib().zpx_qoi_decode(ctx.handle if ctx else None, None, bytes(data), len(data), C.byref(raw)))
    return Image._from_c(raw)


def load_from_buffer(data: bytes, ctx: context.Context | None = None) -> Image:
    """qoi.loadFromBuffer (src/qoi/root.zig:34-38)."""
    return decode(data, ctx)


def load(path: str, ctx: context.Context | None = None) -> Image:
    """qoi.load (src/qoi/root.zig:20-31)."""
    raw = _lib.zpx_image()
    _lib.check(_lib.lib().zpx_qoi_load(ctx.handle if ctx else None, None, path.encode(), C.byref(raw)))
    return Image._from_c(raw)


def probe_buffer(data: bytes) -> bool:
    """qoi.probeBuffer (src/qoi/root.zig:41-49)."""
    return bytes(data[:4]) == b"qoif"


def probe_path(path: str) -> bool:
    """qoi.probePath (src/qoi/root.zig:52-64)."""
    with open(path, "rb") as f:
        return probe_buffer(f.read(4))


def encode_bound(desc: Desc) -> int:
    """The reference's maxSize (src/qoi/encoder.zig:41-42)."""
    d = desc._c()
    return int(_lib.lib().zpx_qoi_encode_bound(C.byref(d)))


def encode(pixels, desc: Desc, ctx: context.Context | None = None) -> bytes:
    """qoi.encode (src/qoi/encoder.zig:29-132) on the GPU: RGB(A) bytes -> QOI file bytes."""
    c = ctx or context.default()
    px = np.ascontiguousarray(np.asarray(pixels, dtype=np.uint8).reshape(-1))
    d = desc._c()
    out = C.POINTER(C.c_uint8)()
    n = C.c_size_t(0)
    L = _lib.lib()
    _lib.check(L.zpx_qoi_encode(c.handle, None, px.ctypes.data if px.size else None, px.size, C.byref(d),
                                C.byref(out), C.byref(n)), c.handle)
    try:
        return C.string_at(out, n.value)
    finally:
        _lib.libc_free(out)


def encode_device(d_pixels: int, desc: Desc, d_out: int, out_cap: int, d_out_len: int, stream=None,
                  ctx: context.Context | None = None) -> None:
    """Device form: pointers into HBM (e.g. torch tensors' data_ptr()); the
    encoded length is written to the device uint64 at d_out_len."""
    c = ctx or context.default()
    d = desc._c()
    _lib.check(_lib.lib().zpx_qoi_encode_device(c.handle, C.c_void_p(d_pixels), C.byref(d), C.c_void_p(d_out),
                                                out_cap, C.c_void_p(d_out_len), stream), c.handle)
