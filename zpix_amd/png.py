"""png module mirror (src/png/root.zig): load / load_from_buffer / decode /
probe_*; plus the host inflate stage for batching."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib, context
from .image import Image

PNG_SIGNATURE = b"\x89PNG\r\n\x1a\n"
INPUT_PAD = 256  # ZPX_PNG_INPUT_PAD
# zpx_png_depth (ColorBitDepth, src/png/decoder.zig:88-118)
DEPTHS = {"g1": 1, "g2": 2, "g4": 3, "g8": 4, "ga8": 5, "tc8": 6, "p1": 7, "p2": 8, "p4": 9, "p8": 10,
          "tca8": 11, "g16": 12, "ga16": 13, "tc16": 14, "tca16": 15}


def decode(data: bytes, ctx: context.Context | None = None) -> Image:
    """png.decode (src/png/decoder.zig:143-221) over an in-memory buffer."""
    c = ctx or context.default()
    raw = _lib.zpx_image()
    _lib.check(_lib.lib().zpx_png_decode(c.handle, None, bytes(data), len(data), C.byref(raw)), c.handle)
    return Image._from_c(raw)


def load_from_buffer(data: bytes, ctx: context.Context | None = None) -> Image:
    """png.loadFromBuffer (src/png/root.zig:29-34)."""
    return decode(data, ctx)


def load(path: str, ctx: context.Context | None = None) -> Image:
    """png.load (src/png/root.zig:13-27)."""
    c = ctx or context.default()
    raw = _lib.zpx_image()
    _lib.check(_lib.lib().zpx_png_load(c.handle, None, path.encode(), C.byref(raw)), c.handle)
    return Image._from_c(raw)


def decode_config(data: bytes):
    """(width, height) from the signature + IHDR (png/decoder.zig:224-401)."""
    w, h = C.c_uint32(0), C.c_uint32(0)
    _lib.check(_lib.lib().zpx_png_decode_config(bytes(data), len(data), C.byref(w), C.byref(h)))
    return w.value, h.value


def probe_buffer(data: bytes) -> bool:
    """png.probeBuffer (src/png/root.zig:37-40)."""
    return bytes(data[:8]) == PNG_SIGNATURE


def probe_path(path: str) -> bool:
    """png.probePath (src/png/root.zig:43-52)."""
    with open(path, "rb") as f:
        return probe_buffer(f.read(8))


class Stream:
    """Host stage output: the inflated filtered stream in pinned memory."""

    def __init__(self, data: bytes):
        h = C.c_void_p()
        self._data = bytes(data)
        _lib.check(_lib.lib().zpx_png_inflate(self._data, len(self._data), C.byref(h)))
        self.handle = h
        self.frame = _lib.zpx_png_frame()
        n = C.c_size_t(0)
        _lib.check(_lib.lib().zpx_png_stream_frame(h, C.byref(self.frame), C.byref(n)))
        self.filtered_len = n.value

    def filtered(self) -> np.ndarray:
        """The filtered stream (+INPUT_PAD zero bytes) as a host numpy view."""
        ptr = _lib.lib().zpx_png_stream_data(self.handle)
        return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(self.filtered_len + INPUT_PAD,))

    def slab(self):
        """The band slab (ZPX_PNG_LAYOUT_SLAB: the paired-row kernel's input
        layout, png_slab.cpp) as a host numpy view, or None when that kernel
        does not take the image."""
        p, n = C.c_void_p(), C.c_size_t(0)
        rc = _lib.lib().zpx_png_stream_slab(self.handle, C.byref(p), C.byref(n))
        if rc and _lib.error_name(rc) == "Unsupported":
            return None
        _lib.check(rc)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(n.value,))

    def close(self):
        if self.handle:
            _lib.lib().zpx_png_stream_free(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
