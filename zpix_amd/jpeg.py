"""jpeg module mirror (src/jpeg/root.zig): load / load_from_buffer / decode /
probe_*; plus decode_rgba (decode + Image.rgbaPixels fused on the GPU) and
the host entropy stage for batching."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib, context
from .image import Image


def decode(data: bytes, ctx: context.Context | None = None) -> Image:
    """jpeg.decode (src/jpeg/decoder.zig:155-176) over an in-memory buffer."""
    c = ctx or context.default()
    raw = _lib.zpx_image()
    _lib.check(_lib.lib().zpx_jpeg_decode(c.handle, None, bytes(data), len(data), C.byref(raw)), c.handle)
    return Image._from_c(raw)


def load_from_buffer(data: bytes, ctx: context.Context | None = None) -> Image:
    """jpeg.loadFromBuffer (src/jpeg/root.zig:10-15)."""
    return decode(data, ctx)


def load(path: str, ctx: context.Context | None = None) -> Image:
    """jpeg.load (src/jpeg/root.zig:36-53)."""
    c = ctx or context.default()
    raw = _lib.zpx_image()
    _lib.check(_lib.lib().zpx_jpeg_load(c.handle, None, path.encode(), C.byref(raw)), c.handle)
    return Image._from_c(raw)


MODELS = {0: "RGB", 1: "YCbCr", 2: "RGBA", 3: "Gray"}


def decode_config(data: bytes):
    """jpeg.decodeConfig (src/jpeg/decoder.zig:178-218) -> (width, height).
    `decode_config_model` also returns the colour model name."""
    w, h, _ = decode_config_model(data)
    return w, h


def decode_config_model(data: bytes):
    w, h, m = C.c_uint32(0), C.c_uint32(0), C.c_int32(0)
    _lib.check(_lib.lib().zpx_jpeg_decode_config(bytes(data), len(data), C.byref(w), C.byref(h), C.byref(m)))
    return w.value, h.value, MODELS[m.value]


def probe_buffer(data: bytes) -> bool:
    """jpeg.probeBuffer (src/jpeg/root.zig:17-21)."""
    return bool(_lib.lib().zpx_jpeg_probe_buffer(bytes(data[:2]), min(len(data), 2)))


def probe_path(path: str) -> bool:
    """jpeg.probePath (src/jpeg/root.zig:23-33)."""
    with open(path, "rb") as f:
        return probe_buffer(f.read(2))


def decode_rgba(data: bytes, ctx: context.Context | None = None):
    """decode + Image.rgbaPixels in one fused kernel: returns (rgba uint8 HxWx4)."""
    c = ctx or context.default()
    out = C.POINTER(C.c_uint8)()
    n = C.c_size_t(0)
    w = C.c_uint32(0)
    h = C.c_uint32(0)
    _lib.check(_lib.lib().zpx_jpeg_decode_rgba(c.handle, None, bytes(data), len(data), C.byref(out), C.byref(n),
                                               C.byref(w), C.byref(h)), c.handle)
    try:
        return np.ctypeslib.as_array(out, shape=(n.value,)).copy().reshape(h.value, w.value, 4)
    finally:
        C.CDLL(None).free(out)


# zig-zag -> natural (decoder.zig:73-82)
_UNZIG = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14,
          21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53,
          60, 61, 54, 47, 55, 62, 63]


class Coefficients:
    """Host entropy stage output (pinned coefficient grids + frame descriptor).

    pieces=True: a baseline frame whose one scan interleaves Y, Cb, Cr keeps
    the compact ZPX_COEFFS_PIECES form (`frame.layout` 1: per-block index
    arrays in `coeffs`, the blocks' zig-zag pieces at `frame.pieces`); other
    frames decode into grids either way."""

    def __init__(self, data: bytes, pieces: bool = False):
        h = C.c_void_p()
        self._data = bytes(data)
        fn = _lib.lib().zpx_jpeg_entropy_decode_pieces if pieces else _lib.lib().zpx_jpeg_entropy_decode
        _lib.check(fn(self._data, len(self._data), C.byref(h)))
        self.handle = h
        self.frame = _lib.zpx_jpeg_frame()
        sizes = (C.c_size_t * 4)()
        _lib.check(_lib.lib().zpx_jpeg_coeffs_frame(h, C.byref(self.frame), sizes))
        self.coeff_bytes = [int(s) for s in sizes]

    @property
    def is_pieces(self) -> bool:
        return self.frame.layout == 1

    def pieces_bytes(self) -> np.ndarray:
        """The ZPX_COEFFS_PIECES frame's pieces (host view, uint8)."""
        n = int(self.frame.pieces_bytes)
        return np.ctypeslib.as_array(C.cast(self.frame.pieces, C.POINTER(C.c_uint8)), shape=(n,))

    def index(self, comp: int) -> np.ndarray:
        """The ZPX_COEFFS_PIECES index words of a component (host view, uint32)."""
        n = self.coeff_bytes[comp] // 4
        return np.ctypeslib.as_array(C.cast(self.frame.coeffs[comp], C.POINTER(C.c_uint32)), shape=(n,))

    def grid(self, comp: int) -> np.ndarray:
        """Coefficient grid of a component as (blocks, 64) int8/int16/int32 (host view; the
        frame's `coeff_bits` is the narrowest width that holds every coefficient).  A pieces
        frame's grid is expanded here (a copy)."""
        ptr = self.frame.coeffs[comp]
        if not ptr:
            return None
        if self.is_pieces:
            ix = self.index(comp)
            per = 16 if self.frame.coeff_bits == 8 else 8
            vals = self.pieces_bytes().view(np.int8 if self.frame.coeff_bits == 8 else np.int16)
            out = np.zeros((len(ix), 64), np.int8 if self.frame.coeff_bits == 8 else np.int16)
            zz = np.array(_UNZIG)
            for b, e in enumerate(ix):
                n, first = int(e) & 15, int(e) >> 4
                if n:
                    z = vals[first * per:first * per + min(64, n * per)]
                    out[b, zz[:len(z)]] = z
            return out
        ct = {8: C.c_int8, 16: C.c_int16, 32: C.c_int32}[self.frame.coeff_bits]
        n = self.coeff_bytes[comp] // C.sizeof(ct)
        return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(n,)).reshape(-1, 64)

    def widen(self, bits: int) -> "Coefficients":
        """Widen every grid to at least `bits` (16 or 32) coefficient bits."""
        _lib.check(_lib.lib().zpx_jpeg_coeffs_widen(self.handle, bits))
        sizes = (C.c_size_t * 4)()
        _lib.check(_lib.lib().zpx_jpeg_coeffs_frame(self.handle, C.byref(self.frame), sizes))
        self.coeff_bytes = [int(s) for s in sizes]
        return self

    def close(self):
        if self.handle:
            _lib.lib().zpx_jpeg_coeffs_free(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
