"""bmp module mirror (src/bmp/root.zig): load / load_from_buffer / decode /
probe_*.  The header is parsed on the host, the row loop runs as a HIP kernel."""
from __future__ import annotations

import ctypes as C

from . import _lib, context
from .image import Image


def decode(data: bytes, ctx: context.Context | None = None) -> Image:
    """bmp.decode (src/bmp/decoder.zig:25-40) over an in-memory buffer."""
    c = ctx or context.default()
    raw = _lib.zpx_image()
    _lib.check(_lib.lib().zpx_bmp_decode(c.handle, None, bytes(data), len(data), C.byref(raw)), c.handle)
    return Image._from_c(raw)


def load_from_buffer(data: bytes, ctx: context.Context | None = None) -> Image:
    """bmp.loadFromBuffer (src/bmp/root.zig:21-25)."""
    return decode(data, ctx)


def load(path: str, ctx: context.Context | None = None) -> Image:
    """bmp.load (src/bmp/root.zig:8-19)."""
    c = ctx or context.default()
    raw = _lib.zpx_image()
    _lib.check(_lib.lib().zpx_bmp_load(c.handle, None, path.encode(), C.byref(raw)), c.handle)
    return Image._from_c(raw)


def probe_buffer(data: bytes) -> bool:
    """bmp.probeBuffer (src/bmp/root.zig:28-31)."""
    return bool(_lib.lib().zpx_bmp_probe_buffer(bytes(data[:2]), min(len(data), 2)))


def probe_path(path: str) -> bool:
    """bmp.probePath (src/bmp/root.zig:34-45)."""
    with open(path, "rb") as f:
        return probe_buffer(f.read(2))
