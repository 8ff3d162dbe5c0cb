"""zpix_amd — MI355X (gfx950) decode path for braheezy/zpix's JPEG/PNG pixel loops.

Mirrors the reference API (src/root.zig, src/jpeg/root.zig, src/png/root.zig,
src/image/image.zig): `from_file_path`, `from_buffer`, `jpeg.load`,
`png.load`, `bmp.load`, `qoi.load` / `qoi.encode`, `Image.rgba_pixels`.  Entropy decoding (Huffman, zlib) runs on the
host inside libzpix_amd.so; dequant/IDCT/colour and PNG unfilter/store run as
HIP kernels.  Device-resident batch plans live in `zpix_amd.device`.
"""
from __future__ import annotations

import ctypes as C

from . import _lib, batch, bmp, context, jpeg, png, qoi
from ._lib import ZpixError
from .context import Context
from .image import Image, Rectangle

__all__ = ["ZpixError", "Context", "Image", "Rectangle", "jpeg", "png", "bmp", "qoi", "from_buffer",
           "from_file_path"]


def from_buffer(data: bytes, ctx: Context | None = None) -> Image:
    """zpix.fromBuffer (src/root.zig:34-40): probes PNG, JPEG, QOI, BMP."""
    c = ctx or context.default()
    raw = _lib.zpx_image()
    _lib.check(_lib.lib().zpx_from_buffer(c.handle, None, bytes(data), len(data), C.byref(raw)), c.handle)
    return Image._from_c(raw)


def from_file_path(path: str, ctx: Context | None = None) -> Image:
    """zpix.fromFilePath (src/root.zig:24-31)."""
    c = ctx or context.default()
    raw = _lib.zpx_image()
    _lib.check(_lib.lib().zpx_from_file_path(c.handle, None, path.encode(), C.byref(raw)), c.handle)
    return Image._from_c(raw)
