"""image.Image mirror (src/image/image.zig:24-131).

An `Image` owns a host copy of the pixel buffer in the reference's layout
(RGBA/NRGBA/CMYK 4 B/px, RGBA64/NRGBA64 8 B/px big-endian, Gray 1, Gray16 2
BE, Paletted 1 + palette; YCbCr = padded planes in one buffer).  `rgba_pixels`
(Image.rgbaPixels, image.zig:103-130) runs on the GPU through the C-ABI.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib

KINDS = ["Gray", "Gray16", "YCbCr", "RGBA", "RGBA64", "NRGBA", "NRGBA64", "CMYK", "Paletted"]
SUBSAMPLES = ["Ratio444", "Ratio422", "Ratio420", "Ratio440", "Ratio411", "Ratio410"]


@dataclass(frozen=True)
class Rectangle:
    """geometry.Rectangle (src/image/geometry.zig:14-55)."""

    min_x: int
    min_y: int
    max_x: int
    max_y: int

    def dx(self) -> int:
        return self.max_x - self.min_x

    def dy(self) -> int:
        return self.max_y - self.min_y


@dataclass
class Image:
    kind: str
    rect: tuple
    pixels: np.ndarray
    stride: int = 0
    y_off: int = 0
    cb_off: int = 0
    cr_off: int = 0
    y_stride: int = 0
    c_stride: int = 0
    subsample: str = ""
    palette: list = field(default_factory=list)  # (r, g, b, a, model) model 0=.rgba 1=.nrgba

    # -- image.Image API
    def bounds(self) -> Rectangle:
        return Rectangle(*self.rect)

    @property
    def width(self) -> int:
        return self.rect[2] - self.rect[0]

    @property
    def height(self) -> int:
        return self.rect[3] - self.rect[1]

    def planes(self):
        """YCbCr y/cb/cr views (reference layout, padded strides)."""
        p = self.pixels
        return p[self.y_off:], p[self.cb_off:], p[self.cr_off:]

    def at(self, x: int, y: int):
        """Image.at(x, y): the concrete colour as (model, values) (image.zig:54-66)."""
        if not (self.rect[0] <= x < self.rect[2] and self.rect[1] <= y < self.rect[3]):
            return None
        dx, dy = x - self.rect[0], y - self.rect[1]
        k = self.kind
        if k == "YCbCr":
            sub = self.subsample
            cx = dx // 4 if sub in ("Ratio411", "Ratio410") else dx // 2 if sub in ("Ratio422", "Ratio420") else dx
            cy = dy // 2 if sub in ("Ratio420", "Ratio440", "Ratio410") else dy
            ci = cy * self.c_stride + cx
            return ("ycbcr", (int(self.pixels[self.y_off + dy * self.y_stride + dx]),
                              int(self.pixels[self.cb_off + ci]), int(self.pixels[self.cr_off + ci])))
        n = {"Gray": 1, "Gray16": 2, "RGBA": 4, "NRGBA": 4, "CMYK": 4, "RGBA64": 8, "NRGBA64": 8,
             "Paletted": 1}[k]
        s = self.pixels[dy * self.stride + dx * n:][:n]
        if k == "Gray":
            return ("gray", (int(s[0]),))
        if k == "Gray16":
            return ("gray16", ((int(s[0]) << 8) | int(s[1]),))
        if k in ("RGBA64", "NRGBA64"):
            return (k.lower(), tuple((int(s[2 * i]) << 8) | int(s[2 * i + 1]) for i in range(4)))
        if k == "Paletted":
            r, g, b, a, m = self.palette[int(s[0])]
            return ("rgba" if m == 0 else "nrgba", (r, g, b, a))
        return (k.lower(), tuple(int(v) for v in s))

    def rgba_pixels(self, ctx=None) -> np.ndarray:
        """Image.rgbaPixels on the GPU: 8-bit RGBA, 4*dX*dY bytes."""
        from . import context

        c = ctx or context.default()
        raw = self._to_c()
        out = C.POINTER(C.c_uint8)()
        n = C.c_size_t(0)
        _lib.check(_lib.lib().zpx_image_rgba_pixels(c.handle, None, C.byref(raw), C.byref(out), C.byref(n)),
                   c.handle)
        try:
            return np.ctypeslib.as_array(out, shape=(n.value,)).copy() if n.value else np.zeros(0, np.uint8)
        finally:
            C.CDLL(None).free(out)

    def free(self) -> None:
        """Image.free: host memory is owned by numpy here; kept for API parity."""
        self.pixels = np.zeros(0, np.uint8)

    # -- C interop
    def _to_c(self) -> _lib.zpx_image:
        raw = _lib.zpx_image()
        raw.kind = KINDS.index(self.kind)
        raw.min_x, raw.min_y, raw.max_x, raw.max_y = self.rect
        self._keep_px = np.ascontiguousarray(self.pixels, np.uint8)
        raw.pixels = self._keep_px.ctypes.data_as(C.POINTER(C.c_uint8))
        raw.pixels_len = self._keep_px.size
        raw.stride = self.stride
        raw.y_off, raw.cb_off, raw.cr_off = self.y_off, self.cb_off, self.cr_off
        raw.y_stride, raw.c_stride = self.y_stride, self.c_stride
        raw.subsample = SUBSAMPLES.index(self.subsample) if self.subsample else 0
        if self.kind == "Paletted":
            pal = (_lib.zpx_color * 256)()
            for i, (r, g, b, a, m) in enumerate(self.palette):
                pal[i].r, pal[i].g, pal[i].b, pal[i].a, pal[i].model = r, g, b, a, m
            self._keep_pal = pal
            raw.palette = C.cast(pal, C.POINTER(_lib.zpx_color))
            raw.palette_len = len(self.palette)
        return raw

    @classmethod
    def _from_c(cls, raw: _lib.zpx_image) -> "Image":
        """Copy a library-owned zpx_image into numpy and free the C buffers."""
        n = raw.pixels_len
        px = np.ctypeslib.as_array(raw.pixels, shape=(n,)).copy() if n else np.zeros(0, np.uint8)
        pal = []
        if raw.kind == 8 and raw.palette:
            for i in range(raw.palette_len):
                c = raw.palette[i]
                pal.append((c.r, c.g, c.b, c.a, c.model))
        img = cls(
            kind=KINDS[raw.kind],
            rect=(raw.min_x, raw.min_y, raw.max_x, raw.max_y),
            pixels=px,
            stride=raw.stride,
            y_off=raw.y_off,
            cb_off=raw.cb_off,
            cr_off=raw.cr_off,
            y_stride=raw.y_stride,
            c_stride=raw.c_stride,
            subsample=SUBSAMPLES[raw.subsample] if raw.kind == 2 else "",
            palette=pal,
        )
        _lib.lib().zpx_image_free(None, C.byref(raw))
        return img
