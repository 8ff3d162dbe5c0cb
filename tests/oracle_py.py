"""ctypes binding of the CPU parity oracle (oracle/zpix_oracle.c).

Test infrastructure only: used by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the *checker*; never by the product.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "libzpix_oracle.so")

KIND_NAMES = ["Gray", "Gray16", "YCbCr", "RGBA", "RGBA64", "NRGBA", "NRGBA64", "CMYK", "Paletted"]
SUBSAMPLE_NAMES = ["Ratio444", "Ratio422", "Ratio420", "Ratio440", "Ratio411", "Ratio410"]


class ZoImage(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("min_x", C.c_int32),
        ("min_y", C.c_int32),
        ("max_x", C.c_int32),
        ("max_y", C.c_int32),
        ("pixels", C.POINTER(C.c_uint8)),
        ("pixels_len", C.c_size_t),
        ("stride", C.c_size_t),
        ("y_off", C.c_size_t),
        ("cb_off", C.c_size_t),
        ("cr_off", C.c_size_t),
        ("y_stride", C.c_size_t),
        ("c_stride", C.c_size_t),
        ("subsample", C.c_int32),
        ("palette", C.POINTER(C.c_uint8)),
        ("palette_len", C.c_int32),
    ]


class ZoJpegCoeffs(C.Structure):
    _fields_ = [
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("n_comp", C.c_int32),
        ("h", C.c_int32 * 4),
        ("v", C.c_int32 * 4),
        ("tq", C.c_int32 * 4),
        ("mxx", C.c_int32),
        ("myy", C.c_int32),
        ("progressive", C.c_int32),
        ("jfif", C.c_int32),
        ("adobe_valid", C.c_int32),
        ("adobe_transform", C.c_int32),
        ("comp_id", C.c_int32 * 4),
        ("grid", C.POINTER(C.c_int32) * 4),
        ("quant", (C.c_int32 * 64) * 4),
    ]


_lib = None


def build_oracle() -> None:
    import subprocess

    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build_oracle()
        L = C.CDLL(ORACLE_SO)
        L.zo_error_name.restype = C.c_char_p
        L.zo_error_name.argtypes = [C.c_int]
        for fn in (L.zo_jpeg_decode, L.zo_png_decode, L.zo_bmp_decode, L.zo_qoi_decode):
            fn.restype = C.c_int
            fn.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(ZoImage)]
        L.zo_rgba_pixels.restype = C.c_int
        L.zo_rgba_pixels.argtypes = [C.POINTER(ZoImage), C.c_void_p]
        L.zo_image_free.argtypes = [C.POINTER(ZoImage)]
        L.zo_idct.argtypes = [C.c_void_p]
        L.zo_jpeg_decode_coeffs.restype = C.c_int
        L.zo_jpeg_decode_coeffs.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(ZoJpegCoeffs)]
        L.zo_jpeg_coeffs_free.argtypes = [C.POINTER(ZoJpegCoeffs)]
        L.zo_png_unfilter.restype = C.c_int
        L.zo_png_unfilter.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
        L.zo_jpeg_reconstruct_grids.argtypes = [
            C.c_int32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32,
            C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
        ]
        L.zo_qoi_encode.restype = C.c_int
        L.zo_qoi_encode.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint8, C.c_uint8,
                                    C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_size_t)]
        L.free.argtypes = [C.c_void_p]
        L.zo_png_unfilter_seconds.restype = C.c_double
        L.zo_png_unfilter_seconds.argtypes = []
        _lib = L
    return _lib


class OracleError(Exception):
    def __init__(self, name: str):
        super().__init__(name)
        self.name = name


@dataclass
class OImage:
    """A host copy of an oracle image.Image (kind + rect + pixel buffer)."""

    kind: str
    rect: tuple  # (min_x, min_y, max_x, max_y)
    pixels: np.ndarray
    stride: int = 0
    y_off: int = 0
    cb_off: int = 0
    cr_off: int = 0
    y_stride: int = 0
    c_stride: int = 0
    subsample: str = ""
    palette: list = field(default_factory=list)  # (r,g,b,a,tag) tag 0=.rgba 1=.nrgba
    _raw: object = None

    @property
    def width(self):
        return self.rect[2] - self.rect[0]

    @property
    def height(self):
        return self.rect[3] - self.rect[1]

    def rgba_pixels(self) -> np.ndarray:
        """Image.rgbaPixels through the oracle."""
        out = np.zeros(self.width * self.height * 4, np.uint8)
        lib().zo_rgba_pixels(C.byref(self._raw), out.ctypes.data)
        return out

    def planes(self):
        """YCbCr planes as (y, cb, cr) flat views, reference layout."""
        p = self.pixels
        return p[self.y_off:], p[self.cb_off:], p[self.cr_off:]


def _wrap(raw: ZoImage) -> OImage:
    n = raw.pixels_len
    px = np.ctypeslib.as_array(raw.pixels, shape=(n,)).copy() if n else np.zeros(0, np.uint8)
    pal = []
    if raw.palette_len > 0 and raw.palette:
        p = np.ctypeslib.as_array(raw.palette, shape=(256 * 5,)).reshape(256, 5)
        pal = [tuple(int(x) for x in p[i]) for i in range(raw.palette_len)]
    img = OImage(
        kind=KIND_NAMES[raw.kind],
        rect=(raw.min_x, raw.min_y, raw.max_x, raw.max_y),
        pixels=px,
        stride=raw.stride,
        y_off=raw.y_off,
        cb_off=raw.cb_off,
        cr_off=raw.cr_off,
        y_stride=raw.y_stride,
        c_stride=raw.c_stride,
        subsample=SUBSAMPLE_NAMES[raw.subsample] if raw.kind == 2 else "",
        palette=pal,
    )
    # keep a private C copy alive for rgba_pixels(); point it at our numpy buffer
    keep = ZoImage()
    C.pointer(keep)[0] = raw
    img._px_keep = px  # type: ignore[attr-defined]
    keep.pixels = px.ctypes.data_as(C.POINTER(C.c_uint8))
    if raw.palette_len > 0 and raw.palette:
        palbuf = np.ctypeslib.as_array(raw.palette, shape=(256 * 5,)).copy()
        img._pal_keep = palbuf  # type: ignore[attr-defined]
        keep.palette = palbuf.ctypes.data_as(C.POINTER(C.c_uint8))
    img._raw = keep
    lib().zo_image_free(C.byref(raw))
    return img


def error_name(code: int) -> str:
    return lib().zo_error_name(code).decode()


def jpeg_decode(data: bytes) -> OImage:
    raw = ZoImage()
    e = lib().zo_jpeg_decode(data, len(data), C.byref(raw))
    if e:
        raise OracleError(error_name(e))
    return _wrap(raw)


def png_decode(data: bytes) -> OImage:
    raw = ZoImage()
    e = lib().zo_png_decode(data, len(data), C.byref(raw))
    if e:
        raise OracleError(error_name(e))
    return _wrap(raw)


def bmp_decode(data: bytes) -> OImage:
    raw = ZoImage()
    e = lib().zo_bmp_decode(data, len(data), C.byref(raw))
    if e:
        raise OracleError(error_name(e))
    return _wrap(raw)


def qoi_decode(data: bytes) -> OImage:
    raw = ZoImage()
    e = lib().zo_qoi_decode(data, len(data), C.byref(raw))
    if e:
        raise OracleError(error_name(e))
    return _wrap(raw)


def qoi_encode(pixels, width: int, height: int, channels: int, colorspace: int = 0) -> bytes:
    """qoi.encode (src/qoi/encoder.zig:29-132) through the oracle."""
    px = np.ascontiguousarray(np.asarray(pixels, np.uint8).reshape(-1))
    out = C.POINTER(C.c_uint8)()
    n = C.c_size_t(0)
    e = lib().zo_qoi_encode(px.ctypes.data if px.size else None, width, height, channels, colorspace,
                            C.byref(out), C.byref(n))
    if e:
        raise OracleError(error_name(e))
    try:
        return C.string_at(out, n.value)
    finally:
        lib().free(out)


def decode(data: bytes) -> OImage:
    """zpix.fromBuffer (src/root.zig:34-40): PNG, JPEG, QOI, BMP in that order."""
    if data[:8] == b"\x89PNG\r\n\x1a\n":
        return png_decode(data)
    if data[:2] == b"\xff\xd8":
        return jpeg_decode(data)
    if data[:4] == b"qoif":
        return qoi_decode(data)
    if data[:2] == b"BM":
        return bmp_decode(data)
    raise OracleError("UnknownImageFormat")


def idct(block) -> np.ndarray:
    b = np.ascontiguousarray(np.asarray(block, np.int32).reshape(64)).copy()
    lib().zo_idct(b.ctypes.data)
    return b


@dataclass
class JpegCoeffs:
    width: int
    height: int
    n_comp: int
    h: list
    v: list
    tq: list
    mxx: int
    myy: int
    progressive: bool
    grids: list  # per component: int32 array (nblocks, 64) natural order, or None
    quant_zigzag: np.ndarray  # (4, 64) int32
    comp_id: list
    jfif: bool
    adobe_valid: bool
    adobe_transform: int


def jpeg_coefficients(data: bytes) -> JpegCoeffs:
    raw = ZoJpegCoeffs()
    e = lib().zo_jpeg_decode_coeffs(data, len(data), C.byref(raw))
    if e:
        raise OracleError(error_name(e))
    grids = []
    for c in range(raw.n_comp):
        if raw.grid[c]:
            nb = raw.mxx * raw.myy * raw.h[c] * raw.v[c]
            grids.append(np.ctypeslib.as_array(raw.grid[c], shape=(nb * 64,)).reshape(nb, 64).copy())
        else:
            grids.append(None)
    out = JpegCoeffs(
        width=raw.width, height=raw.height, n_comp=raw.n_comp,
        h=list(raw.h), v=list(raw.v), tq=list(raw.tq), mxx=raw.mxx, myy=raw.myy,
        progressive=bool(raw.progressive), grids=grids,
        quant_zigzag=np.array([[raw.quant[t][i] for i in range(64)] for t in range(4)], np.int32),
        comp_id=list(raw.comp_id), jfif=bool(raw.jfif), adobe_valid=bool(raw.adobe_valid),
        adobe_transform=raw.adobe_transform,
    )
    lib().zo_jpeg_coeffs_free(C.byref(raw))
    return out


def reconstruct_grids(n_comp, width, height, h, v, mxx, myy, grids, qts_zigzag, progressive,
                      planes, strides, timing: list | None = None):
    """zo_jpeg_reconstruct_grids: grids are int32 (nblocks,64) arrays (copied; mutated in C).
    timing: if given, the C call's wall seconds are appended (CPU-baseline stage split)."""
    import time

    gcopies = [np.ascontiguousarray(g, np.int32).copy() if g is not None else None for g in grids]
    gptrs = (C.c_void_p * 4)(*[g.ctypes.data if g is not None else None for g in gcopies] + [None] * (4 - len(gcopies)))
    qcopies = [np.ascontiguousarray(q, np.int32) for q in qts_zigzag]
    qptrs = (C.c_void_p * 4)(*[q.ctypes.data for q in qcopies] + [None] * (4 - len(qcopies)))
    pptrs = (C.c_void_p * 4)(*[p.ctypes.data for p in planes] + [None] * (4 - len(planes)))
    harr = (C.c_int32 * 4)(*h[:4])
    varr = (C.c_int32 * 4)(*v[:4])
    sarr = (C.c_size_t * 4)(*list(strides) + [0] * (4 - len(strides)))
    t0 = time.perf_counter()
    lib().zo_jpeg_reconstruct_grids(n_comp, width, height, C.addressof(harr), C.addressof(varr),
                                    mxx, myy, C.addressof(gptrs), C.addressof(qptrs),
                                    int(progressive), C.addressof(pptrs), C.addressof(sarr))
    if timing is not None:
        timing.append(time.perf_counter() - t0)


def png_unfilter(filtered: np.ndarray, rows: int, row_bytes: int, bpp: int) -> np.ndarray:
    out = np.zeros(rows * row_bytes, np.uint8)
    f = np.ascontiguousarray(filtered, np.uint8)
    e = lib().zo_png_unfilter(f.ctypes.data, rows, row_bytes, bpp, out.ctypes.data)
    if e:
        raise OracleError(error_name(e))
    return out


def png_unfilter_seconds() -> float:
    """Seconds this thread spent in PNG unfilter + pixel store since the last call (CPU-baseline stage split)."""
    return float(lib().zo_png_unfilter_seconds())
