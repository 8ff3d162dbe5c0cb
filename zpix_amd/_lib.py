"""ctypes binding of libzpix_amd.so (the C-ABI in include/zpix_amd.h).

The shared library is built in-tree (zpix_amd/libzpix_amd.so) by
`__graft_entry__.build()` / `make -C zpix_amd/csrc`.  If it is missing this
module raises: there is no Python or CPU fallback for the pixel path.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# ZPX_LIB_PATH: an alternative build of the same library (kernel A/B experiments)
LIB_PATH = os.environ.get("ZPX_LIB_PATH") or os.path.join(HERE, "libzpix_amd.so")

# one HIP runtime per process: if torch is importable, let it load its
# libamdhip64 first so device pointers from torch tensors and from this
# library share the runtime (same SONAME, so ours resolves to the loaded one).
try:  # pragma: no cover - import side effect only
    import torch  # noqa: F401
except Exception:  # torch is plumbing, not required for the C-ABI itself
    torch = None


class ZpixError(Exception):
    """A decode error carrying the reference's Zig error name (e.g. 'UnexpectedEof')."""

    def __init__(self, name: str, detail: str = ""):
        super().__init__(name if not detail else f"{name}: {detail}")
        self.name = name
        self.detail = detail


class zpx_color(C.Structure):
    _fields_ = [("r", C.c_uint8), ("g", C.c_uint8), ("b", C.c_uint8), ("a", C.c_uint8),
                ("model", C.c_uint8), ("pad", C.c_uint8 * 3)]


class zpx_image(C.Structure):
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
        ("palette", C.POINTER(zpx_color)),
        ("palette_len", C.c_int32),
    ]


class zpx_jpeg_frame(C.Structure):
    _fields_ = [
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("n_comp", C.c_int32),
        ("h", C.c_int32 * 4),
        ("v", C.c_int32 * 4),
        ("mxx", C.c_int32),
        ("myy", C.c_int32),
        ("rule", C.c_int32 * 4),
        ("coeff_bits", C.c_int32),
        ("narrow", C.c_int32),
        ("color", C.c_int32),
        ("coeffs", C.c_void_p * 4),
        ("qt", (C.c_int32 * 64) * 4),
        ("planes", C.c_void_p * 4),
        ("strides", C.c_size_t * 4),
        ("rgba", C.c_void_p),
        ("rgba_stride", C.c_size_t),
        ("layout", C.c_int32),
        ("pieces", C.c_void_p),
        ("pieces_bytes", C.c_size_t),
    ]


class zpx_png_frame(C.Structure):
    _fields_ = [
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("depth", C.c_int32),
        ("interlace", C.c_int32),
        ("use_transparent", C.c_int32),
        ("transparent", C.c_uint8 * 6),
        ("layout", C.c_uint8),  # zpx_png_layout: 0 stream, 1 band slab
        ("pad", C.c_uint8),
        ("filtered", C.c_void_p),
        ("out", C.c_void_p),
        ("out_stride", C.c_size_t),
        ("max_index", C.c_void_p),
    ]


class zpx_batch_item(C.Structure):
    _fields_ = [
        ("buf", C.c_void_p),
        ("len", C.c_size_t),
        ("dst", C.c_void_p),
        ("dst_stride", C.c_size_t),
        ("dst_capacity", C.c_size_t),
        ("status", C.c_int32),
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("format", C.c_int32),
    ]


class zpx_batch_opts(C.Structure):
    _fields_ = [("host_threads", C.c_int32), ("depth", C.c_int32), ("dst_on_host", C.c_int32)]


class zpx_batch_stats(C.Structure):
    _fields_ = [
        ("wall_s", C.c_double),
        ("host_s", C.c_double),
        ("h2d_bytes", C.c_double),
        ("d2h_bytes", C.c_double),
        ("pixels", C.c_double),
        ("host_threads", C.c_int32),
        ("depth", C.c_int32),
        ("failed", C.c_int32),
        ("pad", C.c_int32),
        ("host_jpeg_s", C.c_double),
        ("host_png_s", C.c_double),
        ("jpeg_items", C.c_int32),
        ("png_items", C.c_int32),
    ]


class zpx_qoi_desc(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("channels", C.c_uint8), ("colorspace", C.c_uint8),
                ("pad", C.c_uint8 * 2)]


class zpx_gather_stats(C.Structure):
    _fields_ = [("decode_s", C.c_double), ("gather_s", C.c_double), ("gather_bytes", C.c_double),
                ("ndev", C.c_int32), ("pad", C.c_int32), ("tail_s", C.c_double), ("comm_setup_s", C.c_double),
                ("comm_ranks", C.c_int32), ("pad2", C.c_int32)]


# every symbol include/zpix_amd.h declares (checked by tests/test_abi.py)
# ZPX_ABI_VERSION of include/zpix_amd.h that the structs below mirror
ABI_VERSION = 2

EXPORTS = [
    "zpx_abi_version", "zpx_error_name", "zpx_last_error", "zpx_ctx_create", "zpx_ctx_destroy", "zpx_ctx_stream",
    "zpx_ctx_device", "zpx_ctx_synchronize", "zpx_image_free", "zpx_image_rgba_pixels",
    "zpx_jpeg_decode", "zpx_jpeg_load", "zpx_jpeg_probe_buffer", "zpx_jpeg_decode_rgba",
    "zpx_png_decode", "zpx_png_load", "zpx_png_probe_buffer", "zpx_from_buffer", "zpx_from_file_path",
    "zpx_jpeg_plan_create", "zpx_png_plan_create", "zpx_plan_launch", "zpx_plan_bytes",
    "zpx_plan_kernel_count", "zpx_plan_destroy", "zpx_dev_rgba_pixels", "zpx_rgba_plan_create", "zpx_jpeg_entropy_decode", "zpx_jpeg_entropy_decode_pieces",
    "zpx_jpeg_coeffs_frame", "zpx_jpeg_coeffs_free", "zpx_jpeg_coeffs_widen", "zpx_png_inflate", "zpx_png_stream_frame",
    "zpx_png_stream_data", "zpx_png_stream_slab", "zpx_png_stream_free", "zpx_batch_decode_rgba", "zpx_batch_start",
    "zpx_batch_wait", "zpx_jpeg_decode_config", "zpx_png_decode_config", "zpx_plan_status",
    "zpx_batch_decode_sharded", "zpx_debug_png_stall", "zpx_debug_jpeg_parallel_scans", "zpx_debug_png_device_slab",
    "zpx_debug_jpeg_parallel_progressive",
    "zpx_bmp_decode", "zpx_bmp_load", "zpx_bmp_probe_buffer", "zpx_qoi_decode", "zpx_qoi_load",
    "zpx_qoi_probe_buffer", "zpx_qoi_encode", "zpx_qoi_encode_bound", "zpx_qoi_encode_device",
    "zpx_debug_jpeg_sparse_grids", "zpx_debug_inflate_parallel", "zpx_debug_png_inflate_pair", "zpx_batch_wait_prefix",
    "zpx_debug_shard_fake_comm", "zpx_debug_option", "zpx_host_pools_trim",
    "zpx_batch_cache_trim",
]

_lib = None


def lib():
    """Load libzpix_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    vp, i32, sz, u8p = C.c_void_p, C.c_int, C.c_size_t, C.POINTER(C.c_uint8)
    sig = {
        "zpx_abi_version": (i32, []),
        "zpx_host_pools_trim": (sz, []),
        "zpx_batch_cache_trim": (sz, []),
        "zpx_error_name": (C.c_char_p, [i32]),
        "zpx_last_error": (C.c_char_p, [vp]),
        "zpx_ctx_create": (i32, [i32, C.POINTER(vp)]),
        "zpx_ctx_destroy": (None, [vp]),
        "zpx_ctx_stream": (vp, [vp]),
        "zpx_ctx_device": (i32, [vp]),
        "zpx_ctx_synchronize": (i32, [vp]),
        "zpx_image_free": (None, [vp, C.POINTER(zpx_image)]),
        "zpx_image_rgba_pixels": (i32, [vp, vp, C.POINTER(zpx_image), C.POINTER(u8p), C.POINTER(sz)]),
        "zpx_jpeg_decode": (i32, [vp, vp, C.c_char_p, sz, C.POINTER(zpx_image)]),
        "zpx_jpeg_load": (i32, [vp, vp, C.c_char_p, C.POINTER(zpx_image)]),
        "zpx_jpeg_probe_buffer": (i32, [C.c_char_p, sz]),
        "zpx_jpeg_decode_rgba": (i32, [vp, vp, C.c_char_p, sz, C.POINTER(u8p), C.POINTER(sz),
                                       C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
        "zpx_png_decode": (i32, [vp, vp, C.c_char_p, sz, C.POINTER(zpx_image)]),
        "zpx_png_load": (i32, [vp, vp, C.c_char_p, C.POINTER(zpx_image)]),
        "zpx_png_probe_buffer": (i32, [C.c_char_p, sz]),
        "zpx_from_buffer": (i32, [vp, vp, C.c_char_p, sz, C.POINTER(zpx_image)]),
        "zpx_from_file_path": (i32, [vp, vp, C.c_char_p, C.POINTER(zpx_image)]),
        "zpx_jpeg_plan_create": (i32, [vp, C.POINTER(zpx_jpeg_frame), i32, i32, C.POINTER(vp)]),
        "zpx_png_plan_create": (i32, [vp, C.POINTER(zpx_png_frame), i32, C.POINTER(vp)]),
        "zpx_plan_launch": (i32, [vp, vp]),
        "zpx_plan_bytes": (C.c_uint64, [vp]),
        "zpx_plan_kernel_count": (i32, [vp]),
        "zpx_plan_destroy": (None, [vp]),
        "zpx_dev_rgba_pixels": (i32, [vp, C.POINTER(zpx_image), vp, vp]),
        "zpx_rgba_plan_create": (i32, [vp, C.POINTER(zpx_image), C.POINTER(vp), i32, C.POINTER(vp)]),
        "zpx_jpeg_entropy_decode": (i32, [C.c_char_p, sz, C.POINTER(vp)]),
        "zpx_jpeg_entropy_decode_pieces": (i32, [C.c_char_p, sz, C.POINTER(vp)]),
        "zpx_jpeg_coeffs_frame": (i32, [vp, C.POINTER(zpx_jpeg_frame), C.POINTER(sz)]),
        "zpx_jpeg_coeffs_free": (None, [vp]),
        "zpx_jpeg_coeffs_widen": (i32, [vp, i32]),
        "zpx_png_inflate": (i32, [C.c_char_p, sz, C.POINTER(vp)]),
        "zpx_png_stream_frame": (i32, [vp, C.POINTER(zpx_png_frame), C.POINTER(sz)]),
        "zpx_png_stream_data": (vp, [vp]),
        "zpx_png_stream_slab": (i32, [vp, C.POINTER(vp), C.POINTER(sz)]),
        "zpx_png_stream_free": (None, [vp]),
        "zpx_batch_decode_rgba": (i32, [vp, C.POINTER(zpx_batch_item), i32, C.POINTER(zpx_batch_opts),
                                        C.POINTER(zpx_batch_stats)]),
        "zpx_batch_start": (i32, [vp, C.POINTER(zpx_batch_item), i32, C.POINTER(zpx_batch_opts), C.POINTER(vp)]),
        "zpx_batch_wait": (i32, [vp, C.POINTER(zpx_batch_stats)]),
        "zpx_batch_wait_prefix": (i32, [vp, i32]),
        "zpx_debug_shard_fake_comm": (i32, [i32]),
        "zpx_debug_option": (i32, [C.c_char_p, i32]),
        "zpx_jpeg_decode_config": (i32, [C.c_char_p, sz, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                         C.POINTER(C.c_int32)]),
        "zpx_png_decode_config": (i32, [C.c_char_p, sz, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
        "zpx_plan_status": (i32, [vp, vp]),
        "zpx_batch_decode_sharded": (i32, [C.POINTER(vp), i32, C.POINTER(zpx_batch_item), i32,
                                           C.POINTER(zpx_batch_opts), C.POINTER(zpx_batch_stats),
                                           C.POINTER(zpx_gather_stats)]),
        "zpx_debug_png_stall": (i32, [vp, C.c_uint32, C.POINTER(C.c_double)]),
        "zpx_debug_png_device_slab": (i32, [vp, vp, vp, sz, C.POINTER(sz)]),
        "zpx_debug_jpeg_parallel_scans": (C.c_int64, []),
        "zpx_debug_jpeg_parallel_progressive": (C.c_int64, []),
        "zpx_bmp_decode": (i32, [vp, vp, C.c_char_p, sz, C.POINTER(zpx_image)]),
        "zpx_bmp_load": (i32, [vp, vp, C.c_char_p, C.POINTER(zpx_image)]),
        "zpx_bmp_probe_buffer": (i32, [C.c_char_p, sz]),
        "zpx_qoi_decode": (i32, [vp, vp, C.c_char_p, sz, C.POINTER(zpx_image)]),
        "zpx_qoi_load": (i32, [vp, vp, C.c_char_p, C.POINTER(zpx_image)]),
        "zpx_qoi_probe_buffer": (i32, [C.c_char_p, sz]),
        "zpx_qoi_encode": (i32, [vp, vp, vp, sz, C.POINTER(zpx_qoi_desc), C.POINTER(u8p), C.POINTER(sz)]),
        "zpx_qoi_encode_bound": (sz, [C.POINTER(zpx_qoi_desc)]),
        "zpx_qoi_encode_device": (i32, [vp, vp, C.POINTER(zpx_qoi_desc), vp, sz, vp, vp]),
        "zpx_debug_jpeg_sparse_grids": (C.c_int64, [C.c_char_p, sz, vp, sz]),
        "zpx_debug_inflate_parallel": (i32, [C.c_char_p, sz, vp, sz, i32]),
        "zpx_debug_png_inflate_pair": (i32, [C.c_char_p, sz, C.c_char_p, sz, C.POINTER(vp), C.POINTER(vp),
                                             C.POINTER(i32)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.zpx_abi_version() != ABI_VERSION:
        raise ImportError(f"{LIB_PATH} is ABI version {L.zpx_abi_version()}; this binding mirrors {ABI_VERSION}")
    _lib = L
    return L


def libc_free(p) -> None:
    """free() for buffers the library returned from the default (NULL) allocator."""
    C.CDLL(None).free(C.cast(p, C.c_void_p))


def error_name(code: int) -> str:
    return lib().zpx_error_name(code).decode()


def check(code: int, ctx=None) -> None:
    if code:
        detail = ""
        if ctx is not None:
            detail = (lib().zpx_last_error(ctx) or b"").decode()
        raise ZpixError(error_name(code), detail)
