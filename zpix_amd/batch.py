"""Batch / streaming decode: many encoded JPEG/PNG buffers -> RGBA8.

Thin mirror of `zpx_batch_decode_rgba` (include/zpix_amd.h).  Per image the
result equals `zpix.fromBuffer(buf)` followed by `img.rgbaPixels()`
(src/root.zig:34-40, src/image/image.zig:103-130).  Host entropy decoding runs
on a native thread pool inside libzpix_amd.so, overlapped with pinned H2D
copies and the kernels; nothing here is on the per-pixel path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

from . import _lib, context


@dataclass
class BatchResult:
    status: str          # "Ok" or the reference's error name for this image
    width: int
    height: int
    format: str          # "jpeg", "png" or "unknown"
    rgba: object = None  # torch uint8 tensor (H, W, 4) on the device, or numpy on the host


@dataclass
class BatchStats:
    wall_s: float
    host_s: float
    h2d_bytes: float
    d2h_bytes: float
    pixels: float
    host_threads: int
    depth: int
    failed: int
    host_jpeg_s: float = 0.0  # host_s split by stage: JPEG entropy decode
    host_png_s: float = 0.0   # PNG chunk walk + inflate
    jpeg_items: int = 0
    png_items: int = 0

    @property
    def mpix_s(self) -> float:
        return self.pixels / self.wall_s / 1e6 if self.wall_s > 0 else 0.0


def _probe_dims(data: bytes):
    """Width/height from the header, to size each destination (decodeConfig)."""
    from .jpeg import decode_config as jcfg
    from .png import decode_config as pcfg

    try:
        if data[:8] == b"\x89PNG\r\n\x1a\n":
            return pcfg(data)
        if data[:2] == b"\xff\xd8":
            return jcfg(data)
    except _lib.ZpixError:
        pass  # the batch reports the image's own error
    return None


def _bind(buffers, on_host: bool, c, dst):
    """The zpx_batch_item array for `buffers` and the destinations it points at."""
    import numpy as np

    n = len(buffers)
    items = (_lib.zpx_batch_item * max(1, n))()
    keep = [bytes(b) for b in buffers]
    outs = []
    for i, b in enumerate(keep):
        dims = _probe_dims(b) if dst is None else None
        it = items[i]
        it.buf = C.cast(C.c_char_p(b), C.c_void_p)
        it.len = len(b)
        if dst is not None:
            t = dst[i]
            outs.append(t)
            if t is None:
                it.dst = None
                it.dst_capacity = 0
            else:
                it.dst = t.data_ptr() if hasattr(t, "data_ptr") else t.ctypes.data
                it.dst_capacity = t.numel() if hasattr(t, "numel") else t.nbytes
            it.dst_stride = 0
            continue
        if dims is None:
            outs.append(None)
            it.dst = None
            it.dst_capacity = 0
            continue
        w, h = dims
        if on_host:
            arr = np.zeros((h, w, 4), np.uint8)
            outs.append(arr)
            it.dst = arr.ctypes.data
        else:
            import torch

            t = torch.empty((h, w, 4), dtype=torch.uint8, device=f"cuda:{c.device}")
            outs.append(t)
            it.dst = t.data_ptr()
        it.dst_capacity = w * h * 4
        it.dst_stride = 0
    if not on_host:
        import torch

        torch.cuda.synchronize(c.device)  # destinations allocated on torch's stream
    return items, keep, outs


def _results(items, outs, n):
    res = []
    fmt = {1: "jpeg", 2: "png"}
    for i in range(n):
        it = items[i]
        ok = it.status == 0
        res.append(BatchResult(_lib.error_name(it.status), it.width, it.height, fmt.get(it.format, "unknown"),
                               outs[i] if ok else None))
    return res


def _stats(st) -> BatchStats:
    return BatchStats(st.wall_s, st.host_s, st.h2d_bytes, st.d2h_bytes, st.pixels, st.host_threads, st.depth,
                      st.failed, st.host_jpeg_s, st.host_png_s, st.jpeg_items, st.png_items)


def decode_rgba(buffers, on_host: bool = False, host_threads: int = 0, depth: int = 0, ctx=None,
                dst=None, with_stats: bool = False):
    """Decodes every buffer to RGBA8.

    on_host=False: results are torch uint8 tensors (H, W, 4) on the context's
    device (or the caller's `dst` tensors / device buffers); True: numpy arrays.
    Images that fail carry their error name in `status` and no pixels."""
    c = ctx or context.default()
    n = len(buffers)
    items, keep, outs = _bind(buffers, on_host, c, dst)
    opts = _lib.zpx_batch_opts(host_threads, depth, 1 if on_host else 0)
    st = _lib.zpx_batch_stats()
    _lib.check(_lib.lib().zpx_batch_decode_rgba(c.handle, items, n, C.byref(opts), C.byref(st)), c.handle)
    res = _results(items, outs, n)
    return (res, _stats(st)) if with_stats else res


class Running:
    """A batch started with start_rgba: its pipeline runs on a native thread.
    wait(n) blocks until images 0..n-1 are final (zpx_batch_wait_prefix: their
    RGBA is complete in dst), so finished results can move on while later
    images still decode; finish() joins and returns (results, stats)."""

    def __init__(self, handle, items, keep, outs, n, ctx):
        self._h, self._items, self._keep, self._outs, self._n, self._ctx = handle, items, keep, outs, n, ctx

    def wait(self, n: int) -> int:
        if self._h is None:
            return self._n
        return _lib.lib().zpx_batch_wait_prefix(self._h, n)

    def statuses(self, lo: int, hi: int) -> list:
        """Error names of images lo..hi-1 (final once wait(hi) returned >= hi)."""
        return [_lib.error_name(self._items[i].status) for i in range(lo, hi)]

    def finish(self):
        st = _lib.zpx_batch_stats()
        h, self._h = self._h, None
        if h is not None:
            _lib.check(_lib.lib().zpx_batch_wait(h, C.byref(st)), self._ctx.handle)
        return _results(self._items, self._outs, self._n), _stats(st)


def start_rgba(buffers, host_threads: int = 0, depth: int = 0, ctx=None, dst=None) -> Running:
    """zpx_batch_start: decode_rgba into device memory, asynchronously."""
    c = ctx or context.default()
    n = len(buffers)
    items, keep, outs = _bind(buffers, False, c, dst)
    opts = _lib.zpx_batch_opts(host_threads, depth, 0)
    h = C.c_void_p()
    _lib.check(_lib.lib().zpx_batch_start(c.handle, items, n, C.byref(opts), C.byref(h)), c.handle)
    return Running(h, items, keep, outs, n, c)
