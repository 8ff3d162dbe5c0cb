"""Per-GPU decode context (owns the HIP stream the kernels run on)."""
from __future__ import annotations

import ctypes as C
import threading

from . import _lib

_default = {}
_lock = threading.Lock()


class Context:
    """zpx_ctx: one per GPU; not shared by host threads concurrently."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        code = _lib.lib().zpx_ctx_create(device, C.byref(h))
        if code:
            raise _lib.ZpixError(_lib.error_name(code), f"no usable HIP device {device}")
        self.handle = h
        self.device = device

    @property
    def stream(self) -> int:
        """The hipStream_t (as an int) the context launches on."""
        return _lib.lib().zpx_ctx_stream(self.handle) or 0

    def synchronize(self) -> None:
        _lib.check(_lib.lib().zpx_ctx_synchronize(self.handle), self.handle)

    def close(self) -> None:
        if self.handle:
            _lib.lib().zpx_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def default(device: int | None = None) -> Context:
    """Process-wide context for `device` (default: current torch device or 0)."""
    if device is None:
        device = 0
        try:
            import torch

            if torch.cuda.is_available():
                device = torch.cuda.current_device()
        except Exception:
            pass
    with _lock:
        if device not in _default:
            _default[device] = Context(device)
        return _default[device]
