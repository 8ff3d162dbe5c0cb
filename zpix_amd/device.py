"""Device-resident batches over the plan C-ABI (zpx_*_plan_create / launch).

Inputs (coefficient grids, filtered PNG streams) are uploaded once into HBM
(torch.uint8 arenas: torch is plumbing for device memory and streams here);
`launch()` then only enqueues the plan's kernels on a stream, which is what
bench.py times.  No host work or copy happens inside `launch()`.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib, context
from .jpeg import Coefficients
from .png import INPUT_PAD, Stream

ALIGN = 256


def _torch():
    import torch

    return torch


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass
class JpegLayout:
    """makeImg layout (src/jpeg/decoder.zig:1708-1783; image.zig:484-555)."""

    subsample: int
    y_stride: int
    y_rows: int
    c_stride: int
    c_rows: int
    cb_off: int
    cr_off: int
    total: int


def jpeg_layout(frame) -> JpegLayout:
    if frame.n_comp == 1:
        ys, yr = 8 * frame.mxx, 8 * frame.myy
        return JpegLayout(0, ys, yr, 0, 0, 0, 0, ys * yr)
    h0, v0 = frame.h[0], frame.v[0]
    hr, vr = h0 // frame.h[1], v0 // frame.v[1]
    sub = {0x11: 0, 0x12: 3, 0x21: 1, 0x22: 2, 0x41: 4, 0x42: 5}[(hr << 4) | vr]
    w, h = 8 * h0 * frame.mxx, 8 * v0 * frame.myy
    cw = {0: w, 1: (w + 1) // 2, 2: (w + 1) // 2, 3: w, 4: (w + 3) // 4, 5: (w + 3) // 4}[sub]
    ch = {0: h, 1: h, 2: (h + 1) // 2, 3: (h + 1) // 2, 4: h, 5: (h + 1) // 2}[sub]
    return JpegLayout(sub, w, h, cw, ch, w * h, w * h + cw * ch, w * h + 2 * cw * ch)


class _Plan:
    def __init__(self, handle, ctx):
        self.handle = handle
        self.ctx = ctx

    @property
    def bytes(self) -> int:
        return int(_lib.lib().zpx_plan_bytes(self.handle))

    @property
    def kernel_count(self) -> int:
        return int(_lib.lib().zpx_plan_kernel_count(self.handle))

    def launch(self, stream: int | None = None) -> None:
        _lib.check(_lib.lib().zpx_plan_launch(self.handle, stream or None), self.ctx.handle)

    def status(self, stream: int | None = None) -> None:
        """zpx_plan_status: waits for `stream` and raises ZpixError('Hip') if
        any launch since the last call timed out in a PNG wavefront hand-off."""
        _lib.check(_lib.lib().zpx_plan_status(self.handle, stream or None), self.ctx.handle)

    def close(self):
        if self.handle:
            _lib.lib().zpx_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class JpegBatch:
    """A batch of JPEG frames resident in HBM, reconstructed by one plan.

    items: host entropy results (`jpeg.Coefficients`, grids or pieces); `slots[i]` picks which
    item fills device slot i (a slot owns its own copy of the grids and its
    own output, so repeating an item does not share any buffer).
    output: "rgba" (fused reconstruct + rgbaPixels) or "planes".
    """

    def __init__(self, items: list[Coefficients], slots: list[int] | None = None, output: str = "rgba",
                 device: int = 0, ctx: context.Context | None = None):
        torch = _torch()
        self.ctx = ctx or context.default(device)
        self.device = torch.device("cuda", self.ctx.device)
        self.items = items
        self.slots = list(range(len(items))) if slots is None else list(slots)
        self.output = output
        frames = (_lib.zpx_jpeg_frame * len(self.slots))()
        # (a pieces frame: its index arrays in coeff_bytes, then its pieces)
        in_bytes = sum(_align(b) for i in self.slots for b in items[i].coeff_bytes)
        in_bytes += sum(_align(int(items[i].frame.pieces_bytes)) for i in self.slots if items[i].frame.layout == 1)
        self.layouts = [jpeg_layout(items[i].frame) for i in self.slots]
        if output == "rgba":
            out_sizes = [_align(items[i].frame.width * items[i].frame.height * 4) for i in self.slots]
        else:
            out_sizes = [_align(lay.total) for lay in self.layouts]
        self.coeff_arena = torch.empty(max(in_bytes, 1), dtype=torch.uint8, device=self.device)
        self.out_arena = torch.zeros(max(sum(out_sizes), 1), dtype=torch.uint8, device=self.device)
        base_in = self.coeff_arena.data_ptr()
        base_out = self.out_arena.data_ptr()
        off_in = 0
        off_out = 0
        self.out_offsets = []
        for s, i in enumerate(self.slots):
            f = frames[s]
            C.pointer(f)[0] = items[i].frame
            for c in range(4):
                n = items[i].coeff_bytes[c]
                if not n:
                    continue
                host = np.ctypeslib.as_array(C.cast(items[i].frame.coeffs[c], C.POINTER(C.c_uint8)), shape=(n,))
                self.coeff_arena[off_in:off_in + n].copy_(torch.from_numpy(host), non_blocking=False)
                f.coeffs[c] = base_in + off_in
                off_in += _align(n)
            if f.layout == 1:
                n = int(f.pieces_bytes)
                host = np.ctypeslib.as_array(C.cast(items[i].frame.pieces, C.POINTER(C.c_uint8)), shape=(n,))
                self.coeff_arena[off_in:off_in + n].copy_(torch.from_numpy(host), non_blocking=False)
                f.pieces = base_in + off_in
                off_in += _align(n)
            self.out_offsets.append(off_out)
            if output == "rgba":
                f.rgba = base_out + off_out
                f.rgba_stride = f.width * 4
            else:
                lay = self.layouts[s]
                p = base_out + off_out
                f.planes[0] = p
                f.strides[0] = lay.y_stride
                if f.n_comp >= 3:
                    f.planes[1] = p + lay.cb_off
                    f.planes[2] = p + lay.cr_off
                    f.strides[1] = f.strides[2] = lay.c_stride
            off_out += out_sizes[s]
        self.out_sizes = out_sizes
        torch.cuda.synchronize(self.device)
        h = C.c_void_p()
        _lib.check(_lib.lib().zpx_jpeg_plan_create(self.ctx.handle, frames, len(self.slots),
                                                   1 if output == "rgba" else 0, C.byref(h)), self.ctx.handle)
        self.plan = _Plan(h, self.ctx)
        self.frames = frames
        self.pixels = sum(items[i].frame.width * items[i].frame.height for i in self.slots)

    @property
    def bytes(self) -> int:
        return self.plan.bytes

    def launch(self, stream: int | None = None) -> None:
        self.plan.launch(stream)

    def output_tensor(self, slot: int):
        """Device view of slot's output (RGBA HxWx4, or the flat planes buffer)."""
        f = self.frames[slot]
        o = self.out_offsets[slot]
        if self.output == "rgba":
            n = f.width * f.height * 4
            return self.out_arena[o:o + n].view(f.height, f.width, 4)
        return self.out_arena[o:o + self.layouts[slot].total]


class PngBatch:
    """A batch of PNG images resident in HBM, unfiltered + stored by one plan."""

    def __init__(self, items: list[Stream], slots: list[int] | None = None, device: int = 0,
                 ctx: context.Context | None = None, layout: str = "auto"):
        """layout: "auto" uploads each image's host-built band slab where
        the paired-row kernel takes it (Stream.slab), else the inflated
        stream; "stream" always the inflated stream, as parseIdat hands it to
        readImagePass (png/decoder.zig:516-523), which the kernels read as
        is (the paired-row kernel's stream instance; what png.decode and the
        batch pipeline do); "mixed" (tests) slabs for even item indices,
        streams for odd ones.  The plan is made here, so the test switch
        png_device_slab applies as it is set now."""
        torch = _torch()
        self.ctx = ctx or context.default(device)
        self.device = torch.device("cuda", self.ctx.device)
        self.items = items
        self.slots = list(range(len(items))) if slots is None else list(slots)
        frames = (_lib.zpx_png_frame * len(self.slots))()
        inputs = {}
        for i in set(self.slots):
            sl = items[i].slab() if layout == "auto" or (layout == "mixed" and i % 2 == 0) else None
            inputs[i] = (sl, 1) if sl is not None else (items[i].filtered(), 0)
        in_sizes = [_align(len(inputs[i][0])) for i in self.slots]
        out_sizes = [_align(items[i].frame.out_stride * items[i].frame.height) for i in self.slots]
        self.in_arena = torch.empty(max(sum(in_sizes), 1), dtype=torch.uint8, device=self.device)
        self.out_arena = torch.zeros(max(sum(out_sizes), 1), dtype=torch.uint8, device=self.device)
        self.max_index = torch.zeros(len(self.slots) * 4, dtype=torch.int32, device=self.device)
        oi = oo = 0
        self.out_offsets = []
        for s, i in enumerate(self.slots):
            st = items[i]
            f = frames[s]
            C.pointer(f)[0] = st.frame
            data, lay = inputs[i]
            self.in_arena[oi:oi + len(data)].copy_(torch.from_numpy(data))
            f.filtered = self.in_arena.data_ptr() + oi
            f.layout = lay
            f.out = self.out_arena.data_ptr() + oo
            f.max_index = self.max_index.data_ptr() + 16 * s
            self.out_offsets.append(oo)
            oi += in_sizes[s]
            oo += out_sizes[s]
        torch.cuda.synchronize(self.device)
        h = C.c_void_p()
        _lib.check(_lib.lib().zpx_png_plan_create(self.ctx.handle, frames, len(self.slots), C.byref(h)),
                   self.ctx.handle)
        self.plan = _Plan(h, self.ctx)
        self.frames = frames
        self.pixels = sum(items[i].frame.width * items[i].frame.height for i in self.slots)

    @property
    def bytes(self) -> int:
        return self.plan.bytes

    def launch(self, stream: int | None = None) -> None:
        self.plan.launch(stream)

    def status(self, stream: int | None = None) -> None:
        self.plan.status(stream)

    def output_tensor(self, slot: int):
        f = self.frames[slot]
        o = self.out_offsets[slot]
        return self.out_arena[o:o + f.out_stride * f.height]


class RgbaBatch:
    """Image.rgbaPixels (image.zig:103-130) of a batch of images resident in
    HBM, as one plan (zpx_rgba_plan_create): `items` are host `Image`s,
    uploaded once; `slots[i]` picks the item of device slot i; launch()
    converts every slot to RGBA8 (stride 4 * width) in HBM."""

    def __init__(self, items, slots: list[int] | None = None, device: int = 0,
                 ctx: context.Context | None = None):
        torch = _torch()
        self.ctx = ctx or context.default(device)
        self.device = torch.device("cuda", self.ctx.device)
        self.items = items
        self.slots = list(range(len(items))) if slots is None else list(slots)
        in_sizes = [_align(np.asarray(items[i].pixels).size) + _align(256 * C.sizeof(_lib.zpx_color))
                    for i in self.slots]
        out_sizes = [_align(items[i].width * items[i].height * 4) for i in self.slots]
        self.in_arena = torch.empty(max(sum(in_sizes), 1), dtype=torch.uint8, device=self.device)
        self.out_arena = torch.zeros(max(sum(out_sizes), 1), dtype=torch.uint8, device=self.device)
        imgs = (_lib.zpx_image * len(self.slots))()
        outs = (C.c_void_p * len(self.slots))()
        oi = oo = 0
        self.out_offsets = []
        for s, i in enumerate(self.slots):
            img = items[i]
            raw = img._to_c()  # (its palette pointer lives until the next _to_c of this item)
            px = np.ascontiguousarray(img.pixels, np.uint8)
            self.in_arena[oi:oi + px.size].copy_(torch.from_numpy(px))
            imgs[s] = raw
            imgs[s].pixels = C.cast(C.c_void_p(self.in_arena.data_ptr() + oi), C.POINTER(C.c_uint8))
            if img.kind == "Paletted" and raw.palette:
                pal = np.ctypeslib.as_array(C.cast(raw.palette, C.POINTER(C.c_uint8)),
                                            shape=(256 * C.sizeof(_lib.zpx_color),)).copy()
                po = oi + _align(px.size)
                self.in_arena[po:po + pal.size].copy_(torch.from_numpy(pal))
                imgs[s].palette = C.cast(C.c_void_p(self.in_arena.data_ptr() + po), C.POINTER(_lib.zpx_color))
            outs[s] = self.out_arena.data_ptr() + oo
            self.out_offsets.append(oo)
            oi += in_sizes[s]
            oo += out_sizes[s]
        torch.cuda.synchronize(self.device)
        h = C.c_void_p()
        _lib.check(_lib.lib().zpx_rgba_plan_create(self.ctx.handle, imgs, outs, len(self.slots), C.byref(h)),
                   self.ctx.handle)
        self.plan = _Plan(h, self.ctx)
        self.pixels = sum(items[i].width * items[i].height for i in self.slots)

    @property
    def bytes(self) -> int:
        return self.plan.bytes

    def launch(self, stream: int | None = None) -> None:
        self.plan.launch(stream)

    def output_tensor(self, slot: int):
        img = self.items[self.slots[slot]]
        o = self.out_offsets[slot]
        return self.out_arena[o:o + img.width * img.height * 4].view(img.height, img.width, 4)
