"""GPU parity of the PNG pixel path (wavefront unfilter + pixel store + Adam7
scatter) and of Image.rgbaPixels, against the oracle and the reference goldens.

- PngSuite .sng goldens (src/png/decoder_test.zig) through the GPU decode;
- BMP parity pairs (src/bmp/decoder_test.zig, pins Avg + rgbaPixels);
- every colour type x bit depth x interlace x tRNS on random sizes that
  exercise partial chunks, one-row images, many 64-row bands;
- at the bench size (4096^2 tc8, mixed Sub/Up/Avg/Paeth): unfilter(filter(x))
  == x, a size-independent round trip.
"""
import glob
import os

import numpy as np
import pytest

import oracle_py as O
import sng
from conftest import golden, read
from test_oracle import BMP_PAIRS, PNGSUITE, bmp_rgba_premultiplied
from tools import synthetic as S

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import zpix_amd  # noqa: E402
from zpix_amd import device  # noqa: E402
from zpix_amd import png as P  # noqa: E402


def assert_same_png(got, want):
    assert got.kind == want.kind
    assert tuple(got.rect) == tuple(want.rect)
    assert got.stride == want.stride
    assert np.array_equal(got.pixels, want.pixels)
    if want.kind == "Paletted":
        assert [tuple(p) for p in got.palette] == [tuple(p) for p in want.palette]


@pytest.mark.parametrize("name", PNGSUITE)
def test_pngsuite_gpu(name):
    path = golden("pngsuite", name + ".png")
    img = P.load(path)
    assert_same_png(img, O.png_decode(read("pngsuite", name + ".png")))
    if name == "basn4a16":
        return
    with open(golden("pngsuite", name + ".sng")) as f:
        sng.compare_with_golden(sng.sng(path, img), f.read())


@pytest.mark.parametrize("name", BMP_PAIRS)
def test_bmp_parity_gpu(name):
    pytest.importorskip("PIL")
    img = P.load(golden("testdata", name + ".png"))
    rgba = img.rgba_pixels().reshape(img.height, img.width, 4)
    assert np.array_equal(rgba, bmp_rgba_premultiplied(golden("testdata", name + ".bmp")))


# (depth, color_type) pairs the reference accepts (png/decoder.zig:366-397)
COMBOS = [(1, 0), (2, 0), (4, 0), (8, 0), (16, 0), (8, 2), (16, 2), (1, 3), (2, 3), (4, 3), (8, 3),
          (8, 4), (16, 4), (8, 6), (16, 6)]
SIZES = [(1, 1), (3, 2), (17, 5), (64, 65), (130, 200), (33, 129)]


def _palette(n):
    rng = np.random.default_rng(n)
    return bytes(rng.integers(0, 256, 3 * n, dtype=np.uint8))


@pytest.mark.parametrize("depth,ct", COMBOS)
@pytest.mark.parametrize("interlace", [0, 1])
def test_png_all_depths(depth, ct, interlace):
    for k, (w, h) in enumerate(SIZES):
        seed = depth * 1000 + ct * 100 + interlace * 10 + k
        pal = _palette(min(1 << depth, 200)) if ct == 3 else None
        data = S.png_generic(seed, w, h, depth, ct, interlace=interlace, palette=pal)
        assert_same_png(P.decode(data), O.png_decode(data))


@pytest.mark.parametrize("depth,ct,trns", [
    (8, 2, b"\x00\x10\x00\x20\x00\x30"), (16, 2, b"\x12\x34\x56\x78\x9a\xbc"), (8, 0, b"\x00\x40"),
    (16, 0, b"\x40\x41"), (1, 0, b"\x00\x01"), (2, 0, b"\x00\x02"), (4, 0, b"\x00\x07"), (8, 3, None)])
@pytest.mark.parametrize("interlace", [0, 1])
def test_png_trns(depth, ct, trns, interlace):
    for k, (w, h) in enumerate(SIZES[2:]):
        pal = _palette(50) if ct == 3 else None
        t = trns if ct != 3 else bytes(np.random.default_rng(k).integers(0, 256, 30, dtype=np.uint8))
        data = S.png_generic(k + 77, w, h, depth, ct, interlace=interlace, trns=t, palette=pal)
        want = O.png_decode(data)
        got = P.decode(data)
        assert_same_png(got, want)
        assert np.array_equal(got.rgba_pixels(), want.rgba_pixels())


def test_png_out_of_range_palette_index_grows_palette():
    # indices up to 15 with a 4-entry PLTE: implicit palette growth
    data = S.png_generic(5, 40, 9, 4, 3, palette=_palette(16)[:12])
    got, want = P.decode(data), O.png_decode(data)
    assert_same_png(got, want)


@pytest.mark.parametrize("w,h", [(4096, 256), (333, 1000), (1000, 333), (7, 3000)])
def test_png_tc8_mixed_filters(w, h):
    data = S.png_tc8_mixed(w + h, w, h)
    assert_same_png(P.decode(data), O.png_decode(data))


class _device_slab:
    """Test switch png_device_slab: stream-layout frames on the paired-row
    kernel get their band slab built on the device (png_slab_kernels.hip)
    and the kernel's slab instance reads it."""

    def __init__(self, on):
        self.on = on

    def __enter__(self):
        from zpix_amd import _lib
        self.prev = _lib.lib().zpx_debug_option(b"png_device_slab", int(self.on))

    def __exit__(self, *a):
        from zpix_amd import _lib
        _lib.lib().zpx_debug_option(b"png_device_slab", self.prev)


LAYOUTS = ["auto", "stream", "stream_devslab"]


def _layout(layout):
    return ("stream" if layout.startswith("stream") else layout), _device_slab(layout.endswith("devslab"))


@pytest.mark.parametrize("layout", LAYOUTS)
def test_png_bench_size_roundtrip(layout):
    """4096^2 tc8 with per-row Sub/Up/Avg/Paeth: the GPU unfilter must return
    exactly the generator's raw pixels (unfilter(filter(x)) == x), from the
    host-built band slab ("auto"), from the inflated stream ("stream": the
    kernel's stream instance) and from a slab the plan builds on the device
    at every launch ("stream_devslab")."""
    raw, filt = S.png_filtered_tc8(0, 4096, 4096)
    data = S.encode_png(4096, 4096, 8, 2, filt.tobytes())
    st = P.Stream(data)
    lay, sw = _layout(layout)
    with sw:
        batch = device.PngBatch([st], slots=[0, 0], layout=lay)
    assert [f.layout for f in batch.frames] == [int(layout == "auto")] * 2
    for _ in range(2):  # relaunch: scratch must be re-initialised every call
        batch.launch(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    want = np.concatenate([raw.reshape(4096, 4096, 3), np.full((4096, 4096, 1), 255, np.uint8)], 2)
    for s in range(2):
        got = batch.output_tensor(s).cpu().numpy().reshape(4096, 4096, 4)
        assert np.array_equal(got, want)
    assert batch.bytes == 2 * (4096 * (1 + 4096 * 3) + 4096 * 4096 * 4)


def test_png_adam7_rgba16_roundtrip():
    data = S.png_rgba16_adam7(3, 1024, 768)
    assert_same_png(P.decode(data), O.png_decode(data))


def test_png_errors_gpu():
    base = S.png_generic(3, 37, 21, 8, 2)
    with pytest.raises(zpix_amd.ZpixError) as ei:
        P.decode(base[:-5])
    want = None
    try:
        O.png_decode(base[:-5])
    except O.OracleError as e:
        want = e.name
    assert ei.value.name == want


# ---------------------------------------------------------------- rgbaPixels
ALL_KIND_FILES = [("pngsuite", n + ".png") for n in PNGSUITE] + [
    ("testdata", n) for n in ("video-001.jpeg", "video-001.q50.410.jpeg", "video-001.q50.411.jpeg",
                              "video-001.q50.440.jpeg", "video-001.cmyk.jpeg", "video-001.rgb.jpeg",
                              "video-005.gray.jpeg", "video-001.221212.jpeg")]


@pytest.mark.parametrize("where,name", ALL_KIND_FILES)
def test_rgba_pixels_every_kind(where, name):
    data = read(where, name)
    want = O.decode(data)
    got = zpix_amd.from_buffer(data)
    assert got.kind == want.kind
    assert np.array_equal(got.rgba_pixels(), want.rgba_pixels())


@pytest.mark.parametrize("layout", LAYOUTS)
def test_png_adam7_rgba16_4k_matches_oracle(layout):
    """configs[4] PNG at its bench size: 4096^2 Adam7 RGBA16 -> NRGBA64 (7
    passes scattered by mergePassInto), bit-exact against the oracle, twice
    through one plan (relaunch), plus zpx_plan_status; host slab, the
    stream, device-built slab."""
    data = S.png_rgba16_adam7(2000, 4096, 4096)
    want = O.png_decode(data).pixels
    st = P.Stream(data)
    lay, sw = _layout(layout)
    with sw:
        batch = device.PngBatch([st], slots=[0, 0], layout=lay)
    for _ in range(2):
        batch.launch(torch.cuda.current_stream().cuda_stream)
    batch.status(torch.cuda.current_stream().cuda_stream)
    for s in range(2):
        got = batch.output_tensor(s).cpu().numpy()
        assert np.array_equal(got.reshape(-1)[:want.size], want.reshape(-1))


@pytest.mark.parametrize("layout", ["stream", "auto", "mixed", "stream_devslab", "mixed_devslab"])
@pytest.mark.parametrize("depth,ct,il", [(8, 2, 0), (8, 6, 1), (16, 6, 1), (16, 2, 0), (8, 0, 0), (16, 0, 0),
                                         (8, 2, 1)])
def test_png_plan_layouts(layout, depth, ct, il):
    """zpx_png_plan on both input layouts: the band slab (paired-row kernel,
    zpx_png_stream_slab) and the inflated stream (the paired-row kernel's
    stream instance where it takes the image, else the one-row-per-lane
    kernel; *_devslab: the slab built on the device from it), and both in
    one plan (two launches), bit-exact against the oracle, in one ragged
    batch of four sizes."""
    datas = [S.png_generic(depth * 100 + ct * 10 + il + k, w, h, depth, ct, interlace=il, filters=(0, 1, 2, 3, 4))
             for k, (w, h) in enumerate([(17, 5), (130, 200), (33, 129), (300, 260)])]
    streams = [P.Stream(d) for d in datas]
    lay, sw = layout.split("_")[0], _device_slab(layout.endswith("devslab"))
    with sw:
        b = device.PngBatch(streams, layout=lay)
    # (auto: a slab wherever the paired-row kernel takes the image -- not
    # the smallest Adam7 passes -- and always the 300 x 260 one)
    slab = [lay == "auto" or (lay == "mixed" and i % 2 == 0) for i in range(4)]
    assert [f.layout for f in b.frames] == [int(s and st.slab() is not None) for s, st in zip(slab, streams)]
    assert b.frames[3].layout == (1 if lay == "auto" else 0)
    b.launch(torch.cuda.current_stream().cuda_stream)
    b.status(torch.cuda.current_stream().cuda_stream)
    for s, d in enumerate(datas):
        want = O.png_decode(d).pixels.reshape(-1)
        assert np.array_equal(b.output_tensor(s).cpu().numpy().reshape(-1)[:want.size], want)


@pytest.mark.parametrize("depth,ct,w,h,il", [
    (8, 2, 70, 300, 0),     # TC8: 12-byte chunks, a partial last band
    (8, 6, 33, 130, 0),     # TCA8
    (16, 6, 21, 40, 1),     # TCA16 Adam7
    (16, 2, 17, 17, 1),     # TC16 Adam7, tiny passes
    (8, 0, 100, 129, 0),    # G8
    (16, 0, 64, 64, 0),     # G16
    (8, 2, 1500, 300, 0),   # TC8: 375 chunks a row, several 16-group windows per band
    (8, 6, 700, 260, 1),    # TCA8 Adam7, wide passes
    (16, 2, 2049, 131, 0),  # TC16, odd width, rows past the band
])
def test_png_device_slab_matches_model(depth, ct, w, h, il):
    """The band slab the plans build on the device from the inflated stream
    (png_slab_kernels.hip) holds exactly the bytes the paired-row kernel
    reads (the Python model of tests/test_png_slab.py, which also pins the
    host builder)."""
    import ctypes as C

    from test_png_slab import check_slab
    from zpix_amd import _lib

    d = S.png_generic(3 + w, w, h, depth, ct, interlace=il, filters=(0, 1, 2, 3, 4))
    st = P.Stream(d)
    ctx = zpix_amd.context.default()
    n = C.c_size_t(0)
    _lib.check(_lib.lib().zpx_debug_png_device_slab(ctx.handle, st.handle, None, 0, C.byref(n)), ctx.handle)
    out = np.zeros(n.value, np.uint8)
    _lib.check(_lib.lib().zpx_debug_png_device_slab(ctx.handle, st.handle, out.ctypes.data, n.value, C.byref(n)),
               ctx.handle)
    check_slab(st, out)


def test_png_plans_recreated_at_same_addresses():
    """Plans of one geometry made and destroyed back to back (their boundary
    buffers handed out again at the same addresses): each plan's launches
    use epochs from a window of their own (PngControl), so granules a
    destroyed plan wrote -- which another XCD's L2 may still hold -- never
    pass for this launch's; every launch bit-exact, slab and stream
    instances alternating."""
    datas = [S.png_tc8_mixed(70 + i, 640, 1000) for i in range(2)]
    streams = [P.Stream(d) for d in datas]
    want = [O.png_decode(d).pixels.reshape(-1) for d in datas]
    for k in range(6):
        b = device.PngBatch(streams, slots=[0, 1] * 4, layout=("stream", "auto")[k % 2])
        for _ in range(2):
            b.launch(torch.cuda.current_stream().cuda_stream)
        b.status(torch.cuda.current_stream().cuda_stream)
        for s in range(8):
            assert np.array_equal(b.output_tensor(s).cpu().numpy().reshape(-1)[:want[s % 2].size], want[s % 2]), (k, s)
        del b


class _EpochCycle:
    """Test switch png_epoch_cycle: control blocks created inside the block
    cycle through `n` epochs, so their launches wrap (PngControl)."""

    def __init__(self, n):
        self.n = n

    def __enter__(self):
        from zpix_amd import _lib
        self.prev = _lib.lib().zpx_debug_option(b"png_epoch_cycle", self.n)

    def __exit__(self, *exc):
        from zpix_amd import _lib
        _lib.lib().zpx_debug_option(b"png_epoch_cycle", self.prev)


EPOCH_CASES = {
    "tc8": lambda seed: S.png_tc8_mixed(seed, 700, 900),            # paired-row kernel
    "adam7_rgba16": lambda seed: S.png_rgba16_adam7(seed, 300, 520),  # two launches a plan launch
    "ga8": lambda seed: S.png_generic(seed, 333, 300, 8, 4),          # one-row-per-lane kernel
}


@pytest.mark.parametrize("case", sorted(EPOCH_CASES))
def test_png_epoch_cycle_wraps_with_changing_input(case):
    """A plan whose control block wraps its epoch cycle every few launches
    (png_epoch_cycle 4; Adam7 groups take two epochs a launch): the input
    bytes change between launches -- two images of one geometry, different
    filters and pixels, swapped in place -- so a band that took a granule
    left from an earlier launch would unfilter from the wrong row above and
    differ.  Every launch bit-exact against the oracle (readImagePass,
    png/decoder.zig:798-842)."""
    a, b = EPOCH_CASES[case](301), EPOCH_CASES[case](302)
    st = torch.cuda.current_stream().cuda_stream
    with _EpochCycle(4):
        streams = [P.Stream(a), P.Stream(b)]
        want = [O.png_decode(d).pixels.reshape(-1) for d in (a, b)]
        data = [s.filtered() for s in streams]
        assert len(data[0]) == len(data[1])
        bt = device.PngBatch(streams, slots=[0], layout="stream")
        n = len(data[0])
        for k in range(11):
            bt.in_arena[:n].copy_(torch.from_numpy(data[k % 2]))
            bt.out_arena.zero_()
            bt.launch(st)
            bt.status(st)
            got = bt.output_tensor(0).cpu().numpy().reshape(-1)[:want[k % 2].size]
            assert np.array_equal(got, want[k % 2]), k


def test_png_epoch_cycle_wraps_in_batch_slots():
    """The batch pipeline's slots with a 4-epoch cycle: one slot decodes PNGs
    of changing geometry one after the other (so a granule may stay unread
    for many launches), wrapping several times; every image bit-exact."""
    from zpix_amd import batch
    bufs = []
    for i in range(14):
        w, h = 90 + 37 * (i % 5), 140 + 61 * (i % 3)
        bufs.append(S.png_rgba16_adam7(400 + i, w, h) if i % 3 == 0 else S.png_tc8_mixed(400 + i, w, h))
    with _EpochCycle(4):
        res = batch.decode_rgba(bufs, host_threads=1, depth=1)
    for data, r in zip(bufs, res):
        img = O.png_decode(data)
        want = img.rgba_pixels().reshape(img.height, img.width, 4)
        assert r.status == "Ok"
        assert np.array_equal(r.rgba.cpu().numpy(), want)
