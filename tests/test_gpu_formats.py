"""GPU parity of the format edges: bmp.decode's row loop
and qoi.encode's segmented scan, against the oracle's restatements of
src/bmp/decoder.zig and src/qoi/encoder.zig (pinned in test_oracle.py by the
reference's BMP/PNG parity pairs and by Pillow's independent QOI codec).

- BMP: the reference's parity pairs (src/bmp/decoder_test.zig:24-61) and
  synthetic files over every bpp, ragged widths, top-down rows, V4/V5 headers
  (alpha kept) and BI_BITFIELDS with the default masks; bit-exact image +
  palette; truncated files are EndOfStream;
- QOI encode: byte-identical to the serial encoder on images that put runs,
  index hits and every chunk type across segment and block boundaries, RGB and
  RGBA, sizes not a multiple of the segment, and a 4096^2 frame;
- QOI decode (host) and zpix.fromBuffer's QOI/BMP dispatch.
"""
import io

import numpy as np
import pytest

import oracle_py as O
from conftest import golden, read
from test_oracle import BMP_PAIRS
from tools import synthetic as S

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import zpix_amd  # noqa: E402
from zpix_amd import bmp as B  # noqa: E402
from zpix_amd import qoi as Q  # noqa: E402


def assert_same_image(got, want):
    assert got.kind == want.kind
    assert tuple(got.rect) == tuple(want.rect)
    assert got.stride == want.stride
    assert np.array_equal(got.pixels, want.pixels)
    if want.kind == "Paletted":
        assert [tuple(p[:4]) for p in got.palette] == [tuple(p[:4]) for p in want.palette]


@pytest.mark.parametrize("name", BMP_PAIRS)
def test_bmp_pairs_gpu(name):
    """bmp: decode parity with png (src/bmp/decoder_test.zig:24-61) on the GPU path."""
    data = read("testdata", name + ".bmp")
    img = B.load(golden("testdata", name + ".bmp"))
    assert_same_image(img, O.bmp_decode(data))
    png = zpix_amd.png.load(golden("testdata", name + ".png"))
    assert tuple(img.rect) == tuple(png.rect)
    assert np.array_equal(img.rgba_pixels(), png.rgba_pixels())
    assert np.array_equal(zpix_amd.from_buffer(data).pixels, img.pixels)


CASES = [(bpp, w) for bpp in (1, 2, 4, 8, 24, 32) for w in (1, 3, 4, 5, 17, 64, 67)]


@pytest.mark.parametrize("bpp,w", CASES)
@pytest.mark.parametrize("top_down", [False, True])
def test_bmp_synthetic_gpu(bpp, w, top_down):
    h = 1 + (w * 7 + bpp) % 23
    for header in (40, 124):
        data, _ = S.bmp_bytes(bpp * 100 + w, w, h, bpp, top_down=top_down, header=header,
                              bitfields=header > 40 and bpp == 32)
        assert_same_image(B.decode(data), O.bmp_decode(data))


def test_bmp_short_palette_and_errors_gpu():
    data, _ = S.bmp_bytes(7, 33, 9, 8, ncol=17)
    assert_same_image(B.decode(data), O.bmp_decode(data))
    good, _ = S.bmp_bytes(8, 40, 30, 24)
    for cut in (0, 1, 17, 30, 54, 54 + 120 * 5 + 7, len(good) - 1):
        with pytest.raises(zpix_amd.ZpixError) as e:
            B.decode(good[:cut])
        with pytest.raises(O.OracleError) as eo:
            O.bmp_decode(good[:cut])
        assert e.value.name == eo.value.name == "EndOfStream", cut
    bad = bytearray(good)
    bad[28] = 16  # 16 bpp
    with pytest.raises(zpix_amd.ZpixError) as e:
        B.decode(bytes(bad))
    assert e.value.name == "UnsupportedBPP"
    # empty images: Paletted (0,0,0,0), RGBA keeps its width
    for bpp, want in ((8, (0, 0, 0, 0)), (24, (0, 0, 5, 0))):
        data, _ = S.bmp_bytes(9, 5, 0, bpp)
        img = B.decode(data)
        assert tuple(img.rect) == want == O.bmp_decode(data).rect


def _qoi_image(seed, w, h, ch, kind):
    rng = np.random.default_rng(seed)
    if kind == "noise":
        px = rng.integers(0, 256, (h, w, ch))
    elif kind == "smooth":  # DIFF / LUMA chunks
        px = np.clip(128 + np.cumsum(rng.integers(-3, 3, (h, w, ch)), axis=1), 0, 255)
    elif kind == "palette":  # INDEX hits
        pal = rng.integers(0, 256, (40, ch))
        px = pal[rng.integers(0, 40, (h, w))]
    elif kind == "runs":  # runs of every length across segment/block edges
        vals = rng.integers(0, 3, (h * w // 37 + 2, ch)) * 100
        lens = rng.integers(1, 400, len(vals))
        px = np.repeat(vals, lens, axis=0)[: h * w].reshape(h, w, ch) if lens.sum() >= h * w else np.zeros((h, w, ch))
    elif kind == "init":  # a leading run of {0,0,0,255} (never entered in the index)
        px = np.zeros((h, w, ch))
        if ch == 4:
            px[..., 3] = 255
        px[h // 2:, w // 2:] = rng.integers(0, 256, ch)
    else:  # "mixed"
        px = np.where(rng.random((h, w, 1)) < 0.5, rng.integers(0, 4, (h, w, ch)) * 63,
                      np.clip(128 + np.cumsum(rng.integers(-2, 2, (h, w, ch)), axis=1), 0, 255))
    if ch == 4 and kind in ("smooth", "mixed"):
        px[..., 3] = np.where(rng.random((h, w)) < 0.97, 255, rng.integers(0, 256, (h, w)))
    return np.ascontiguousarray(px.astype(np.uint8))


SHAPES = [(1, 1), (3, 1), (5, 7), (128, 1), (129, 3), (64 * 128 + 5, 1), (301, 257), (1024, 77)]


@pytest.mark.parametrize("ch", [3, 4])
@pytest.mark.parametrize("kind", ["noise", "smooth", "palette", "runs", "init", "mixed"])
@pytest.mark.parametrize("shape", SHAPES)
def test_qoi_encode_gpu_matches_serial(shape, kind, ch):
    w, h = shape
    px = _qoi_image(w * 31 + h + ch, w, h, ch, kind)
    got = Q.encode(px, Q.Desc(w, h, ch, 1))
    want = O.qoi_encode(px, w, h, ch, 1)
    assert got == want


@pytest.mark.parametrize("segment", [16, 64, 256, 1024])
def test_qoi_encode_segment_sizes(segment):
    """The segment size is a tuning knob (test switch "qoi_segment"); the
    bytes must not depend on it."""
    from zpix_amd import _lib

    prev = _lib.lib().zpx_debug_option(b"qoi_segment", segment)
    try:
        for k, (w, h) in enumerate([(1000, 37), (77, 64 * 16 + 3), (5, 5)]):
            for kind in ("runs", "mixed", "init"):
                px = _qoi_image(k, w, h, 4, kind)
                assert Q.encode(px, Q.Desc(w, h, 4, 0)) == O.qoi_encode(px, w, h, 4, 0), (segment, w, h, kind)
    finally:
        _lib.lib().zpx_debug_option(b"qoi_segment", prev)


def test_qoi_encode_4k_gpu():
    px = S.content(3, 4096, 4096, 4)
    px[100:900, 200:3000] = px[100:900, 200:201]  # long horizontal runs
    got = Q.encode(px, Q.Desc(4096, 4096, 4, 0))
    assert got == O.qoi_encode(px, 4096, 4096, 4, 0)
    img = Q.decode(got)
    assert np.array_equal(img.pixels.reshape(4096, 4096, 4), px)


def test_qoi_encode_device_form():
    w, h = 257, 129
    px = _qoi_image(5, w, h, 4, "mixed")
    desc = Q.Desc(w, h, 4, 0)
    cap = Q.encode_bound(desc)
    d_px = torch.from_numpy(px.reshape(-1)).cuda()
    d_out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx = zpix_amd.context.default()
    stream = torch.cuda.current_stream().cuda_stream
    Q.encode_device(d_px.data_ptr(), desc, d_out.data_ptr(), cap, d_len.data_ptr(), stream, ctx)
    torch.cuda.synchronize()
    n = int(d_len.item())
    assert bytes(d_out[:n].cpu().numpy()) == O.qoi_encode(px, w, h, 4, 0)


def test_qoi_encode_device_two_streams_share_scratch():
    """Encodes on two streams of one context share its scratch (tables,
    prefixes, slots): each is ordered after the previous user's work
    (zpx_ctx::scratch_ev), so back-to-back encodes of different images on
    different streams, and the context's own stream, all stay exact."""
    ctx = zpix_amd.context.default()
    streams = [torch.cuda.Stream(), torch.cuda.Stream(), None]
    jobs = []
    for k in range(6):
        w, h = 640 + 64 * k, 480 - 32 * k
        px = _qoi_image(40 + k, w, h, 4, "mixed")
        desc = Q.Desc(w, h, 4, 0)
        cap = Q.encode_bound(desc)
        d_px = torch.from_numpy(px.reshape(-1)).cuda()
        d_out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
        d_len = torch.zeros(1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        st = streams[k % 3]
        Q.encode_device(d_px.data_ptr(), desc, d_out.data_ptr(), cap, d_len.data_ptr(),
                        st.cuda_stream if st is not None else None, ctx)
        jobs.append((px, w, h, d_px, d_out, d_len))
    torch.cuda.synchronize()
    ctx.synchronize()
    for px, w, h, _, d_out, d_len in jobs:
        n = int(d_len.item())
        assert bytes(d_out[:n].cpu().numpy()) == O.qoi_encode(px, w, h, 4, 0), (w, h)


def test_qoi_decode_and_from_buffer():
    from PIL import Image

    for k, (w, h, ch) in enumerate([(1, 1, 4), (77, 31, 3), (300, 200, 4)]):
        px = _qoi_image(k, w, h, ch, "mixed")
        for data in (O.qoi_encode(px, w, h, ch, 0), _pillow_qoi(px, ch)):
            want = O.qoi_decode(data)
            got = Q.decode(data)
            assert_same_image(got, want)
            assert_same_image(zpix_amd.from_buffer(data), want)
            rgba = np.asarray(Image.open(io.BytesIO(data)).convert("RGBA"))
            assert np.array_equal(got.pixels.reshape(h, w, 4), rgba)


def _pillow_qoi(px, ch):
    from PIL import Image

    b = io.BytesIO()
    Image.fromarray(px, "RGBA" if ch == 4 else "RGB").save(b, format="QOI")
    return b.getvalue()
