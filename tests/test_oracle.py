"""Pin the CPU oracle against every golden the reference's own tests hold.

- PNG: 35 PngSuite files vs .sng goldens (src/png/decoder_test.zig:8-129),
  bit-exact, with the silent-exit-on-failure bug removed (a load failure fails).
- PNG Avg filter + rgbaPixels: BMP parity pairs (src/bmp/decoder_test.zig:24-61),
  through the oracle's bmp.decode restatement, with Pillow's BMP reader as a
  second, independent reader of the same .bmp files.
- QOI (src/qoi/encoder.zig, decoder.zig): the reference holds no QOI fixture,
  so the restatement is pinned against Pillow's independent QOI codec (the
  published qoi.h algorithm): identical chunk bytes from the encoder, identical
  pixels from the decoder.
- JPEG: baseline == progressive planes for 10 pairs (src/jpeg/decoder.zig:1843-1920),
  assorted decodes (:1922-1940) and the error cases (:1942-2279).
"""
import numpy as np
import pytest

import oracle_py as O
import sng
from conftest import golden, read

PNGSUITE = [
    "basn0g01", "basn0g01-30", "basn0g02", "basn0g02-29", "basn0g04", "basn0g04-31",
    "basn0g08", "basn0g16", "basn2c08", "basn2c16", "basn3p01", "basn3p02", "basn3p04",
    "basn3p04-31i", "basn3p08", "basn3p08-trns", "basn4a08", "basn4a16", "basn6a08",
    "basn6a16", "ftbbn0g01", "ftbbn0g02", "ftbbn0g04", "ftbbn2c16", "ftbbn3p08",
    "ftbgn2c16", "ftbgn3p08", "ftbrn2c08", "ftbwn0g16", "ftbwn3p08", "ftbyn3p08",
    "ftp0n0g08", "ftp0n2c08", "ftp0n3p08", "ftp1n3p08",
]
BMP_PAIRS = ["colormap", "colormap-0", "colormap-251", "video-001", "yellow_rose-small",
             "yellow_rose-small-v5", "bmp_1bpp", "bmp_4bpp", "bmp_8bpp"]
JPEG_PAIRS = ["video-001", "video-001.q50.410", "video-001.q50.411", "video-001.q50.420",
              "video-001.q50.422", "video-001.q50.440", "video-001.q50.444", "video-005.gray.q50",
              "video-005.gray.q50.2x2", "video-001.separate.dc.progression"]


@pytest.mark.parametrize("name", PNGSUITE)
def test_pngsuite_sng(name):
    img = O.png_decode(read("pngsuite", name + ".png"))
    if name == "basn4a16":  # decoder_test.zig:58-65 checks one pixel
        assert img.kind == "NRGBA64"
        p = img.pixels[1 * img.stride + 2 * 8:][:8]
        vals = [(int(p[i]) << 8) | int(p[i + 1]) for i in range(0, 8, 2)]
        assert vals == [0x11A7, 0x11A7, 0x11A7, 0x1085]
        return
    got = sng.sng(golden("pngsuite", name + ".png"), img)
    with open(golden("pngsuite", name + ".sng")) as f:
        sng.compare_with_golden(got, f.read())


def bmp_rgba_premultiplied(path):
    from PIL import Image

    ba = np.asarray(Image.open(path).convert("RGBA"))
    a = ba[..., 3:4].astype(np.uint32)
    pm = ((ba[..., :3].astype(np.uint32) * 0x101 * a) // 0xFF) >> 8
    return np.concatenate([pm.astype(np.uint8), ba[..., 3:4]], -1)


@pytest.mark.parametrize("name", BMP_PAIRS)
def test_png_bmp_parity(name):
    pytest.importorskip("PIL")
    img = O.png_decode(read("testdata", name + ".png"))
    rgba = img.rgba_pixels().reshape(img.height, img.width, 4)
    assert np.array_equal(rgba, bmp_rgba_premultiplied(golden("testdata", name + ".bmp")))


@pytest.mark.parametrize("name", BMP_PAIRS)
def test_bmp_decode_parity_with_png(name):
    """bmp: decode parity with png (src/bmp/decoder_test.zig:24-61)."""
    b = O.bmp_decode(read("testdata", name + ".bmp"))
    p = O.png_decode(read("testdata", name + ".png"))
    assert b.rect == p.rect
    assert np.array_equal(b.rgba_pixels(), p.rgba_pixels())


def test_bmp_empty_input_is_end_of_stream():
    """bmp: empty input returns eof (src/bmp/decoder_test.zig:63-69)."""
    with pytest.raises(O.OracleError) as e:
        O.bmp_decode(b"")
    assert e.value.name == "EndOfStream"


def _qoi_pixels(seed, w, h, ch):
    rng = np.random.default_rng(seed)
    # runs, index hits, small diffs, luma diffs and literals all occur
    base = rng.integers(0, 4, (h, w, ch)) * 63
    walk = np.cumsum(rng.integers(-2, 2, (h, w, ch)), axis=1)
    # clipped so no channel step exceeds 207: the reference takes differences
    # in i16 without wrapping (encoder.zig:97-101) while qoi.h/Pillow wrap them
    # mod 256, and the two agree whenever no wrapped step is small
    px = np.where(rng.random((h, w, 1)) < 0.5, base, np.clip(128 + walk, 48, 207)).astype(np.uint8)
    px[:, : w // 3] = px[:, :1]  # long runs (>62)
    return px


@pytest.mark.parametrize("ch", [3, 4])
@pytest.mark.parametrize("shape", [(1, 1), (7, 3), (61, 5), (200, 31)])
def test_qoi_encode_matches_pillow(shape, ch):
    from PIL import Image
    import io

    w, h = shape
    px = _qoi_pixels(w * h + ch, w, h, ch)
    ours = O.qoi_encode(px, w, h, ch, 0)
    buf = io.BytesIO()
    Image.fromarray(px, "RGBA" if ch == 4 else "RGB").save(buf, format="QOI")
    theirs = buf.getvalue()
    assert ours[:13] == theirs[:13] and ours[13] == 0  # Pillow writes colorspace 1
    assert ours[14:] == theirs[14:]
    img = O.qoi_decode(ours)
    assert img.kind == "RGBA" and img.rect == (0, 0, w, h)
    want = px if ch == 4 else np.concatenate([px, np.full((h, w, 1), 255, np.uint8)], -1)
    assert np.array_equal(img.pixels.reshape(h, w, 4), want)
    assert np.array_equal(np.asarray(Image.open(io.BytesIO(ours)).convert("RGBA")), want)


def test_qoi_encode_diffs_do_not_wrap():
    """255 -> 0 is a 4-byte QOI_OP_RGB in the reference (i16 differences,
    encoder.zig:97-113), not the 1-byte wrapped QOI_OP_DIFF of qoi.h."""
    px = np.array([[[255, 10, 10, 255], [0, 10, 10, 255]]], np.uint8)
    out = O.qoi_encode(px, 2, 1, 4)
    assert out[14:] == bytes([0xFE, 255, 10, 10, 0xFE, 0, 10, 10]) + bytes(7) + b"\x01"
    assert np.array_equal(O.qoi_decode(out).pixels.reshape(1, 2, 4), px)


def test_qoi_decode_wrapping_diff():
    """A qoi.h-style stream whose DIFF step wraps (255 -> 0 as dr = +1, the
    1-byte QOI_OP_DIFF Pillow's encoder emits): the reference's @intCast
    (decoder.zig:97-114) traps on it in a safety-checked build; the oracle
    and the product wrap mod 256 as the QOI specification does (documented
    deviation, formats_api.cpp) -- the same pixels as Pillow's decoder."""
    from PIL import Image
    import io

    px = np.array([[[255, 10, 10, 255], [0, 10, 10, 255], [1, 9, 255, 255], [255, 255, 0, 255]]], np.uint8)
    buf = io.BytesIO()
    Image.fromarray(px, "RGBA").save(buf, format="QOI")
    data = buf.getvalue()
    assert any((b & 0xC0) == 0x40 for b in data[14:-8])  # a DIFF chunk is in there
    img = O.qoi_decode(data)
    assert np.array_equal(img.pixels.reshape(1, 4, 4), px)
    assert np.array_equal(np.asarray(Image.open(io.BytesIO(data)).convert("RGBA")), px)


def test_qoi_errors():
    with pytest.raises(O.OracleError) as e:
        O.qoi_encode(np.zeros(4, np.uint8), 0, 1, 4)
    assert e.value.name == "InvalidQoiHeader"
    with pytest.raises(O.OracleError) as e:
        O.qoi_decode(b"qoif" + bytes(10))
    assert e.value.name == "InvalidQoiData"
    with pytest.raises(O.OracleError) as e:
        O.qoi_decode(b"qoix" + bytes(30))
    assert e.value.name == "InvalidQoiHeader"


def _check_blocks(bounds, p0, p1, s0, s1):
    """check(), src/jpeg/decoder.zig:1803-1836."""
    w, h = bounds
    assert s0 % 8 == 0 and s1 % 8 == 0
    rows = min(len(p0) // s0, len(p1) // s1)
    for y in range(0, rows, 8):
        for x in range(0, min(s0, s1), 8):
            if x >= w or y >= h:
                continue
            for j in range(8):
                a = p0[(y + j) * s0 + x:(y + j) * s0 + x + 8]
                b = p1[(y + j) * s1 + x:(y + j) * s1 + x + 8]
                assert np.array_equal(a, b), (x, y, j)


@pytest.mark.parametrize("name", JPEG_PAIRS)
def test_jpeg_baseline_equals_progressive(name):
    a = O.jpeg_decode(read("testdata", name + ".jpeg"))
    b = O.jpeg_decode(read("testdata", name + ".progressive.jpeg"))
    assert a.rect == b.rect == (0, 0, 150, 103)
    assert a.kind == b.kind
    if a.kind == "Gray":
        _check_blocks((150, 103), a.pixels, b.pixels, a.stride, b.stride)
    else:
        assert a.kind == "YCbCr"
        for pa, pb, sa, sb in zip(a.planes(), b.planes(), (a.y_stride, a.c_stride, a.c_stride),
                                  (b.y_stride, b.c_stride, b.c_stride)):
            _check_blocks((150, 103), pa, pb, sa, sb)


@pytest.mark.parametrize("name,kind", [("video-001.cmyk", "CMYK"), ("video-001.221212", "YCbCr"),
                                       ("video-005.gray", "Gray"), ("video-001.rgb", "RGBA"),
                                       ("video-001.separate.dc.progression", "YCbCr")])
def test_jpeg_assorted(name, kind):
    assert O.jpeg_decode(read("testdata", name + ".jpeg")).kind == kind


def _err(data):
    try:
        O.jpeg_decode(data)
        return "OK"
    except O.OracleError as e:
        return e.name


def test_jpeg_truncated_sos():
    b = read("testdata", "video-005.gray.q50.jpeg")
    i = b.index(b"\xff\xda") + 2
    for k in range(i, min(i + 10, len(b))):
        assert _err(b[:k]) == "UnexpectedEof"


def test_jpeg_large_image_short_data():
    assert _err(read("testdata", "large_short.jpeg")) == "UnexpectedEof"


def test_jpeg_padded_rst():
    assert _err(read("testdata", "padded_rst.jpeg")) == "OK"


def test_jpeg_truncated_24():
    assert _err(read("testdata", "video-001.jpeg")[:24]) == "UnexpectedEof"


RST_CASES = [(b"PASS:", "OK"), (b"PASS:\x00", "OK"), (b"PASS:\x61", "OK"),
             (b"PASS:\x61\x62\x63\xff\x00\x64", "OK"), (b"PASS:\xff", "OK"), (b"PASS:\xff\x00", "OK"),
             (b"PASS:\xff\xff\xff\x00\xff\x00\x00\xff\xff\xff", "OK"),
             (b"FAIL:\xff\x03", "BadRSTMarker"), (b"FAIL:\xff\xd5", "BadRSTMarker"),
             (b"FAIL:\xff\xff\xd5", "BadRSTMarker")]


@pytest.mark.parametrize("infix,want", RST_CASES)
def test_jpeg_bad_restart_marker(infix, want):
    r = read("testdata", "video-001.restart2.jpeg")
    assert len(r) == 4855 and r[2816:2818] == b"\xff\xd1"
    assert _err(r[:2816] + infix[5:] + r[2816:]) == want


def test_idct_dc_shortcut_identity():
    """The row pass DC-only shortcut (idct.zig:84-97) equals the full path for every
    DC value a conforming 8-bit stream can produce; the GPU path relies on this."""
    dc = np.arange(-(1 << 16), 1 << 16, dtype=np.int64)
    full = ((dc << 11) + 128) >> 8
    assert np.array_equal(full, dc << 3)


def test_jpeg_vs_png_sanity():
    """Loose absolute check (JPEG pixels are otherwise unpinned): the JPEG and PNG of
    the same frame agree within 4 LSB (the survey's measured bound)."""
    a = O.jpeg_decode(read("testdata", "video-001.jpeg")).rgba_pixels().astype(int)
    p = O.png_decode(read("testdata", "video-001.png")).rgba_pixels().astype(int)
    assert np.abs(a - p).max() <= 4


@pytest.mark.parametrize("bpp", [1, 2, 4, 8, 24, 32])
@pytest.mark.parametrize("header", [40, 124])
def test_bmp_synthetic_vs_pillow(bpp, header):
    """The oracle's bmp.decode on generated files agrees with Pillow's reader
    (rgbaPixels premultiplies; Pillow keeps straight alpha)."""
    from PIL import Image
    import io
    from tools import synthetic as S

    for w, h, td in [(1, 1, False), (5, 3, True), (67, 9, False)]:
        data, _ = S.bmp_bytes(w + bpp, w, h, bpp, top_down=td, header=header,
                              bitfields=header > 40 and bpp == 32)
        try:
            ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGBA"))
        except Exception:
            pytest.skip(f"Pillow does not read {bpp} bpp")
        img = O.bmp_decode(data)
        a = ref[..., 3:4].astype(np.uint32)
        pm = ((ref[..., :3].astype(np.uint32) * 0x101 * a) // 0xFF) >> 8
        want = np.concatenate([pm.astype(np.uint8), ref[..., 3:4]], -1)
        assert np.array_equal(img.rgba_pixels().reshape(h, w, 4), want), (w, h, td)
