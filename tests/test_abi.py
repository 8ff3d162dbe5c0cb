"""CPU-side checks of the drop-in boundary and the host (serial) stages.

- libzpix_amd.so loads and exports every function include/zpix_amd.h declares;
- error codes map 1:1 onto the reference's error names;
- the product's host JPEG entropy stage produces the oracle's coefficient
  grids for every fixture (and the same error names for malformed input);
- the product's host PNG stage (chunks, CRC, inflate, filter-byte checks)
  yields the exact filtered stream and the reference's error names.
No compute kernel runs here (no GPU in this container).
"""
import glob
import os
import re
import struct
import zlib

import numpy as np
import pytest

import oracle_py as O
from conftest import ROOT, golden, read
from tools import synthetic as S

zpix_amd = pytest.importorskip("zpix_amd")
from zpix_amd import _lib  # noqa: E402
from zpix_amd import jpeg as J  # noqa: E402
from zpix_amd import png as P  # noqa: E402

HEADER = os.path.join(ROOT, "include", "zpix_amd.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zpx_[a-z0-9_]+)\s*\(", src)))


def test_header_declarations_match_exports():
    assert declared_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), name


def test_error_names_match_reference():
    L = _lib.lib()
    assert L.zpx_error_name(0) == b"Ok"
    names = [L.zpx_error_name(i).decode() for i in range(80)]
    for ref_name in ["UnexpectedEof", "InvalidSOIMarker", "BadRSTMarker", "MissingFF00", "BadHuffmanCode",
                     "InvalidFilterType", "InvalidChecksum", "EmptyIdatData", "InvalidPngHeader",
                     "InvalidColorTypeDepthCombo", "UnsupportedMarker"]:
        assert ref_name in names, ref_name
    # the oracle uses the same names for the shared prefix of codes
    for i in range(1, 66):
        assert names[i] == O.error_name(i)


def test_ctx_create_without_gpu_fails_cleanly():
    import ctypes as C

    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = C.c_void_p()
    assert _lib.lib().zpx_ctx_create(0, C.byref(h)) == list(map(bytes.decode, [_lib.lib().zpx_error_name(i) for i in range(80)])).index("Hip")


JPEGS = sorted(glob.glob(golden("testdata", "*.jpeg"))) + [golden("testdata", "iceberg.jpg")]


@pytest.mark.parametrize("path", JPEGS, ids=os.path.basename)
def test_host_entropy_matches_oracle(path):
    data = open(path, "rb").read()
    try:
        oc = O.jpeg_coefficients(data)
    except O.OracleError as e:
        with pytest.raises(_lib.ZpixError) as ei:
            J.Coefficients(data)
        assert ei.value.name == e.name
        return
    pc = J.Coefficients(data)
    f = pc.frame
    assert (f.width, f.height, f.n_comp, f.mxx, f.myy) == (oc.width, oc.height, oc.n_comp, oc.mxx, oc.myy)
    for c in range(oc.n_comp):
        assert (f.h[c], f.v[c]) == (oc.h[c], oc.v[c])
        g = pc.grid(c)
        if oc.grids[c] is None:
            assert g is None
        else:
            assert np.array_equal(oc.grids[c], g.astype(np.int32))
            # quant table used for reconstruction, natural order
            unzig = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27,
                     20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58,
                     59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63]
            nat = np.zeros(64, np.int32)
            nat[unzig] = oc.quant_zigzag[oc.tq[c]]
            assert np.array_equal(np.array(f.qt[c][:]), nat)


@pytest.mark.parametrize("path", JPEGS, ids=os.path.basename)
def test_host_coefficient_width_is_narrowest(path):
    """The frame's coefficient grids share the narrowest of int8/int16/int32
    that holds every coefficient of every component."""
    data = open(path, "rb").read()
    try:
        oc = O.jpeg_coefficients(data)
    except O.OracleError:
        return
    m = max(int(np.abs(g).max()) for g in oc.grids if g is not None)
    want = 8 if m <= 127 else 16 if m <= 32767 else 32
    pc = J.Coefficients(data)
    assert pc.frame.coeff_bits == want
    for c in range(oc.n_comp):
        if oc.grids[c] is not None:
            assert pc.grid(c).dtype == {8: np.int8, 16: np.int16, 32: np.int32}[want]
            assert pc.coeff_bytes[c] == oc.grids[c].size * want // 8


@pytest.mark.parametrize("block", range(3))
def test_host_entropy_random(block):
    """The host entropy stage (processSos / Huffman / refinement,
    decoder.zig) on 40 random JPEGs a block, seeded: sizes 1-299, qualities
    5-100, baseline and progressive, 4:4:4 / 4:2:2 / 4:2:0 / gray, with and
    without restart intervals (the restart-parallel scan path) -- every
    grid, the frame geometry and the narrowest transport width as the
    oracle's, or the oracle's error name where the reference refuses the
    stream."""
    import io

    from PIL import Image

    rng = np.random.default_rng(5000 + block)
    for _ in range(40):
        w, h = int(rng.integers(1, 300)), int(rng.integers(1, 300))
        gray = rng.random() < 0.15
        kw = dict(quality=int(rng.integers(5, 101)), progressive=bool(rng.integers(2)))
        if not gray:
            kw["subsampling"] = int(rng.integers(3))
        if rng.random() < 0.4:
            kw["restart_marker_blocks"] = int(rng.integers(1, 40))
        px = S.content(int(rng.integers(1 << 30)), w, h, 1 if gray else 3)
        b = io.BytesIO()
        Image.fromarray(px[..., 0] if gray else px).save(b, "JPEG", **kw)
        data = b.getvalue()
        case = (w, h, gray, kw)
        try:
            oc = O.jpeg_coefficients(data)
        except O.OracleError as e:  # the reference's error, by name
            assert _jpeg_err_product(data) == e.name, case
            continue
        pc = J.Coefficients(data)
        f = pc.frame
        assert (f.width, f.height, f.n_comp, f.mxx, f.myy) == (oc.width, oc.height, oc.n_comp, oc.mxx, oc.myy), case
        m = max(int(np.abs(g).max()) for g in oc.grids if g is not None)
        assert f.coeff_bits == (8 if m <= 127 else 16 if m <= 32767 else 32), case
        for c in range(oc.n_comp):
            assert (f.h[c], f.v[c]) == (oc.h[c], oc.v[c]), case
            assert np.array_equal(oc.grids[c], pc.grid(c).astype(np.int32)), (case, c)


def _jpeg_err_product(data):
    try:
        J.Coefficients(data)
        return "OK"
    except _lib.ZpixError as e:
        return e.name


def test_host_entropy_error_cases():
    b = read("testdata", "video-005.gray.q50.jpeg")
    i = b.index(b"\xff\xda") + 2
    for k in range(i, min(i + 10, len(b))):
        assert _jpeg_err_product(b[:k]) == "UnexpectedEof"
    assert _jpeg_err_product(read("testdata", "large_short.jpeg")) == "UnexpectedEof"
    assert _jpeg_err_product(read("testdata", "video-001.jpeg")[:24]) == "UnexpectedEof"
    r = read("testdata", "video-001.restart2.jpeg")
    for infix, want in [(b"", "OK"), (b"\x61\x62\x63\xff\x00\x64", "OK"), (b"\xff\xff\xff\x00\xff\x00\x00\xff\xff\xff", "OK"),
                        (b"\xff\x03", "BadRSTMarker"), (b"\xff\xd5", "BadRSTMarker"), (b"\xff\xff\xd5", "BadRSTMarker")]:
        assert _jpeg_err_product(r[:2816] + infix + r[2816:]) == want


def _dri_jpegs():
    """Baseline JPEGs with restart intervals: the reference's restart2
    fixture and Pillow encodes (restart every N MCUs / every row)."""
    import io

    from PIL import Image
    from tools import synthetic as S

    out = [("restart2", read("testdata", "video-001.restart2.jpeg"))]
    for name, sub, w, h, kw in [("420_b7", 2, 264, 120, {"restart_marker_blocks": 7}),
                                ("444_b1", 0, 96, 40, {"restart_marker_blocks": 1}),
                                ("422_rows", 1, 200, 72, {"restart_marker_rows": 1}),
                                ("gray_b5", None, 120, 56, {"restart_marker_blocks": 5})]:
        b = io.BytesIO()
        px = S.content(w * 3 + h, w, h)
        if sub is None:
            Image.fromarray(px[..., 0]).save(b, "JPEG", quality=85, **kw)
        else:
            Image.fromarray(px).save(b, "JPEG", quality=85, subsampling=sub, **kw)
        out.append((name, b.getvalue()))
    return out


def test_host_entropy_restart_parallel_matches_oracle(monkeypatch):
    """Restart-interval-parallel Huffman (jpeg_host.cpp restart_parallel,
    splitting at decoder.zig:1432-1452): the same coefficients as the serial
    oracle on every DRI file, the same error names on corrupted segments, and
    the parallel path actually taken on the clean files."""
    monkeypatch.setenv("ZPX_HUFF_PAR_MIN_MCUS", "1")  # small files still split
    L = _lib.lib()
    for name, data in _dri_jpegs():
        before = L.zpx_debug_jpeg_parallel_scans()
        oc = O.jpeg_coefficients(data)
        pc = J.Coefficients(data)
        assert L.zpx_debug_jpeg_parallel_scans() == before + 1, name
        for c in range(oc.n_comp):
            assert np.array_equal(oc.grids[c], pc.grid(c).astype(np.int32)), (name, c)
        m = max(int(np.abs(g).max()) for g in oc.grids if g is not None)
        assert pc.frame.coeff_bits == (8 if m <= 127 else 16), name  # narrowest width, as serially
    # corrupted segments: every outcome equals the oracle's (serial fallback)
    r = read("testdata", "video-001.restart2.jpeg")
    for infix in [b"", b"\x61\x62\x63\xff\x00\x64", b"\xff\xff\xff\x00\xff\x00\x00\xff\xff\xff",
                  b"\xff\x03", b"\xff\xd5", b"\xff\xff\xd5"]:
        data = r[:2816] + infix + r[2816:]
        try:
            oc = O.jpeg_coefficients(data)
        except O.OracleError as e:
            assert _jpeg_err_product(data) == e.name
            continue
        pc = J.Coefficients(data)
        for c in range(oc.n_comp):
            assert np.array_equal(oc.grids[c], pc.grid(c).astype(np.int32))
    rng = np.random.default_rng(3)
    srcs = [d for _, d in _dri_jpegs()]
    for it in range(40):
        d = bytearray(srcs[it % len(srcs)])
        for _ in range(rng.integers(1, 3)):
            d[rng.integers(len(d) // 4, len(d))] = rng.integers(0, 256)
        data = bytes(d)
        try:
            oc = O.jpeg_coefficients(data)
        except O.OracleError as e:
            assert _jpeg_err_product(data) == e.name
            continue
        pc = J.Coefficients(data)
        for c in range(oc.n_comp):
            if oc.grids[c] is not None:
                assert np.array_equal(oc.grids[c], pc.grid(c).astype(np.int32))


def test_host_entropy_fuzz_matches_oracle():
    """Random byte corruption of fixtures: same coefficients or same error name."""
    rng = np.random.default_rng(7)
    srcs = [read("testdata", n) for n in ("video-001.q50.420.jpeg", "video-001.q50.420.progressive.jpeg",
                                          "video-001.restart2.jpeg", "video-005.gray.q50.jpeg")]
    for it in range(60):
        d = bytearray(srcs[it % len(srcs)])
        for _ in range(rng.integers(1, 4)):
            d[rng.integers(0, len(d))] = rng.integers(0, 256)
        data = bytes(d)
        try:
            oc = O.jpeg_coefficients(data)
        except O.OracleError as e:
            assert _jpeg_err_product(data) == e.name
            continue
        pc = J.Coefficients(data)
        for c in range(oc.n_comp):
            if oc.grids[c] is not None:
                assert np.array_equal(oc.grids[c], pc.grid(c).astype(np.int32))


def _idat_stream(png_bytes):
    pos, z = 8, b""
    while pos < len(png_bytes):
        n = struct.unpack(">I", png_bytes[pos:pos + 4])[0]
        if png_bytes[pos + 4:pos + 8] == b"IDAT":
            z += png_bytes[pos + 8:pos + 8 + n]
        pos += 12 + n
    return zlib.decompress(z)


PNGS = sorted(glob.glob(golden("pngsuite", "*.png"))) + sorted(glob.glob(golden("testdata", "*.png")))


@pytest.mark.parametrize("path", PNGS, ids=os.path.basename)
def test_host_inflate_stream(path):
    data = open(path, "rb").read()
    st = P.Stream(data)
    want = _idat_stream(data)
    got = st.filtered()[:st.filtered_len]
    assert bytes(got) == want[:st.filtered_len]


def _png_err_product(data):
    try:
        P.Stream(data)
        return "OK"
    except _lib.ZpixError as e:
        return e.name


def _png_err_oracle(data):
    try:
        O.png_decode(data)
        return "OK"
    except O.OracleError as e:
        return e.name


def test_host_png_errors_match_oracle():
    base = S.png_generic(3, 37, 21, 8, 2)
    cases = [base[:20], base[:-5], b"\x89PNX" + base[4:]]
    # bad CRC of IHDR
    bad_crc = bytearray(base)
    bad_crc[29] ^= 0xFF
    cases.append(bytes(bad_crc))
    # invalid filter type in row 3
    raw = np.frombuffer(_idat_stream(base), np.uint8).copy().reshape(21, -1)
    raw[3, 0] = 7
    cases.append(S.encode_png(37, 21, 8, 2, raw.tobytes()))
    # truncated zlib stream
    cases.append(S.encode_png(37, 21, 8, 2, raw.tobytes()[: raw.size // 2]))
    # bad colour type / depth combination
    cases.append(S.encode_png(5, 5, 4, 2, b"\x00" * 100))
    rng = np.random.default_rng(11)
    for _ in range(40):
        d = bytearray(base)
        d[rng.integers(8, len(d))] ^= 1 << int(rng.integers(0, 8))
        cases.append(bytes(d))
    for d in cases:
        want = _png_err_oracle(d)
        got = _png_err_product(d)
        assert got == want, (got, want)


def _png_single(data):
    """(status, frame fields, filtered bytes) of zpx_png_inflate."""
    import ctypes as C

    L = _lib.lib()
    h = C.c_void_p()
    rc = L.zpx_png_inflate(data, len(data), C.byref(h))
    if rc:
        return rc, None, None
    try:
        return 0, *_png_stream_view(h)
    finally:
        L.zpx_png_stream_free(h)


def _png_stream_view(h):
    import ctypes as C

    L = _lib.lib()
    f, n = _lib.zpx_png_frame(), C.c_size_t(0)
    _lib.check(L.zpx_png_stream_frame(h, C.byref(f), C.byref(n)))
    fields = (f.width, f.height, f.depth, f.interlace, f.use_transparent, bytes(f.transparent), f.out_stride, n.value)
    ptr = L.zpx_png_stream_data(h)
    return fields, bytes(np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(n.value,)))


def _png_pair_cases():
    cases = [open(p, "rb").read() for p in PNGS]
    base = S.png_generic(3, 37, 21, 8, 2)
    raw = np.frombuffer(_idat_stream(base), np.uint8).copy().reshape(21, -1)
    bad_filter = raw.copy()
    bad_filter[3, 0] = 7
    cases += [base[:20], base[:-5], S.encode_png(37, 21, 8, 2, bad_filter.tobytes()),
              S.encode_png(37, 21, 8, 2, raw.tobytes()[: raw.size // 2])]
    # an IDAT run, another chunk, a second IDAT run (the second one is the image)
    z1, z2 = zlib.compress(raw.tobytes()[:100]), zlib.compress(raw.tobytes())
    ch = lambda t, d: struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)  # noqa: E731
    head = base[:33]
    cases += [head + ch(b"IDAT", z1) + ch(b"tEXt", b"k\x00v") + ch(b"IDAT", z2) + ch(b"IEND", b""),
              head + ch(b"IDAT", z2) + ch(b"tEXt", b"k\x00v") + ch(b"IDAT", z1) + ch(b"IEND", b"")]
    # a bad CRC after the image data (the image's own error ranks first when it has one)
    good = S.png_generic(5, 300, 200, 8, 2, interlace=1)
    cases += [good[:-4] + b"\x00\x00\x00\x00", S.encode_png(37, 21, 8, 2, bad_filter.tobytes())[:-4] + b"\x00" * 4]
    # larger streams: the fast zones of both run side by side
    cases += [S.png_tc8_mixed(7, 700, 300), S.png_generic(8, 513, 257, 16, 6, interlace=1),
              S.png_generic(9, 640, 480, 8, 0)]
    rng = np.random.default_rng(11)
    for _ in range(6):
        d = bytearray(cases[-3])
        d[rng.integers(40, len(d))] ^= 1 << int(rng.integers(0, 8))
        cases.append(bytes(d))
    # corrupted zlib data behind valid CRCs (the inflate's own errors)
    _, f = S.png_filtered_tc8(4, 400, 160)
    z = zlib.compress(f.tobytes())
    head = S.encode_png(400, 160, 8, 2, b"")[:33]
    for i in range(16):  # (half of them in the first block's header: code sets, invalid codes)
        zz = bytearray(z)
        zz[rng.integers(2, 40 if i % 2 else len(zz))] ^= 1 << int(rng.integers(0, 8))
        cases.append(head + ch(b"IDAT", bytes(zz)) + ch(b"IEND", b""))
    return cases


def test_png_inflate_pair_matches_single():
    """A batch worker's two-PNG host stage (png_parse_pair: the chunk walks
    deferred past IDAT, both inflates in one loop) gives each image
    zpx_png_inflate's status, frame and bytes: every fixture, truncated and
    corrupted streams, a second IDAT run, a chunk error after the image."""
    import ctypes as C

    L = _lib.lib()
    cases = _png_pair_cases()
    single = [_png_single(d) for d in cases]
    pairs = [(i, (i + 1) % len(cases)) for i in range(len(cases))] + [(i, i) for i in range(0, len(cases), 7)]
    pairs += [(i, len(cases) - 1 - i) for i in range(len(cases) // 2)]
    for a, b in pairs:
        h0, h1, st = C.c_void_p(), C.c_void_p(), (C.c_int * 2)()
        _lib.check(L.zpx_debug_png_inflate_pair(cases[a], len(cases[a]), cases[b], len(cases[b]), C.byref(h0),
                                                C.byref(h1), st))
        for k, (idx, h) in enumerate(((a, h0), (b, h1))):
            want = single[idx]
            assert st[k] == want[0], (a, b, k, _lib.error_name(st[k]), _lib.error_name(want[0]))
            if want[0] == 0:
                assert h.value
                assert _png_stream_view(h) == want[1:], (a, b, k)
                L.zpx_png_stream_free(h)
            else:
                assert not h.value


# ---------------------------------------------------------------- decodeConfig
def test_jpeg_decode_config_matches_decode():
    """jpeg.decodeConfig (decoder.zig:178-218): dims of every fixture equal the
    full decode's; 1 component -> Gray, 3 or 4 -> YCbCr (the reference's TODO)."""
    for p in sorted(glob.glob(golden("testdata", "*.jp*g"))):
        data = open(p, "rb").read()
        try:
            img = O.jpeg_decode(data)
        except O.OracleError:
            continue
        w, h, model = J.decode_config_model(data)
        assert (w, h) == (img.width, img.height), p
        assert model == ("Gray" if img.kind == "Gray" else "YCbCr"), p


def test_jpeg_decode_config_errors():
    with pytest.raises(zpix_amd.ZpixError) as e:
        J.decode_config(b"\x00\x01garbage")
    assert e.value.name == "InvalidSOIMarker"
    data = read("testdata", "video-001.q50.420.jpeg")
    with pytest.raises(zpix_amd.ZpixError) as e:
        J.decode_config(data[:20])
    assert e.value.name == "UnexpectedEof"


def test_png_decode_config():
    for p in sorted(glob.glob(golden("pngsuite", "*.png")))[:12]:
        data = open(p, "rb").read()
        img = O.png_decode(data)
        assert P.decode_config(data) == (img.width, img.height)
    with pytest.raises(zpix_amd.ZpixError) as e:
        P.decode_config(b"\x89PNX\r\n\x1a\n" + b"\x00" * 30)
    assert e.value.name == "InvalidPngHeader"


def _png_with_stream(w, h, z):
    """A gray8 PNG whose IDAT is the given zlib stream (split in 3 chunks)."""
    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)
    ihdr = struct.pack(">IIBBBBB", w, h, 8, 0, 0, 0, 0)
    k = max(1, len(z) // 3)
    idats = b"".join(chunk(b"IDAT", z[i:i + k]) for i in range(0, len(z), k))
    return b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + idats + chunk(b"IEND", b"")


@pytest.mark.parametrize("level,strategy", [(0, zlib.Z_DEFAULT_STRATEGY), (1, zlib.Z_DEFAULT_STRATEGY),
                                            (6, zlib.Z_DEFAULT_STRATEGY), (9, zlib.Z_DEFAULT_STRATEGY),
                                            (6, zlib.Z_FILTERED), (6, zlib.Z_HUFFMAN_ONLY), (6, zlib.Z_RLE),
                                            (6, zlib.Z_FIXED)])
def test_inflate_matches_zlib(level, strategy):
    """The host inflate (fast decoder, zlib fallback) gives zlib's bytes for
    stored, fixed and dynamic blocks, long matches and every strategy; and
    truncated / corrupted streams keep zlib's error names."""
    rng = np.random.default_rng(level * 10 + strategy)
    w, h = 333, 97
    rows = []
    for y in range(h):  # filter-type byte 0 + mixed noise / runs / repeats
        kind = y % 3
        if kind == 0:
            r = rng.integers(0, 256, w, dtype=np.uint8)
        elif kind == 1:
            r = np.repeat(rng.integers(0, 256, w // 37 + 1, dtype=np.uint8), 37)[:w]
        else:
            r = np.tile(rng.integers(0, 256, 7, dtype=np.uint8), w // 7 + 1)[:w]
        rows.append(b"\x00" + r.tobytes())
    raw = b"".join(rows)
    co = zlib.compressobj(level, zlib.DEFLATED, 15, 8, strategy)
    z = co.compress(raw) + co.flush()
    st = P.Stream(_png_with_stream(w, h, z))
    assert np.array_equal(st.filtered()[:st.filtered_len], np.frombuffer(raw, np.uint8))
    # truncation and corruption: the same error name as the oracle (zlib)
    for cut in (len(z) // 2, len(z) - 5):
        bad = _png_with_stream(w, h, z[:cut])
        try:
            O.png_decode(bad)
            want = "OK"
        except O.OracleError as e:
            want = e.name
        try:
            P.Stream(bad)
            got = "OK"
        except _lib.ZpixError as e:
            got = e.name
        assert got == want, (cut, got, want)
    for k in range(6):
        b = bytearray(z)
        b[int(rng.integers(2, len(b)))] ^= int(rng.integers(1, 256))
        bad = _png_with_stream(w, h, bytes(b))
        try:
            want = O.png_decode(bad).pixels.tobytes()[:0] or "OK"
        except O.OracleError as e:
            want = e.name
        try:
            P.Stream(bad)
            got = "OK"
        except _lib.ZpixError as e:
            got = e.name
        assert got == want, (k, got, want)


def _raw_qoi_decode(data: bytes):
    import ctypes as C

    from zpix_amd.image import Image

    raw = _lib.zpx_image()
    code = _lib.lib().zpx_qoi_decode(None, None, data, len(data), C.byref(raw))
    if code:
        return _lib.error_name(code), None
    return "Ok", Image._from_c(raw)


def test_qoi_decode_host_matches_oracle():
    """qoi.decode is a host loop (no context needed): same pixels and errors as the oracle."""
    import io

    from PIL import Image as PI

    rng = np.random.default_rng(0)
    for k, (w, h, ch) in enumerate([(1, 1, 4), (5, 3, 3), (64, 17, 4), (130, 40, 3)]):
        px = np.clip(128 + np.cumsum(rng.integers(-3, 3, (h, w, ch)), axis=1), 0, 255).astype(np.uint8)
        px[: h // 2, : w // 2] = px[0, 0]
        b = io.BytesIO()
        PI.fromarray(px, "RGBA" if ch == 4 else "RGB").save(b, format="QOI")
        for data in (O.qoi_encode(px, w, h, ch, 0), b.getvalue()):
            name, img = _raw_qoi_decode(data)
            want = O.qoi_decode(data)
            assert name == "Ok" and img.kind == "RGBA" and tuple(img.rect) == want.rect
            assert np.array_equal(img.pixels, want.pixels)
            # truncations: header errors, payload past the end (Panic) or a short image
            for cut in (0, 13, 21, 22, len(data) - 9, len(data) - 1):
                name, img = _raw_qoi_decode(data[:cut])
                try:
                    want = O.qoi_decode(data[:cut])
                    assert name == "Ok" and np.array_equal(img.pixels, want.pixels), cut
                except O.OracleError as e:
                    assert name == e.name, cut


def test_qoi_decode_host_wrapping_diff():
    """The product's host QOI decode wraps a qoi.h-style DIFF step mod 256, as
    the oracle does (tests/test_oracle.py::test_qoi_decode_wrapping_diff)."""
    import io

    from PIL import Image as PI

    px = np.array([[[255, 10, 10, 255], [0, 10, 10, 255], [1, 9, 255, 255], [255, 255, 0, 255]]], np.uint8)
    b = io.BytesIO()
    PI.fromarray(px, "RGBA").save(b, format="QOI")
    name, img = _raw_qoi_decode(b.getvalue())
    assert name == "Ok" and np.array_equal(img.pixels.reshape(1, 4, 4), px)


def test_bmp_header_errors_match_oracle():
    """bmp readHeader's errors (src/bmp/decoder.zig:42-158) come from the host
    parse, before any device work, so they are checked without a GPU."""
    import ctypes as C

    from tools import synthetic as S

    good, _ = S.bmp_bytes(1, 9, 4, 4, header=108)
    variants = [b"", b"BM", b"XM" + good[2:], good[:30]]
    for off, val in [(14, 12), (26, 2), (28, 16), (30, 1), (46, 17), (10, 99), (22, 0x80)]:
        v = bytearray(good)
        v[off] = val
        if off == 22:
            v[22:26] = (0x80000000).to_bytes(4, "little")
        variants.append(bytes(v))
    for data in variants:
        raw = _lib.zpx_image()
        code = _lib.lib().zpx_bmp_decode(None, None, data, len(data), C.byref(raw))
        with pytest.raises(O.OracleError) as e:
            O.bmp_decode(data)
        assert _lib.error_name(code) == e.value.name, data[:32]


def _sparse_grids(data: bytes, cap: int = 1 << 22):
    import ctypes as C

    out = np.zeros(cap, np.int32)
    n = _lib.lib().zpx_debug_jpeg_sparse_grids(data, len(data), out.ctypes.data, cap)
    return n, out


@pytest.mark.parametrize("quality", [75, 98])
@pytest.mark.parametrize("sub", [0, 1, 2])
def test_jpeg_pieces_match_oracle_grids(sub, quality):
    """The batch pipeline's compact coefficient upload (ZPX_COEFFS_PIECES,
    SURVEY §8(f)1): the zig-zag pieces a baseline interleaved scan emits,
    expanded with the device kernels' index -> block mapping, equal the
    oracle's coefficient grids (q98: int16 pieces)."""
    from tools import synthetic as S

    for seed, (w, h) in enumerate([(8, 8), (37, 21), (129, 67), (256, 200)]):
        data = S.jpeg_subsampled(seed, w, h, sub, quality)
        n, flat = _sparse_grids(data)
        assert n > 0, (sub, w, h)
        c = O.jpeg_coefficients(data)
        off = 0
        for i, g in enumerate(c.grids):
            g = np.asarray(g, np.int32).reshape(-1)
            assert np.array_equal(flat[off:off + g.size], g), (sub, w, h, i)
            off += g.size
        assert n * 64 == off


def _flat_then_busy(seed: int, w: int, h: int, quality: int) -> bytes:
    """A frame whose first rows are flat and whose last rows are noise: the
    pieces start int8 and widen to int16 part way through the scan."""
    import io

    from PIL import Image

    rng = np.random.default_rng(seed)
    img = np.full((h, w, 3), 128, np.uint8)
    img[h // 2:] = rng.integers(0, 256, (h - h // 2, w, 3), dtype=np.uint8)
    b = io.BytesIO()
    Image.fromarray(img).save(b, "JPEG", quality=quality, subsampling=2)
    return b.getvalue()


def test_jpeg_pieces_widen_midway():
    """Pieces written as int8 are widened to int16 when a later block needs
    it (JpegPieces::widen): same grids as the oracle, int16 width, and the
    layout's invariants (piece 0 zeros, every block's pieces inside the
    data) hold."""
    from zpix_amd import jpeg as J

    data = _flat_then_busy(5, 96, 160, 100)
    n, flat = _sparse_grids(data)
    c = O.jpeg_coefficients(data)
    want = np.concatenate([np.asarray(g, np.int32).reshape(-1) for g in c.grids])
    assert n * 64 == want.size and np.array_equal(flat[:want.size], want)
    co = J.Coefficients(data, pieces=True)
    assert co.is_pieces and co.frame.coeff_bits == 16
    raw = co.pieces_bytes()
    assert not raw[:16].any()
    for comp in range(3):
        ix = co.index(comp).astype(np.int64)
        n_p, first = ix & 15, ix >> 4
        assert ((n_p == 0) == (first == 0)).all()
        assert (first + n_p <= len(raw) // 16).all() and (n_p <= 8).all()
        assert np.array_equal(co.grid(comp).astype(np.int32).reshape(-1), np.asarray(c.grids[comp], np.int32).reshape(-1))


def test_jpeg_pieces_fall_back_to_grids():
    """Progressive, gray, non-interleaved and DRI-parallel frames take grids."""
    from tools import synthetic as S

    for data in (S.jpeg_progressive_444(1, 64, 48), S.jpeg_gray(2, 40, 40),
                 read("testdata", "video-001.progressive.jpeg")):
        n, _ = _sparse_grids(data)
        assert n == 0
    # a truncated file reports the reference's error, as the grid decoder does
    data = S.jpeg_420(3, 64, 64)
    n, _ = _sparse_grids(data[: len(data) // 2])
    assert n < 0


def _zstream(raw: bytes, level: int, strategy: int = 0, wbits: int = 15) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, wbits, 8, strategy)
    return c.compress(raw) + c.flush()


@pytest.mark.parametrize("threads", [1, 2, 3, 8])
def test_parallel_inflate_matches_zlib(threads):
    """The speculative multi-threaded inflate returns zlib's
    bytes whenever it accepts a stream; it accepts the usual PNG streams.
    threads = 1 is the serial fast decoder (literal-pair tables), which must
    accept every regular stream."""
    import ctypes as C

    rng = np.random.default_rng(threads)
    noise = (128 + rng.normal(0, 12, 3_000_000)).clip(0, 255).astype(np.uint8).tobytes()
    smooth = np.repeat(rng.integers(0, 256, 40_000, dtype=np.uint8), 60).tobytes()
    mixed = b"".join(noise[i:i + 50_000] + smooth[i:i + 70_000] for i in range(0, 2_000_000, 120_000))
    cases = [(noise, 6, 0), (smooth, 6, 0), (mixed, 9, 0), (mixed, 1, 0), (noise, 6, zlib.Z_FIXED),
             (mixed, 0, 0), (mixed, 6, zlib.Z_HUFFMAN_ONLY), (mixed, 6, zlib.Z_RLE)]
    accepted = 0
    for raw, level, strategy in cases:
        z = _zstream(raw, level, strategy)
        for want in (len(raw), len(raw) // 3):
            out = np.zeros(want + 64, np.uint8)
            ok = _lib.lib().zpx_debug_inflate_parallel(z, len(z), out.ctypes.data, want, threads)
            if ok:
                accepted += 1
                assert out[:want].tobytes() == raw[:want], (level, strategy, want)
        # a corrupted stream is never accepted with wrong bytes
        bad = bytearray(z)
        bad[len(z) // 2] ^= 0x55
        out = np.zeros(len(raw) + 64, np.uint8)
        if _lib.lib().zpx_debug_inflate_parallel(bytes(bad), len(bad), out.ctypes.data, len(raw), threads):
            # like the serial path, only the bytes the PNG reads are checked (no
            # Adler-32: the reader stops at the last byte it needs)
            try:
                ref = zlib.decompressobj(-15).decompress(bytes(bad[2:]))  # raw DEFLATE, no Adler-32
            except zlib.error:
                pytest.fail("accepted a stream whose first bytes zlib rejects")
            assert len(ref) >= len(raw) and out[:len(raw)].tobytes() == ref[:len(raw)]
    assert accepted >= (16 if threads == 1 else 8)  # dynamic-block streams decode in parallel


def _progressive_jpegs():
    """Progressive JPEGs: the reference's progressive fixtures
    (decoder.zig:1843-1920 pairs) and Pillow encodes of every subsampling,
    gray, ragged sizes."""
    import io

    from PIL import Image
    from tools import synthetic as S

    out = [(os.path.basename(p), open(p, "rb").read()) for p in JPEGS if "progressive" in os.path.basename(p)]
    for name, sub, w, h, q in [("420", 2, 333, 177, 80), ("444", 0, 129, 65, 95), ("422", 1, 250, 99, 30),
                               ("444_big", 0, 640, 480, 75), ("gray", None, 203, 77, 60), ("420_tiny", 2, 9, 7, 90)]:
        b = io.BytesIO()
        px = S.content(w * 5 + h, w, h)
        if sub is None:
            Image.fromarray(px[..., 0]).save(b, "JPEG", quality=q, progressive=True)
        else:
            Image.fromarray(px).save(b, "JPEG", quality=q, subsampling=sub, progressive=True)
        out.append((name, b.getvalue()))
    return out


def test_host_entropy_progressive_parallel_matches_oracle():
    """Scan-parallel progressive decoding (jpeg_host.cpp run_deferred_scans:
    the scans of processSos, decoder.zig:1148-1455 / refine :1459-1549, run
    concurrently in dependency order, checked against the serial loop's
    continuation): the oracle's coefficients on every progressive file, the
    parallel path actually taken there, and on truncated or corrupted
    streams -- which the check sends back to the serial loop -- the oracle's
    coefficients or error name."""
    from zpix_amd.shard import host_cpu_budget

    if int(os.environ.get("ZPX_HUFF_THREADS", min(8, host_cpu_budget()))) < 2:  # (jpeg_huff_threads)
        pytest.skip("one host thread: the serial loop decodes progressive scans")
    L = _lib.lib()
    srcs = _progressive_jpegs()
    for name, data in srcs:
        before = L.zpx_debug_jpeg_parallel_progressive()
        oc = O.jpeg_coefficients(data)
        pc = J.Coefficients(data)
        assert L.zpx_debug_jpeg_parallel_progressive() == before + 1, name
        for c in range(oc.n_comp):
            assert np.array_equal(oc.grids[c], pc.grid(c).astype(np.int32)), (name, c)
    rng = np.random.default_rng(11)
    for it in range(60):
        d = bytearray(srcs[it % len(srcs)][1])
        if it % 3 == 0:
            d = d[:int(rng.integers(len(d) // 3, len(d)))]  # truncated inside some scan
        else:
            for _ in range(rng.integers(1, 3)):
                d[rng.integers(len(d) // 4, len(d))] = rng.integers(0, 256)
        data = bytes(d)
        try:
            oc = O.jpeg_coefficients(data)
        except O.OracleError as e:
            assert _jpeg_err_product(data) == e.name, it
            continue
        pc = J.Coefficients(data)
        for c in range(oc.n_comp):
            if oc.grids[c] is not None:
                assert np.array_equal(oc.grids[c], pc.grid(c).astype(np.int32)), (it, c)


def test_batch_cache_trim_without_batches():
    """zpx_batch_cache_trim with nothing cached (no batch has run in this
    process without a GPU) returns 0 and touches no device."""
    assert _lib.lib().zpx_batch_cache_trim() == 0


def test_host_pools_trim():
    """zpx_host_pools_trim releases the host stages' recycled buffers: after
    a PNG parse the IDAT buffer is pooled (reused by the next parse with its
    pages), after a parallel inflate the symbol buffers; a trim returns
    their bytes, a second trim 0, and decoding afterwards is unchanged."""
    L = _lib.lib()
    L.zpx_host_pools_trim()
    data = S.png_tc8_mixed(3, 300, 200)
    rc, frame, got = _png_single(data)
    assert rc == 0
    assert L.zpx_host_pools_trim() > 0
    assert L.zpx_host_pools_trim() == 0
    rng = np.random.default_rng(5)
    raw = (128 + rng.normal(0, 12, 3_000_000)).clip(0, 255).astype(np.uint8).tobytes()
    z = _zstream(raw, 6, 0)
    out = np.zeros(len(raw) + 64, np.uint8)
    if _lib.lib().zpx_debug_inflate_parallel(z, len(z), out.ctypes.data, len(raw), 4):
        assert out[:len(raw)].tobytes() == raw
        assert L.zpx_host_pools_trim() > 0
    assert _png_single(data) == (rc, frame, got)


def test_jpeg_pieces_fixture_geometries():
    """Pieces of every baseline interleaved fixture, whatever its sampling
    (4:1:0, 4:1:1, 4:4:0, 2x2 luma with 1x2 chroma, ...): the per (component,
    block row mod v) streams (JpegPieces) compacted back to back -- every
    piece owned by exactly one block, checked by the hook -- expand to the
    oracle's coefficient grids."""
    import glob

    seen = 0
    for path in sorted(glob.glob(golden("testdata", "*.jp*g"))):
        data = open(path, "rb").read()
        try:
            c = O.jpeg_coefficients(data)
        except O.OracleError:
            continue
        n, flat = _sparse_grids(data, 1 << 24)
        if n <= 0:  # grids, not pieces (progressive, one component, restart-parallel...)
            continue
        seen += 1
        off = 0
        for i, g in enumerate(c.grids):
            g = np.asarray(g, np.int32).reshape(-1)
            assert np.array_equal(flat[off:off + g.size], g), (path, i)
            off += g.size
        assert n * 64 == off, path
    assert seen >= 10
