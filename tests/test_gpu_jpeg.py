"""GPU parity of the JPEG pixel path (jpeg_planar_kernel, jpeg_rgba_kernel,
convertToRGB / applyBlack kernels) against the CPU oracle, bit-exact.

Sizes are ones the oracle finishes in seconds; the 4096^2 bench frame is
checked against the oracle once (both sides are deterministic integer code).
"""
import ctypes as C
import glob
import os

import numpy as np
import pytest

import oracle_py as O
from conftest import golden, read
from tools import synthetic as S

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import zpix_amd  # noqa: E402
from zpix_amd import _lib, device  # noqa: E402
from zpix_amd import jpeg as J  # noqa: E402

JPEGS = sorted(glob.glob(golden("testdata", "*.jpeg"))) + [golden("testdata", "iceberg.jpg")]


def _oracle_or_error(data):
    try:
        return O.jpeg_decode(data), None
    except O.OracleError as e:
        return None, e.name


def assert_same_image(got, want):
    assert got.kind == want.kind
    assert tuple(got.rect) == tuple(want.rect)
    if want.kind == "YCbCr":
        assert (got.y_stride, got.c_stride, got.cb_off, got.cr_off, got.subsample) == (
            want.y_stride, want.c_stride, want.cb_off, want.cr_off, want.subsample)
    else:
        assert got.stride == want.stride
    assert got.pixels.size == want.pixels.size
    assert np.array_equal(got.pixels, want.pixels)


@pytest.mark.parametrize("path", JPEGS, ids=os.path.basename)
def test_jpeg_decode_planes_match_oracle(path):
    data = open(path, "rb").read()
    want, err = _oracle_or_error(data)
    if err:
        with pytest.raises(zpix_amd.ZpixError) as ei:
            J.decode(data)
        assert ei.value.name == err
        return
    assert_same_image(J.decode(data), want)


@pytest.mark.parametrize("path", JPEGS, ids=os.path.basename)
def test_jpeg_decode_rgba_matches_oracle(path):
    data = open(path, "rb").read()
    want, err = _oracle_or_error(data)
    if err:
        return
    got = J.decode_rgba(data)
    assert np.array_equal(got.reshape(-1), want.rgba_pixels())


def test_jpeg_load_and_facade():
    p = golden("testdata", "video-001.q50.422.jpeg")
    want = O.jpeg_decode(read("testdata", "video-001.q50.422.jpeg"))
    assert_same_image(J.load(p), want)
    assert_same_image(zpix_amd.from_file_path(p), want)
    assert J.probe_path(p)


SYNTH = [
    ("420", 2, 333, 177), ("444", 0, 129, 65), ("422", 1, 250, 99), ("420", 2, 17, 9),
    ("420", 2, 1, 1), ("444", 0, 8, 8), ("420", 2, 512, 384),
]


@pytest.mark.parametrize("name,sub,w,h", SYNTH)
@pytest.mark.parametrize("progressive", [False, True])
def test_jpeg_synthetic_sizes(name, sub, w, h, progressive):
    data = S.jpeg_subsampled(w * 7 + h, w, h, sub, quality=80, progressive=progressive)
    want = O.jpeg_decode(data)
    assert_same_image(J.decode(data), want)
    assert np.array_equal(J.decode_rgba(data).reshape(-1), want.rgba_pixels())


@pytest.mark.parametrize("progressive", [False, True])
def test_jpeg_gray_synthetic(progressive):
    data = S.jpeg_gray(5, 203, 77, progressive=progressive)
    want = O.jpeg_decode(data)
    assert_same_image(J.decode(data), want)
    assert np.array_equal(J.decode_rgba(data).reshape(-1), want.rgba_pixels())


def test_jpeg_errors_match_oracle():
    b = read("testdata", "video-005.gray.q50.jpeg")
    i = b.index(b"\xff\xda") + 2
    with pytest.raises(zpix_amd.ZpixError) as ei:
        J.decode(b[:i + 3])
    assert ei.value.name == "UnexpectedEof"
    r = read("testdata", "video-001.restart2.jpeg")
    with pytest.raises(zpix_amd.ZpixError) as ei:
        J.decode(r[:2816] + b"\xff\xd5" + r[2816:])
    assert ei.value.name == "BadRSTMarker"
    assert_same_image(J.decode(r[:2816] + b"\xff\xff\xff\x00\xff\x00\x00\xff\xff\xff" + r[2816:]),
                      O.jpeg_decode(r[:2816] + b"\xff\xff\xff\x00\xff\x00\x00\xff\xff\xff" + r[2816:]))


# ------------------------------------------------------------ kernel level
def _run_planar_grids(grids, qts, h, v, mxx, myy, width, height, rule, coeff_bits, narrow):
    """Launch a one-frame planar plan on raw coefficient grids (device)."""
    n_comp = len(grids)
    f = _lib.zpx_jpeg_frame()
    f.width, f.height, f.n_comp, f.mxx, f.myy = width, height, n_comp, mxx, myy
    f.coeff_bits, f.narrow, f.color = coeff_bits, narrow, 0
    keep = []
    planes = []
    npt = {8: np.int8, 16: np.int16, 32: np.int32}[coeff_bits]
    for c in range(n_comp):
        f.h[c], f.v[c], f.rule[c] = h[c], v[c], rule
        g = torch.from_numpy(np.ascontiguousarray(grids[c]).astype(npt)).to("cuda")
        keep.append(g)
        f.coeffs[c] = g.data_ptr()
        for i in range(64):
            f.qt[c][i] = int(qts[c][i])
        gw, gh = mxx * h[c], myy * v[c]
        p = torch.zeros(gw * 8 * gh * 8, dtype=torch.uint8, device="cuda")
        planes.append(p)
        f.planes[c] = p.data_ptr()
        f.strides[c] = gw * 8
    ctx = zpix_amd.context.default()
    hp = C.c_void_p()
    _lib.check(_lib.lib().zpx_jpeg_plan_create(ctx.handle, C.byref(f), 1, 0, C.byref(hp)), ctx.handle)
    plan = device._Plan(hp, ctx)
    plan.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    plan.close()
    return [p.cpu().numpy() for p in planes]


UNZIG = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27,
                  20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58,
                  59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])


@pytest.mark.parametrize("coeff_bits,scale,narrow,rule", [
    (16, 64, 1, 0), (16, 2000, 0, 0), (32, 1 << 20, 0, 0), (32, 1 << 27, 0, 1), (16, 300, 1, 2),
    (8, 128, 1, 0), (8, 128, 0, 1), (8, 128, 1, 2), (8, 128, 1, 1), (16, 300, 1, 1),
])
@pytest.mark.parametrize("geom", ["7x5", "70x3"])
@pytest.mark.parametrize("kernel", ["block", "strip"])
def test_planar_kernel_random_grids(coeff_bits, scale, narrow, rule, geom, kernel):
    """Random (incl. overflowing) coefficient grids: wrap-around i32 IDCT,
    DC-only shortcut and clamp must match the oracle bit for bit -- on the
    planar block kernel (narrow int8/int16 frames; 70 MCUs = 140 luma block
    columns: three 64-block tasks a row, the last ragged) and on the
    lane-per-row kernel the test switch "jpeg_strip" forces (what int32 and
    wide frames take)."""
    rng = np.random.default_rng(coeff_bits + scale)
    mxx, myy = (7, 5) if geom == "7x5" else (70, 3)
    h, v, width, height = [2, 1, 1], [2, 1, 1], mxx * 16 - 12, myy * 16 - 10
    prev = _lib.lib().zpx_debug_option(b"jpeg_strip", 1 if kernel == "strip" else 0)
    try:
        _planar_random_case(rng, coeff_bits, scale, narrow, rule, h, v, mxx, myy, width, height)
    finally:
        _lib.lib().zpx_debug_option(b"jpeg_strip", prev)


def _planar_random_case(rng, coeff_bits, scale, narrow, rule, h, v, mxx, myy, width, height):
    grids, qz = [], []
    for c in range(3):
        nb = mxx * h[c] * myy * v[c]
        lim = {8: 128, 16: 32767, 32: scale}[coeff_bits]
        g = rng.integers(-min(scale, lim), min(scale, lim), (nb, 64))
        sparse = rng.random((nb, 64)) < 0.7
        g[sparse] = 0
        g[rng.random(nb) < 0.2, 1:] = 0  # DC-only blocks
        grids.append(g.astype(np.int32))
        qz.append(rng.integers(1, 256 if narrow else 65535, 64).astype(np.int32))
    if narrow:  # keep max|coef*q| <= 16384 as the host would certify
        for c in range(3):
            grids[c] = np.clip(grids[c], -(16384 // 255), 16384 // 255)
    qnat = []
    for c in range(3):
        n = np.zeros(64, np.int32)
        n[UNZIG] = qz[c]
        qnat.append(n)
    got = _run_planar_grids(grids, qnat, h, v, mxx, myy, width, height, rule, coeff_bits, narrow)
    want = [np.zeros_like(p) for p in got]
    strides = [mxx * h[c] * 8 for c in range(3)]
    O.reconstruct_grids(3, width, height, h, v, mxx, myy, grids, qz, rule == 1, want, strides)
    if rule == 2:  # scan rule: blocks with bx*8>=W or by*8>=H stay untouched
        for c in range(3):
            gw = mxx * h[c]
            m = np.zeros((myy * v[c] * 8, gw * 8), bool)
            for by in range(myy * v[c]):
                for bx in range(gw):
                    if bx * 8 < width and by * 8 < height:
                        m[by * 8:by * 8 + 8, bx * 8:bx * 8 + 8] = True
            want[c] = np.where(m.reshape(-1), want[c], 0)
    for c in range(3):
        assert np.array_equal(got[c], want[c]), c


@pytest.mark.parametrize("coeff_bits", [8, 16])
def test_planar_kernel_low_frequency_tasks(coeff_bits):
    """The low-frequency path: a task whose 64 blocks are all
    zero outside the top-left 4x4 takes the short transform, any other the
    full one.  Every block here is low-frequency except one outlier per task
    at one of the 48 positions outside 4x4 (all 48 covered, per component),
    plus all-low-frequency tasks: a mask that missed a position would send
    its task down the short path and differ from the oracle."""
    rng = np.random.default_rng(77 + coeff_bits)
    mxx, myy = 70, 3
    h, v, width, height = [2, 1, 1], [2, 1, 1], mxx * 16, myy * 16
    outside = [r * 8 + c for r in range(8) for c in range(8) if r >= 4 or c >= 4]
    lim = 16384 // 255
    for rnd in range(8):
        grids, qz = [], []
        for c in range(3):
            gw, gh = mxx * h[c], myy * v[c]
            g = rng.integers(-lim, lim + 1, (gh, gw, 8, 8))
            g[:, :, 4:, :] = 0
            g[:, :, :, 4:] = 0
            # one outlier in every other 64-block task; positions walk `outside`
            tasks = [(by, x0) for by in range(gh) for x0 in range(0, gw, 64)]
            for t, (by, x0) in enumerate(tasks):
                if (t + rnd) % 2:
                    continue
                k = outside[(rnd * len(tasks) + t) % len(outside)]
                bx = x0 + int(rng.integers(0, min(64, gw - x0)))
                g[by, bx, k // 8, k % 8] = int(rng.integers(1, lim + 1)) * (1 if rng.random() < 0.5 else -1)
            grids.append(g.reshape(gh * gw, 64).astype(np.int32))
            qz.append(rng.integers(1, 256, 64).astype(np.int32))
        qnat = []
        for c in range(3):
            n = np.zeros(64, np.int32)
            n[UNZIG] = qz[c]
            qnat.append(n)
        got = _run_planar_grids(grids, qnat, h, v, mxx, myy, width, height, 0, coeff_bits, 1)
        want = [np.zeros_like(p) for p in got]
        strides = [mxx * h[c] * 8 for c in range(3)]
        O.reconstruct_grids(3, width, height, h, v, mxx, myy, grids, qz, False, want, strides)
        for c in range(3):
            assert np.array_equal(got[c], want[c]), (rnd, c)


def test_jpeg_batch_4k_fused_matches_oracle():
    """The bench workload (4096^2 4:2:0, q75) for one frame, slot-replicated."""
    data = S.jpeg_420(0, 4096, 4096)
    co = J.Coefficients(data)
    # the bench content fits int8 coefficients (max |coef| 75), so this is the
    # int8 transport the bench measures
    assert co.frame.narrow == 1 and co.frame.coeff_bits == 8
    batch = device.JpegBatch([co], slots=[0, 0], output="rgba")
    batch.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    want = O.jpeg_decode(data).rgba_pixels().reshape(4096, 4096, 4)
    for s in range(2):
        assert torch.equal(batch.output_tensor(s).cpu(), torch.from_numpy(want))
    assert batch.bytes == 2 * (393216 * 64 + 4096 * 4096 * 4 + 3 * 256)
    # the same frame through the int16 transport (bench's int16_transport line)
    del batch
    co.widen(16)
    assert co.frame.coeff_bits == 16
    batch = device.JpegBatch([co], slots=[0], output="rgba")
    batch.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(batch.output_tensor(0).cpu(), torch.from_numpy(want))
    assert batch.bytes == 393216 * 128 + 4096 * 4096 * 4 + 3 * 256


def test_jpeg_4k_strip_kernel_matches_oracle():
    """A 4094-wide 4:2:0 frame (width % 4 != 0: the block kernel's edge
    tasks; bench line "odd_width"), and the bench frame on the strip kernel,
    which the test switch "jpeg_strip" forces (the bench's
    odd_width.strip_kernel line does the same)."""
    from zpix_amd import _lib

    data = S.jpeg_420(5, 4094, 4096)
    co = J.Coefficients(data)
    batch = device.JpegBatch([co], slots=[0], output="rgba")
    batch.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    want = O.jpeg_decode(data).rgba_pixels().reshape(4096, 4094, 4)
    assert torch.equal(batch.output_tensor(0).cpu(), torch.from_numpy(want))
    del batch
    data = S.jpeg_420(0, 4096, 4096)
    co = J.Coefficients(data)
    prev = _lib.lib().zpx_debug_option(b"jpeg_strip", 1)
    try:
        batch = device.JpegBatch([co], slots=[0], output="rgba")
        batch.launch(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        _lib.lib().zpx_debug_option(b"jpeg_strip", prev)
    want = O.jpeg_decode(data).rgba_pixels().reshape(4096, 4096, 4)
    assert torch.equal(batch.output_tensor(0).cpu(), torch.from_numpy(want))


def test_jpeg_batch_planes_matches_oracle():
    data = S.jpeg_420(3, 640, 480)
    co = J.Coefficients(data)
    batch = device.JpegBatch([co], output="planes")
    batch.launch()
    torch.cuda.synchronize()
    want = O.jpeg_decode(data)
    got = batch.output_tensor(0).cpu().numpy()
    assert np.array_equal(got, want.pixels)


def test_jpeg_batch_planes_ragged_geometries():
    """One planes plan over frames of different sizes and samplings (one
    planar launch per geometry group, ragged MCU grids inside a group),
    baseline and progressive, int8 and int16 transports."""
    datas = [S.jpeg_subsampled(11, 333, 177, 2), S.jpeg_subsampled(12, 1030, 70, 2),
             S.jpeg_subsampled(13, 129, 65, 0, progressive=True), S.jpeg_subsampled(14, 250, 99, 1),
             S.jpeg_gray(15, 203, 77), S.jpeg_subsampled(16, 17, 9, 2, progressive=True)]
    for bits in (8, 16):
        cos = [J.Coefficients(d) for d in datas]
        for co in cos:
            co.widen(bits)
        batch = device.JpegBatch(cos, slots=[0, 1, 2, 3, 4, 5, 1, 0], output="planes")
        batch.launch(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        for s, i in enumerate(batch.slots):
            want = O.jpeg_decode(datas[i])
            assert np.array_equal(batch.output_tensor(s).cpu().numpy(), want.pixels), (bits, s)


@pytest.mark.parametrize("bits", [8, 16])
def test_jpeg_batch_4k_planes_matches_oracle(bits):
    """jpeg.load's planes of the bench frame (4096^2 4:2:0 q75, the bench's
    "planar" line) on the planar block kernel, both transports."""
    data = S.jpeg_420(0, 4096, 4096)
    co = J.Coefficients(data)
    co.widen(bits)
    batch = device.JpegBatch([co], slots=[0, 0], output="planes")
    batch.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    want = torch.from_numpy(O.jpeg_decode(data).pixels)
    for s in range(2):
        assert torch.equal(batch.output_tensor(s).cpu(), want)
    assert batch.bytes == 2 * (393216 * 64 * (bits // 8) + 393216 * 64 + 3 * 256)


def test_jpeg_progressive_444_4k_matches_oracle():
    """configs[4] JPEG at its bench size: a 4096^2 progressive 4:4:4 frame
    (786,432 blocks, reconstructProgressiveImage's block rule) through the
    fused kernel, bit-exact against the oracle's jpeg.decode + rgbaPixels."""
    data = S.jpeg_progressive_444(1000, 4096, 4096)
    co = J.Coefficients(data)
    batch = device.JpegBatch([co], slots=[0, 0], output="rgba")
    batch.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    want = torch.from_numpy(O.jpeg_decode(data).rgba_pixels().reshape(4096, 4096, 4))
    for s in range(2):
        assert torch.equal(batch.output_tensor(s).cpu(), want)
