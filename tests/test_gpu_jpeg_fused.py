"""The fused RGBA JPEG kernels (block-per-lane and strip) on random coefficient grids.

Each case builds zpx_jpeg_frame descriptors over random device grids and runs
one ZPX_JPEG_RGBA plan through the C-ABI.  The expected RGBA comes from the
oracle: zo_jpeg_reconstruct_grids (reconstructBlock, decoder.zig:1553-1634)
into the reference's plane layout (makeImg, decoder.zig:1708-1783), then
zo_rgba_pixels over the YCbCr / Gray image (Image.rgbaPixels,
image.zig:103-130), or, for Adobe RGB frames, convertToRGB
(decoder.zig:751-783) restated below.  Dword-aligned rows of any width take
the block-per-lane kernel for int8/int16 "narrow" frames of its geometries;
every other case takes the strip kernel.  The batches mix frame
sizes (a ragged plan) and include never-scanned components.
"""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle_py as O  # noqa: E402
import zpix_amd  # noqa: E402
from zpix_amd import _lib, device  # noqa: E402

pytestmark = pytest.mark.gpu

UNZIG = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27,
                  20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58,
                  59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])
YCBCR, RGB, GRAY = 0, 1, 2
# subsample index of the oracle image by (h0/h1, v0/v1) (makeImg, decoder.zig:1740-1752)
SUB = {(1, 1): 0, (2, 1): 1, (2, 2): 2, (1, 2): 3, (4, 1): 4, (4, 2): 5}


def _frame_data(rng, geom, color, width, height, bits, narrow, absent=()):
    """Random grids (natural order, int32) + zigzag quant tables for one frame."""
    (h0, v0), (hc, vc) = geom
    n_comp = 1 if color == GRAY else 3
    h = [h0] + [hc] * (n_comp - 1)
    v = [v0] + [vc] * (n_comp - 1)
    if n_comp == 1:
        h, v = [1], [1]
    mxx = (width + 8 * h[0] - 1) // (8 * h[0])
    myy = (height + 8 * v[0] - 1) // (8 * v[0])
    grids, qz = [], []
    for c in range(n_comp):
        nb = mxx * h[c] * myy * v[c]
        if narrow:  # max|coef*q| <= 16384, the host's narrow certificate
            lim, qmax = 64, 256
        else:
            lim, qmax = {8: 127, 16: 32767, 32: 1 << 20}[bits], 65535
        g = rng.integers(-lim, lim + 1, (nb, 64))
        g[rng.random((nb, 64)) < 0.7] = 0
        g[rng.random(nb) < 0.2, 1:] = 0  # DC-only blocks
        grids.append(None if c in absent else g.astype(np.int32))
        qz.append(rng.integers(1, qmax, 64).astype(np.int32))
    return dict(width=width, height=height, n_comp=n_comp, h=h, v=v, mxx=mxx, myy=myy, grids=grids, qz=qz,
                bits=bits, narrow=narrow, color=color)


def _expected(fd):
    """Oracle RGBA (W*H*4) of one frame."""
    w_all = fd["mxx"] * fd["h"][0] * 8
    h_all = fd["myy"] * fd["v"][0] * 8
    W, H, n = fd["width"], fd["height"], fd["n_comp"]
    planes, strides = [], []
    for c in range(n):
        gw, gh = fd["mxx"] * fd["h"][c], fd["myy"] * fd["v"][c]
        planes.append(np.zeros(gw * 8 * gh * 8, np.uint8))
        strides.append(gw * 8)
    O.reconstruct_grids(n, W, H, fd["h"], fd["v"], fd["mxx"], fd["myy"], fd["grids"], fd["qz"], False, planes,
                        strides)
    if n == 1:
        img = O.ZoImage(kind=0, min_x=0, min_y=0, max_x=W, max_y=H, stride=strides[0])
        buf = planes[0]
    else:
        rx, ry = fd["h"][0] // fd["h"][1], fd["v"][0] // fd["v"][1]
        if fd["color"] == RGB:  # convertToRGB, decoder.zig:751-783
            y = planes[0].reshape(h_all, w_all)[:H, :W]
            cs = strides[1]
            cb = planes[1].reshape(-1, cs)
            cr = planes[2].reshape(-1, cs)
            rows = np.arange(H) // ry
            cols = np.arange(W) // rx
            out = np.empty((H, W, 4), np.uint8)
            out[..., 0] = y
            out[..., 1] = cb[rows][:, cols]
            out[..., 2] = cr[rows][:, cols]
            out[..., 3] = 255
            return out.reshape(-1)
        buf = np.concatenate(planes)
        img = O.ZoImage(kind=2, min_x=0, min_y=0, max_x=W, max_y=H, y_off=0, cb_off=planes[0].size,
                        cr_off=planes[0].size + planes[1].size, y_stride=strides[0], c_stride=strides[1],
                        subsample=SUB[(rx, ry)])
    img.pixels = buf.ctypes.data_as(C.POINTER(C.c_uint8))
    img.pixels_len = buf.size
    out = np.zeros(W * H * 4, np.uint8)
    assert O.lib().zo_rgba_pixels(C.byref(img), out.ctypes.data) == 0
    return out


def _run(frames, stride_pad=0):
    """One RGBA plan over all frames; returns each frame's (H, W*4) output rows."""
    npt = {8: np.int8, 16: np.int16, 32: np.int32}
    arr = (_lib.zpx_jpeg_frame * len(frames))()
    keep, outs = [], []
    for k, fd in enumerate(frames):
        f = arr[k]
        f.width, f.height, f.n_comp, f.mxx, f.myy = fd["width"], fd["height"], fd["n_comp"], fd["mxx"], fd["myy"]
        f.coeff_bits, f.narrow, f.color = fd["bits"], int(fd["narrow"]), fd["color"]
        for c in range(fd["n_comp"]):
            f.h[c], f.v[c] = fd["h"][c], fd["v"][c]
            g = fd["grids"][c]
            if g is None:
                f.rule[c] = 3  # ZPX_BLOCKS_NONE
                f.coeffs[c] = None
            else:
                t = torch.from_numpy(np.ascontiguousarray(g).astype(npt[fd["bits"]])).to("cuda")
                keep.append(t)
                f.coeffs[c] = t.data_ptr()
            qn = np.zeros(64, np.int32)
            qn[UNZIG] = fd["qz"][c]
            for i in range(64):
                f.qt[c][i] = int(qn[i])
        stride = fd["width"] * 4 + stride_pad
        o = torch.full((fd["height"] * stride,), 0x5A, dtype=torch.uint8, device="cuda")
        outs.append((o, stride))
        f.rgba = o.data_ptr()
        f.rgba_stride = stride
    ctx = zpix_amd.context.default()
    hp = C.c_void_p()
    _lib.check(_lib.lib().zpx_jpeg_plan_create(ctx.handle, arr, len(frames), 1, C.byref(hp)), ctx.handle)
    plan = device._Plan(hp, ctx)
    plan.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    plan.close()
    res = []
    for (o, stride), fd in zip(outs, frames):
        rows = o.cpu().numpy().reshape(fd["height"], stride)
        assert (rows[:, fd["width"] * 4:] == 0x5A).all()  # nothing past the row's pixels
        res.append(rows[:, :fd["width"] * 4].reshape(-1))
    return res


GEOMS = {
    "420": ((2, 2), (1, 1)), "422": ((2, 1), (1, 1)), "440": ((1, 2), (1, 1)), "444": ((1, 1), (1, 1)),
    "411": ((4, 1), (1, 1)), "410": ((4, 2), (1, 1)), "2212": ((2, 2), (1, 2)), "2221": ((2, 2), (2, 1)),
    "2121": ((2, 1), (2, 1)), "1212": ((1, 2), (1, 2)), "2222": ((2, 2), (2, 2)),
}


@pytest.mark.parametrize("geom", list(GEOMS))
@pytest.mark.parametrize("bits", [8, 16])
def test_fused_random_grids_ycbcr(geom, bits):
    """A ragged batch of three frames per geometry: two sizes (one wider than
    a 64-block task, one ending mid-MCU) and a width % 4 != 0 in a plan of
    its own, all narrow."""
    rng = np.random.default_rng(sum(map(ord, geom)) * 31 + bits)
    ragged = [
        _frame_data(rng, GEOMS[geom], YCBCR, 1032, 40, bits, True),
        _frame_data(rng, GEOMS[geom], YCBCR, 100, 70, bits, True),
    ]
    odd = [_frame_data(rng, GEOMS[geom], YCBCR, 77, 33, bits, True)]  # (width % 4 != 0)
    for frames in (ragged, odd):
        for fd, got in zip(frames, _run(frames)):
            assert np.array_equal(got, _expected(fd)), (fd["width"], fd["height"])


@pytest.mark.parametrize("geom", ["420", "444", "422", "2222"])
def test_fused_random_grids_rgb_gray_absent(geom):
    rng = np.random.default_rng(7)
    frames = [
        _frame_data(rng, GEOMS[geom], RGB, 264, 24, 8, True),
        _frame_data(rng, GEOMS[geom], YCBCR, 136, 48, 16, True, absent=(1,)),
        _frame_data(rng, GEOMS[geom], YCBCR, 96, 17, 8, True, absent=(0, 2)),
        _frame_data(rng, GEOMS[geom], YCBCR, 37, 17, 8, True, absent=(0, 2)),
    ]
    for fd in frames:
        got = _run([fd])[0]
        assert np.array_equal(got, _expected(fd)), (fd["width"], fd["color"])
    g = [_frame_data(rng, GEOMS[geom], GRAY, 520, 19, 8, True), _frame_data(rng, GEOMS[geom], GRAY, 8, 8, 16, True)]
    for fd, got in zip(g, _run(g)):
        assert np.array_equal(got, _expected(fd))


@pytest.mark.parametrize("bits,narrow", [(8, False), (16, False), (32, False), (32, True)])
def test_fused_random_grids_wide(bits, narrow):
    """Coefficients past the 24-bit bound (32-bit multiplies, wrap-around,
    the DC-only row shortcut) and the int32 transport: the strip kernel."""
    rng = np.random.default_rng(bits * 3 + narrow)
    frames = [_frame_data(rng, GEOMS["420"], YCBCR, 128, 48, bits, narrow),
              _frame_data(rng, GEOMS["444"], YCBCR, 64, 16, bits, narrow)]
    for fd, got in zip(frames, _run(frames)):
        assert np.array_equal(got, _expected(fd))


@pytest.mark.parametrize("geom", ["420", "444", "422"])
@pytest.mark.parametrize("stride_pad", [0, 4])
def test_fused_odd_widths_one_plan(geom, stride_pad):
    """Widths % 4 != 0 on the block kernel (its partial last 4-pixel piece
    leaves as dwords; rows only dword aligned take cached 16-byte stores), in
    one ragged plan with aligned ones: the last piece in the first, a middle
    and the last task of a row; nothing written past a row's pixels."""
    rng = np.random.default_rng(len(geom) * 7 + stride_pad)
    frames = [_frame_data(rng, GEOMS[geom], YCBCR, w, h, 8, True)
              for w, h in [(1030, 24), (77, 33), (513, 16), (96, 8), (1021, 9), (5, 3)]]
    for fd, got in zip(frames, _run(frames, stride_pad=stride_pad)):
        assert np.array_equal(got, _expected(fd)), (fd["width"], fd["height"])


def test_fused_padded_stride():
    """Row stride past the pixels (16-byte aligned: still the block kernel)."""
    rng = np.random.default_rng(11)
    frames = [_frame_data(rng, GEOMS["420"], YCBCR, 200, 40, 8, True)]
    for fd, got in zip(frames, _run(frames, stride_pad=48)):
        assert np.array_equal(got, _expected(fd))


@pytest.mark.parametrize("bits", [8, 16])
@pytest.mark.parametrize("geom", ["420", "444"])
def test_fused_narrow_limit_pairs(bits, geom):
    """The block kernel's packed-pair row pass at the narrow certificate's
    edge: 16-bit quant values up to 16384 with coefficients in {-1, 0, 1},
    and |coef * q| = 16384 exactly (64 * 256 int8, 128 * 128 int16) -- the
    v_pk_mul_lo_u16 products and v_dot2_i32_i16 sums at their largest."""
    rng = np.random.default_rng(97 + bits)
    fd = _frame_data(rng, GEOMS[geom], YCBCR, 264, 40, bits, True)
    lim = 64 if bits == 8 else 128
    for c in range(fd["n_comp"]):
        q = rng.integers(8192, 16385, 64).astype(np.int32)  # zigzag order
        q[rng.random(64) < 0.3] = 16384
        q[rng.random(64) < 0.5] = 16384 // lim
        fd["qz"][c] = q
        qn = np.zeros(64, np.int32)
        qn[UNZIG] = q
        g = rng.integers(-1, 2, fd["grids"][c].shape).astype(np.int32)
        blk = rng.random(g.shape[0]) < 0.25  # these blocks: +-lim wherever q = 16384 / lim
        big = rng.choice(np.array([-lim, lim], np.int32), size=g.shape)
        sel = blk[:, None] & (qn == 16384 // lim)[None, :]
        g[sel] = big[sel]
        fd["grids"][c] = g
        assert np.abs(g.astype(np.int64) * qn[None, :]).max() == 16384  # the certificate's bound, reached
    got = _run([fd])[0]
    assert np.array_equal(got, _expected(fd))
