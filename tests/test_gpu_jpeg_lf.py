"""The low-frequency short transform on every kernel
instance that takes it, bit-exact against the oracle.

A chroma pass of the fused kernel (jpeg_block_kernel), or a task of the
planar kernel (jpeg_plane_block_kernel), whose 64 blocks are all zero
outside the top-left 4x4 skips rows 4-7 of the transform; the test is a
wave ballot over a mask of the 48 positions outside 4x4 in the storage
order -- natural for dense grids, zig-zag for ZPX_COEFFS_PIECES.  The
reference's row pass maps a zero row to zeros (src/jpeg/idct.zig:84-97),
which is what makes the short path exact; a mask that missed a position
would send a block with a coefficient there down the short path and drop
it.

Every chroma block here is low-frequency except one outlier per task (the
fused kernel: per chroma pass, lanes < T the Cb blocks and T..2T-1 the Cr
blocks of the task's T = 64 / H0 MCUs; the planar kernel: per 64-block
segment of a chroma block row).  The outliers walk all 48 positions outside
4x4 (natural positions; in zig-zag storage the same 48 slots), on lane 0,
on the task's last lane and on a random lane; a quarter of the tasks carry
none and take the short path.  Luma is random (the full transform).
Expected pixels: reconstructBlock (src/jpeg/decoder.zig:1553-1634; unzig
:73-82) and rgbaPixels (image.zig:103-130), through the oracle.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle_py as O  # noqa: E402
from test_gpu_jpeg import _run_planar_grids  # noqa: E402
from test_gpu_jpeg_fused import GEOMS, UNZIG, YCBCR, _expected, _run  # noqa: E402
from test_gpu_pieces import _run_pieces  # noqa: E402

pytestmark = pytest.mark.gpu

OUTSIDE = [r * 8 + c for r in range(8) for c in range(8) if r >= 4 or c >= 4]
assert len(OUTSIDE) == 48


def _outlier_value(rng, bits, lim):
    """A nonzero coefficient; int16 also draws values whose low byte is zero
    (the mask must cover both bytes of an int16 coefficient)."""
    if bits == 16 and rng.random() < 0.4:
        v = int(rng.choice([256, 512, 768, 1024]))
    else:
        v = int(rng.integers(1, lim + 1))
    return v if rng.random() < 0.5 else -v


def _lf_frame(rng, geom, bits, mxx, myy):
    """A narrow YCbCr frame: random luma, chroma zero outside 4x4 everywhere."""
    (h0, v0), (hc, vc) = GEOMS[geom]
    h, v = [h0, hc, hc], [v0, vc, vc]
    # narrow certificate: max|coef * q| <= 16384 (int16 outliers reach 1024:
    # their quant values stay <= 16)
    lim, qmax = 64, (256 if bits == 8 else 17)
    grids, qz = [], []
    for c in range(3):
        gw, gh = mxx * h[c], myy * v[c]
        g = rng.integers(-lim, lim + 1, (gh, gw, 8, 8))
        g[rng.random(g.shape) < 0.7] = 0
        if c > 0:
            g[:, :, 4:, :] = 0
            g[:, :, :, 4:] = 0
        grids.append(g)
        qz.append(rng.integers(1, qmax, 64).astype(np.int32))
    return dict(width=mxx * 8 * h0, height=myy * 8 * v0, n_comp=3, h=h, v=v, mxx=mxx, myy=myy, grids=grids,
                qz=qz, bits=bits, narrow=True, color=YCBCR)


def _place_outliers(rng, fd, tasks, walk):
    """tasks: per task, its lanes' (component, block row, block column).
    Task t carries no outlier when t % 4 == 3, else one on lane 0 (t % 4 ==
    0), the task's last lane (1) or a random lane (2), at the next position
    of the 48-position walk.  Returns the walk's new state."""
    for t, lanes in enumerate(tasks):
        mode = t % 4
        if mode == 3:
            continue
        j = 0 if mode == 0 else (len(lanes) - 1 if mode == 1 else int(rng.integers(0, len(lanes))))
        c, by, bx = lanes[j]
        k = OUTSIDE[walk % 48]
        walk += 1
        fd["grids"][c][by, bx, k // 8, k % 8] = _outlier_value(rng, fd["bits"], 64)
    return walk


def _fused_tasks(fd, geom):
    """The fused kernel's chroma-pass lanes (HC = VC = 1 geometries): task
    (my, tx) holds T = 64 / H0 MCUs; lane j < T is Cb block (my, tx T + j),
    lane T + j the Cr block beside it."""
    (h0, _), (hc, vc) = GEOMS[geom]
    assert hc == 1 and vc == 1
    T = 64 // h0
    assert fd["mxx"] % T == 0  # whole tasks: every lane holds a block
    return [[(1, my, tx * T + j) for j in range(T)] + [(2, my, tx * T + j) for j in range(T)]
            for my in range(fd["myy"]) for tx in range(fd["mxx"] // T)]


def _planar_tasks(fd):
    """The planar kernel's chroma tasks: 64 consecutive blocks of one block
    row of one component."""
    out = []
    for c in (1, 2):
        gh, gw = fd["grids"][c].shape[:2]
        for by in range(gh):
            for x0 in range(0, gw, 64):
                out.append([(c, by, x) for x in range(x0, min(gw, x0 + 64))])
    return out


def _flat(fd):
    g = dict(fd)
    g["grids"] = [x.reshape(-1, 64).astype(np.int32) for x in fd["grids"]]
    return g


# per geometry: MCUs across / down -- two whole tasks a row, 32 MCU rows, so
# each frame carries 48 outlier tasks (the whole walk)
SIZES = {"420": (64, 32), "422": (64, 32), "411": (32, 32)}


@pytest.mark.parametrize("geom", ["420", "422", "411"])
@pytest.mark.parametrize("bits", [8, 16])
def test_fused_low_frequency_chroma_passes(geom, bits):
    """The fused kernel on natural-order grids (4:2:0 / 4:2:2 / 4:1:1; on
    4:1:1 the chroma pass fills lanes 0-31 only) and on pieces (zig-zag;
    4:1:1 pieces are expanded to grids first)."""
    rng = np.random.default_rng(1000 + 10 * bits + len(geom) + int(geom))
    walk = 0
    for rnd in range(2):
        fd = _lf_frame(rng, geom, bits, *SIZES[geom])
        walk = _place_outliers(rng, fd, _fused_tasks(fd, geom), walk)
        fl = _flat(fd)
        want = _expected(fl)
        assert np.array_equal(_run([fl])[0], want), (geom, bits, rnd, "grids")
        got, _ = _run_pieces([fl], rng)
        assert np.array_equal(got[0], want), (geom, bits, rnd, "pieces")
    assert walk >= 96  # every position, twice


@pytest.mark.parametrize("geom", ["420", "422"])
@pytest.mark.parametrize("bits", [8, 16])
def test_planar_low_frequency_tasks_grids_and_pieces(geom, bits):
    """The planar kernel's chroma tasks, natural-order grids and pieces."""
    rng = np.random.default_rng(2000 + 10 * bits + int(geom))
    fd = _lf_frame(rng, geom, bits, *SIZES[geom])
    walk = _place_outliers(rng, fd, _planar_tasks(fd), 0)
    assert walk >= 48
    fl = _flat(fd)
    strides = [fl["mxx"] * fl["h"][c] * 8 for c in range(3)]
    want = []
    for c in range(3):
        gw, gh = fl["mxx"] * fl["h"][c], fl["myy"] * fl["v"][c]
        want.append(np.zeros(gw * 8 * gh * 8, np.uint8))
    O.reconstruct_grids(3, fl["width"], fl["height"], fl["h"], fl["v"], fl["mxx"], fl["myy"], fl["grids"], fl["qz"],
                        False, want, strides)
    qnat = []
    for c in range(3):
        n = np.zeros(64, np.int32)
        n[UNZIG] = fl["qz"][c]
        qnat.append(n)
    got = _run_planar_grids(fl["grids"], qnat, fl["h"], fl["v"], fl["mxx"], fl["myy"], fl["width"], fl["height"], 0,
                            bits, 1)
    for c in range(3):
        assert np.array_equal(got[c], want[c]), (geom, bits, c, "grids")
    got, _ = _run_pieces([fl], rng, out="planes")
    for c in range(3):
        assert np.array_equal(got[0][c], want[c]), (geom, bits, c, "pieces")
