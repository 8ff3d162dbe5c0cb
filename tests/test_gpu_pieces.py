"""ZPX_COEFFS_PIECES on the GPU: the compact coefficient transport (a
block's coefficients in zig-zag order up to its last nonzero one, in 16-byte
pieces, indexed by a uint32 per block) read straight into the block kernels'
coefficient image -- the fused RGBA kernel's YCbCr 4:2:0 / 4:2:2 / 4:4:0 /
4:4:4 instances and the planar kernel -- and expanded into dense grids for
every other kernel (jpeg_pieces_expand_kernel).  Every case is bit-exact
against the oracle (reconstructBlock, src/jpeg/decoder.zig:1553-1634, then
Image.rgbaPixels, image.zig:103-130).

The random cases build the pieces from random grids here (blocks placed in a
shuffled order in the data, all-zero blocks with no pieces, DC-only blocks,
ends of block at every position); the encoded cases take the host entropy
stage's own pieces (zpx_jpeg_entropy_decode_pieces)."""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle_py as O  # noqa: E402
import zpix_amd  # noqa: E402
from test_gpu_jpeg_fused import GEOMS, GRAY, RGB, UNZIG, YCBCR, _expected, _frame_data  # noqa: E402
from tools import synthetic as S  # noqa: E402
from zpix_amd import _lib, device  # noqa: E402
from zpix_amd import jpeg as J  # noqa: E402

pytestmark = pytest.mark.gpu


def to_pieces(grids, bits, rng):
    """Pieces of natural-order grids (list per component, None = absent):
    (data uint8, [index uint32 per component or None])."""
    per = 16 if bits == 8 else 8
    dt = np.int8 if bits == 8 else np.int16
    chunks, index = [np.zeros(per, dt)], []
    first = 1
    for g in grids:
        if g is None:
            index.append(None)
            continue
        zz = g[:, UNZIG].astype(dt)
        nz = zz != 0
        eob = np.where(nz.any(1), 64 - np.argmax(nz[:, ::-1], 1), 0)
        npc = (eob + per - 1) // per
        order = rng.permutation(len(g))  # the blocks' places in the data: any order
        ix = np.zeros(len(g), np.uint32)
        for b in order:
            if npc[b]:
                chunks.append(zz[b, :npc[b] * per])
                ix[b] = (first << 4) | npc[b]
                first += int(npc[b])
        index.append(ix)
    data = np.concatenate(chunks).view(np.uint8)
    assert data.size == first * 16
    return data, index


def _pieces_frames(frames, rng, out="rgba", stride_pad=0):
    """zpx_jpeg_frame descriptors (layout pieces) over device copies."""
    arr = (_lib.zpx_jpeg_frame * len(frames))()
    keep, outs = [], []
    for k, fd in enumerate(frames):
        f = arr[k]
        f.width, f.height, f.n_comp, f.mxx, f.myy = fd["width"], fd["height"], fd["n_comp"], fd["mxx"], fd["myy"]
        f.coeff_bits, f.narrow, f.color = fd["bits"], int(fd["narrow"]), fd["color"]
        data, index = to_pieces(fd["grids"], fd["bits"], rng)
        d = torch.from_numpy(data).to("cuda")
        keep.append(d)
        f.layout = 1
        f.pieces = d.data_ptr()
        f.pieces_bytes = data.size
        for c in range(fd["n_comp"]):
            f.h[c], f.v[c] = fd["h"][c], fd["v"][c]
            f.rule[c] = fd.get("rule", 0)
            if index[c] is None:
                f.rule[c] = 3
                f.coeffs[c] = None
            else:
                t = torch.from_numpy(index[c].view(np.int32)).to("cuda")
                keep.append(t)
                f.coeffs[c] = t.data_ptr()
            qn = np.zeros(64, np.int32)
            qn[UNZIG] = fd["qz"][c]
            for i in range(64):
                f.qt[c][i] = int(qn[i])
        if out == "rgba":
            stride = fd["width"] * 4 + stride_pad
            o = torch.full((fd["height"] * stride,), 0x5A, dtype=torch.uint8, device="cuda")
            outs.append((o, stride))
            f.rgba = o.data_ptr()
            f.rgba_stride = stride
        else:
            ps = []
            for c in range(fd["n_comp"]):
                gw, gh = fd["mxx"] * fd["h"][c], fd["myy"] * fd["v"][c]
                p = torch.zeros(gw * 8 * gh * 8, dtype=torch.uint8, device="cuda")
                ps.append(p)
                f.planes[c] = p.data_ptr()
                f.strides[c] = gw * 8
            outs.append(ps)
    return arr, keep, outs


def _run_pieces(frames, rng, out="rgba", stride_pad=0):
    arr, keep, outs = _pieces_frames(frames, rng, out, stride_pad)
    ctx = zpix_amd.context.default()
    hp = C.c_void_p()
    _lib.check(_lib.lib().zpx_jpeg_plan_create(ctx.handle, arr, len(frames), 1 if out == "rgba" else 0, C.byref(hp)),
               ctx.handle)
    plan = device._Plan(hp, ctx)
    plan.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    kernels = plan.kernel_count
    plan.close()
    res = []
    for o, fd in zip(outs, frames):
        if out == "rgba":
            o, stride = o
            rows = o.cpu().numpy().reshape(fd["height"], stride)
            assert (rows[:, fd["width"] * 4:] == 0x5A).all()
            res.append(rows[:, :fd["width"] * 4].reshape(-1))
        else:
            res.append([p.cpu().numpy() for p in o])
    del keep
    return res, kernels


@pytest.mark.parametrize("geom", ["420", "422", "440", "444"])
@pytest.mark.parametrize("bits", [8, 16])
def test_pieces_fused_random(geom, bits):
    """The fused kernel's pieces instances: a ragged batch (a frame wider than
    a 64-block task, one ending mid-MCU) and a width % 4 != 0 frame."""
    rng = np.random.default_rng(sum(map(ord, geom)) * 7 + bits)
    ragged = [_frame_data(rng, GEOMS[geom], YCBCR, 1032, 40, bits, True),
              _frame_data(rng, GEOMS[geom], YCBCR, 100, 70, bits, True)]
    odd = [_frame_data(rng, GEOMS[geom], YCBCR, 77, 33, bits, True)]
    for frames in (ragged, odd):
        got, _ = _run_pieces(frames, rng)
        for fd, g in zip(frames, got):
            assert np.array_equal(g, _expected(fd)), (geom, bits, fd["width"], fd["height"])


@pytest.mark.parametrize("geom", ["411", "2212", "420"])
def test_pieces_expand_fallback(geom):
    """Frames the pieces instances do not take -- other geometries, Adobe
    RGB, gray, a component never scanned -- are expanded into dense grids
    first (the plan's extra launch), same pixels."""
    rng = np.random.default_rng(len(geom) * 13)
    frames = [_frame_data(rng, GEOMS[geom], RGB, 264, 24, 8, True),
              _frame_data(rng, GEOMS[geom], YCBCR, 136, 48, 16, True, absent=(1,)),
              _frame_data(rng, GEOMS[geom], YCBCR, 96, 40, 8, True)]
    for fd in frames:
        got, kernels = _run_pieces([fd], rng)
        assert np.array_equal(got[0], _expected(fd)), (geom, fd["color"])
        direct = geom == "420" and fd["color"] == YCBCR
        assert kernels == (1 if direct else 2), (geom, fd["color"], kernels)
    g = [_frame_data(rng, GEOMS[geom], GRAY, 520, 19, 8, True)]
    got, _ = _run_pieces(g, rng)
    assert np.array_equal(got[0], _expected(g[0]))


def test_pieces_absent_component_direct():
    """A never-scanned chroma component on the direct path: its index is
    null, its blocks read piece 0, and its samples are makeImg's zeros."""
    rng = np.random.default_rng(3)
    for geom in ("420", "444"):
        fd = _frame_data(rng, GEOMS[geom], YCBCR, 136, 48, 8, True, absent=(2,))
        got, _ = _run_pieces([fd], rng)
        assert np.array_equal(got[0], _expected(fd)), geom


def test_pieces_strip_switch_expands():
    """The test switch "jpeg_strip" sends pieces frames through the expand +
    strip kernel path."""
    rng = np.random.default_rng(11)
    fd = _frame_data(rng, GEOMS["420"], YCBCR, 200, 72, 8, True)
    prev = _lib.lib().zpx_debug_option(b"jpeg_strip", 1)
    try:
        got, _ = _run_pieces([fd], rng)
    finally:
        _lib.lib().zpx_debug_option(b"jpeg_strip", prev)
    assert np.array_equal(got[0], _expected(fd))


@pytest.mark.parametrize("bits", [8, 16])
@pytest.mark.parametrize("geom", ["420", "411", "2212"])
def test_pieces_planar_random(bits, geom):
    """The planar block kernel reads pieces directly for every geometry
    (70 MCUs: three 64-block tasks a row, the last ragged)."""
    rng = np.random.default_rng(bits * 5 + len(geom))
    (h0, v0), (hc, vc) = GEOMS[geom]
    fd = _frame_data(rng, GEOMS[geom], YCBCR, 70 * 8 * h0 - 12, 3 * 8 * v0 - 5, bits, True)
    got, _ = _run_pieces([fd], rng, out="planes")
    want = [np.zeros_like(p) for p in got[0]]
    strides = [fd["mxx"] * fd["h"][c] * 8 for c in range(3)]
    O.reconstruct_grids(3, fd["width"], fd["height"], fd["h"], fd["v"], fd["mxx"], fd["myy"], fd["grids"], fd["qz"],
                        False, want, strides)
    for c in range(3):
        assert np.array_equal(got[0][c], want[c]), (bits, geom, c)


@pytest.mark.parametrize("sub,quality", [(2, 75), (1, 90), (0, 98), (2, 100)])
def test_pieces_encoded_frames_match_oracle(sub, quality):
    """The host entropy stage's own pieces (int8 at q75, int16 where the
    coefficients need it) through a pieces plan, RGBA and planes."""
    datas = [S.jpeg_subsampled(40 + sub, 333, 177, sub, quality), S.jpeg_subsampled(50 + sub, 64, 48, sub, quality)]
    cos = [J.Coefficients(d, pieces=True) for d in datas]
    assert all(c.is_pieces for c in cos)
    b = device.JpegBatch(cos, slots=[0, 1, 0], output="rgba")
    b.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for s, i in enumerate(b.slots):
        want = O.jpeg_decode(datas[i]).rgba_pixels().reshape(b.output_tensor(s).shape)
        assert np.array_equal(b.output_tensor(s).cpu().numpy(), want), (s, quality)
    p = device.JpegBatch(cos, output="planes")
    p.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for s in range(len(cos)):
        assert np.array_equal(p.output_tensor(s).cpu().numpy(), O.jpeg_decode(datas[s]).pixels), s


def test_pieces_4k_bench_frame():
    """The bench frame (4096^2 4:2:0 q75) from its pieces: the bench's
    pieces line.  RGBA bit-exact, and the plan's bytes are the pieces, the
    index words and the RGBA -- well under the dense int8 grid's."""
    data = S.jpeg_420(0, 4096, 4096)
    co = J.Coefficients(data, pieces=True)
    assert co.is_pieces and co.frame.coeff_bits == 8 and co.frame.narrow == 1
    b = device.JpegBatch([co], slots=[0, 0], output="rgba")
    b.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    want = torch.from_numpy(O.jpeg_decode(data).rgba_pixels().reshape(4096, 4096, 4))
    for s in range(2):
        assert torch.equal(b.output_tensor(s).cpu(), want)
    pieces = int(co.frame.pieces_bytes)
    assert b.bytes == 2 * (pieces + 393216 * 4 + 4096 * 4096 * 4 + 3 * 256)
    assert pieces < 0.7 * 393216 * 64
