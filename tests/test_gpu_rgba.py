"""GPU parity of Image.rgbaPixels (src/image/image.zig:103-130 with
Color.toRGBA, src/color/color.zig:31-131) on device-resident images: the
per-kind kernels behind zpx_dev_rgba_pixels / zpx_rgba_plan_create (one plan
over a ragged batch of every image kind, widths that are and are not a
multiple of the 4-pixel vector piece), bit-exact against the oracle."""
import numpy as np
import pytest

import oracle_py as O
from conftest import read
from test_gpu_png import ALL_KIND_FILES
from tools import synthetic as S

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import zpix_amd  # noqa: E402
from zpix_amd import device  # noqa: E402


def _png_cases():
    """(name, png bytes): every PNG colour type x depth that yields its own
    image kind (NRGBA64 / RGBA64 / NRGBA / RGBA / Gray16 / Gray / Paletted),
    at a width that fills the 4-pixel pieces and one that does not."""
    out = []
    for depth, ct, kw in [(16, 6, {}), (16, 2, {}), (8, 6, {}), (8, 2, {}), (16, 0, {}), (8, 0, {}), (8, 4, {}),
                          (16, 4, {}), (8, 3, {"palette": bytes(range(48))}), (8, 2, {"trns": b"\x00\x10\x00\x20\x00\x30"})]:
        for w, h in [(64, 9), (37, 11)]:
            out.append((f"d{depth}c{ct}_{w}", S.png_generic(depth * 10 + ct + w, w, h, depth, ct, **kw)))
    return out


def test_rgba_plan_every_kind_ragged_batch():
    """One zpx_rgba_plan over every kind (PNG outputs and the JPEG/PngSuite
    fixtures), repeated items in several slots: every slot equals the
    oracle's Image.rgbaPixels."""
    datas = ([d for _, d in _png_cases()] + [read(w, n) for w, n in ALL_KIND_FILES if w == "testdata"] +
             [read(w, n) for w, n in ALL_KIND_FILES if w == "pngsuite"][::4])
    imgs = [zpix_amd.from_buffer(d) for d in datas]
    slots = list(range(len(imgs))) + [0, len(imgs) - 1, 1]
    b = device.RgbaBatch(imgs, slots=slots)
    b.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    kinds = set()
    for s, i in enumerate(slots):
        want = O.decode(datas[i]).rgba_pixels()
        kinds.add(imgs[i].kind)
        assert np.array_equal(b.output_tensor(s).cpu().numpy().reshape(-1), want), (s, imgs[i].kind)
    assert kinds >= {"NRGBA64", "RGBA64", "NRGBA", "RGBA", "Gray16", "Gray", "Paletted", "YCbCr", "CMYK"}
    assert b.plan.kernel_count == len(kinds)


@pytest.mark.parametrize("name,data", _png_cases(), ids=lambda x: x if isinstance(x, str) else "")
def test_rgba_pixels_per_kind_matches_oracle(name, data):
    """The single-image path (Image.rgba_pixels -> zpx_image_rgba_pixels ->
    the kind's kernel)."""
    got = zpix_amd.from_buffer(data).rgba_pixels()
    assert np.array_equal(got, O.decode(data).rgba_pixels()), name


def test_rgba_plan_nrgba64_4k():
    """The bench's rgbaPixels line: a 4096^2 NRGBA64 image (configs[4]'s
    Adam7 RGBA16 output) in two slots."""
    data = S.png_rgba16_adam7(2000, 1024, 4096)
    img = zpix_amd.from_buffer(data)
    assert img.kind == "NRGBA64"
    b = device.RgbaBatch([img], slots=[0, 0])
    b.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    want = O.decode(data).rgba_pixels()
    for s in range(2):
        assert np.array_equal(b.output_tensor(s).cpu().numpy().reshape(-1), want)
    assert b.bytes == 2 * (1024 * 4096 * 8 + 1024 * 4096 * 4)
