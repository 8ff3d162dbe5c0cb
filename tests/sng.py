"""SNG text formatter used for the PngSuite golden comparison.

Restates the reference's test formatter src/png/sng.zig:48-320 (itself an
approximation of the `sng` tool) so the committed .sng goldens
(tests/golden/pngsuite/*.sng, copied from src/testdata/png) can be compared
line by line, exactly as src/png/decoder_test.zig:46-129 does.

Works on any image object exposing kind / rect / pixels / stride / palette
(tests/oracle_py.OImage and zpix_amd.image.Image both do).
"""
from __future__ import annotations

import os

# sng.zig:15-23
FAKE_IHDR_USINGS = {
    "ftbbn0g01": "    using grayscale;\n",
    "ftbbn0g02": "    using grayscale;\n",
    "ftbbn0g04": "    using grayscale;\n",
    "ftbbn2c16": "    using color;\n",
    "ftbgn2c16": "    using color;\n",
    "ftbrn2c08": "    using color;\n",
    "ftbwn0g16": "    using grayscale;\n",
}
# sng.zig:27-30
FAKE_GAMAS = {"ftbbn0g01": "", "ftbbn0g02": "gAMA {0.45455}\n"}
# sng.zig:34-46
FAKE_BKGDS = {
    "ftbbn0g01": "bKGD {gray: 0;}\n",
    "ftbbn0g02": "bKGD {gray: 0;}\n",
    "ftbbn0g04": "bKGD {gray: 0;}\n",
    "ftbbn2c16": "bKGD {red: 0;  green: 0;  blue: 65535;}\n",
    "ftbbn3p08": "bKGD {index: 245}\n",
    "ftbgn2c16": "bKGD {red: 0;  green: 65535;  blue: 0;}\n",
    "ftbgn3p08": "bKGD {index: 245}\n",
    "ftbrn2c08": "bKGD {red: 255;  green: 0;  blue: 0;}\n",
    "ftbwn0g16": "bKGD {gray: 65535;}\n",
    "ftbwn3p08": "bKGD {index: 0}\n",
    "ftbyn3p08": "bKGD {index: 245}\n",
}
GRAY_AS_NRGBA = ("ftbbn0g01", "ftbbn0g02", "ftbbn0g04")


def _px(img, x, y, n):
    off = (y - img.rect[1]) * img.stride + (x - img.rect[0]) * n
    return img.pixels[off:off + n]


def _u16(b, i):
    return (int(b[i]) << 8) | int(b[i + 1])


def sng(filename: str, img) -> str:
    out = []
    w = img.rect[2] - img.rect[0]
    h = img.rect[3] - img.rect[1]
    kind = img.kind
    if kind in ("RGBA", "NRGBA", "Gray"):
        bit_depth = 8
    elif kind == "Paletted":
        n = len(img.palette)
        bit_depth = 1 if n <= 2 else 2 if n <= 4 else 4 if n <= 16 else 8
    else:
        bit_depth = 16
    base = os.path.basename(filename)
    stem = os.path.splitext(base)[0]
    out.append(f"#SNG: from {base}\nIHDR {{\n")
    out.append(f"    width: {w}; height: {h}; bitdepth: {bit_depth};\n")
    if stem in FAKE_IHDR_USINGS:
        out.append(FAKE_IHDR_USINGS[stem])
    else:
        out.append({
            "Gray": "    using grayscale;\n", "Gray16": "    using grayscale;\n",
            "RGBA": "    using color;\n", "RGBA64": "    using color;\n",
            "NRGBA": "    using color alpha;\n", "NRGBA64": "    using color alpha;\n",
            "Paletted": "    using color palette;\n",
        }.get(kind, "unknown PNG decoder color model\n"))
    out.append("}\n")
    out.append(FAKE_GAMAS.get(stem, "gAMA {1.0000}\n"))
    use_transparent = False
    if kind == "Paletted":
        out.append("PLTE {\n")
        last_alpha = None
        for i, (r, g, b, a, tag) in enumerate(img.palette):
            if tag == 0:
                a = 0xFF
            if a != 0xFF:
                last_alpha = i
            out.append(f"    ({r:3d},{g:3d},{b:3d})     # rgb = (0x{r:02x},0x{g:02x},0x{b:02x})\n")
        out.append("}\n")
        if stem in FAKE_BKGDS:
            out.append(FAKE_BKGDS[stem])
        if last_alpha is not None:
            out.append("tRNS {\n")
            for i in range(last_alpha + 1):
                a = img.palette[i][3]  # toRGBA() alpha >> 8, color.zig:34-72
                out.append(f" {(a | a << 8) >> 8}")
            out.append("}\n")
    elif stem.startswith("ft"):
        if stem in FAKE_BKGDS:
            out.append(FAKE_BKGDS[stem])
        if kind == "NRGBA":
            p = _px(img, img.rect[0], img.rect[1], 4)
            if p[3] == 0:
                use_transparent = True
                out.append("tRNS {\n")
                if stem in GRAY_AS_NRGBA:
                    out.append(f"    gray: {int(p[0])};\n")
                else:
                    out.append(f"    red: {int(p[0])}; green: {int(p[1])}; blue: {int(p[2])};\n")
                out.append("}\n")
        elif kind == "NRGBA64":
            p = _px(img, img.rect[0], img.rect[1], 8)
            if _u16(p, 6) == 0:
                use_transparent = True
                out.append("tRNS {\n")
                if stem == "ftbwn0g16":
                    out.append(f"    gray: {_u16(p, 0)};\n")
                else:
                    out.append(f"    red: {_u16(p, 0)}; green: {_u16(p, 2)}; blue: {_u16(p, 4)};\n")
                out.append("}\n")
    out.append("IMAGE {\n    pixels hex\n")
    x0, y0 = img.rect[0], img.rect[1]
    for y in range(y0, y0 + h):
        line = []
        if kind == "Gray":
            for x in range(x0, x0 + w):
                line.append(f"{int(_px(img, x, y, 1)[0]):02x}")
        elif kind == "Gray16":
            for x in range(x0, x0 + w):
                line.append(f"{_u16(_px(img, x, y, 2), 0):04x} ")
        elif kind == "RGBA":
            for x in range(x0, x0 + w):
                p = _px(img, x, y, 4)
                line.append(f"{int(p[0]):02x}{int(p[1]):02x}{int(p[2]):02x} ")
        elif kind == "RGBA64":
            for x in range(x0, x0 + w):
                p = _px(img, x, y, 8)
                line.append(f"{_u16(p, 0):04x}{_u16(p, 2):04x}{_u16(p, 4):04x} ")
        elif kind == "NRGBA":
            for x in range(x0, x0 + w):
                p = _px(img, x, y, 4)
                if stem in GRAY_AS_NRGBA:
                    line.append(f"{int(p[0]):02x}")
                elif use_transparent:
                    line.append(f"{int(p[0]):02x}{int(p[1]):02x}{int(p[2]):02x} ")
                else:
                    line.append(f"{int(p[0]):02x}{int(p[1]):02x}{int(p[2]):02x}{int(p[3]):02x} ")
        elif kind == "NRGBA64":
            for x in range(x0, x0 + w):
                p = _px(img, x, y, 8)
                if stem == "ftbwn0g16":
                    line.append(f"{_u16(p, 0):04x} ")
                elif use_transparent:
                    line.append(f"{_u16(p, 0):04x}{_u16(p, 2):04x}{_u16(p, 4):04x} ")
                else:
                    line.append(f"{_u16(p, 0):04x}{_u16(p, 2):04x}{_u16(p, 4):04x}{_u16(p, 6):04x} ")
        elif kind == "Paletted":
            b = 0
            c = 0
            for x in range(x0, x0 + w):
                b = (b << bit_depth) | int(_px(img, x, y, 1)[0])
                c += 1
                if c == 8 // bit_depth:
                    line.append(f"{b:02x}")
                    b = 0
                    c = 0
            if c != 0:
                while c != 8 // bit_depth:
                    b <<= bit_depth
                    c += 1
                line.append(f"{b:02x}")
        out.append("".join(line) + "\n")
    out.append("}\n")
    return "".join(out)


def compare_with_golden(actual: str, expected: str) -> None:
    """Line-by-line comparison as decoder_test.zig:92-127 (strips sng color names)."""
    a_lines = actual.split("\n")
    e_lines = expected.split("\n")
    if len(a_lines) != len(e_lines):
        raise AssertionError(f"line count mismatch {len(a_lines)} vs {len(e_lines)}")
    for i, (a, e) in enumerate(zip(a_lines, e_lines)):
        if "# rgb = (" in e and not e.endswith(")"):
            j = e.rfind(") ")
            if j >= 0:
                e = e[: j + 1]
        if a != e:
            raise AssertionError(f"line {i} mismatch:\n  got:  {a!r}\n  want: {e!r}")
