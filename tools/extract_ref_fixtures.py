"""Extract the inline byte fixtures from the reference's JPEG tests into binary
fixture files under tests/golden/testdata/.

Runs only in the build container (it reads /root/reference); its outputs are
committed so the GPU box never needs the reference:
  - large_short.jpeg: the 504-byte 8192x8192 SOF input of the
    "large image with short data" test, src/jpeg/decoder.zig:1974-2017
  - padded_rst.jpeg:  the base64 image of the "padded rst marker" test,
    src/jpeg/decoder.zig:2031-2186 (golang.org/issue/28717)
"""
import base64
import os
import re

REF = "/root/reference/src/jpeg/decoder.zig"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "testdata")


def main():
    src = open(REF).read()
    # 504-byte array literal inside test "large image with short data"
    t = src.index('test "large image with short data"')
    a = src.index("&[_]u8{", t)
    b = src.index("};", a)
    vals = [int(v, 16) for v in re.findall(r"0x([0-9a-fA-F]{2})", src[a:b])]
    assert len(vals) == 504, len(vals)
    with open(os.path.join(OUT, "large_short.jpeg"), "wb") as f:
        f.write(bytes(vals))
    # base64 multi-line string inside test "padded rst marker"
    t = src.index('test "padded rst marker"')
    e = src.index(";", src.index("const base64EncodedImage", t))
    lines = [ln.strip()[2:] for ln in src[t:e].splitlines() if ln.strip().startswith("\\\\")]
    data = base64.b64decode("".join(lines))
    with open(os.path.join(OUT, "padded_rst.jpeg"), "wb") as f:
        f.write(data)
    print("wrote", len(vals), "and", len(data), "bytes")


if __name__ == "__main__":
    main()
