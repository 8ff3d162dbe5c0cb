"""The fast host inflate (zpix_amd/csrc/inflate_fast.cpp) under the host
sanitizers (g++ -fsanitize=address,undefined; host code only): serial,
two-stream (inflate_fast_pair) and speculative parallel decodes of streams whose single DEFLATE blocks expand to
more than a speculative chunk's first output buffer (4 MiB of symbols: long
zero runs, 258-byte matches), so the chunk buffers must grow mid-block."""
import os
import shutil
import subprocess
import zlib

import numpy as np
import pytest

from tools import synthetic as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GXX = shutil.which("g++")


def _streams():
    rng = np.random.default_rng(5)
    noise = lambda n: (128 + rng.normal(0, 12, n)).clip(0, 255).astype(np.uint8).tobytes()  # noqa: E731
    zeros = bytes(12 << 20)
    runs = noise(300_000) + zeros + noise(300_000) + zeros + noise(300_000)
    ramp = b"".join(bytes([i % 251]) * 70_000 + noise(2_000) for i in range(200))
    _, tc8 = S.png_filtered_tc8(3, 640, 400)
    return [("runs", runs, 6), ("runs9", runs, 9), ("ramp", ramp, 6), ("tc8", tc8.tobytes(), 6),
            ("stored", noise(200_000), 0)]


def _build(tmp_path):
    exe = str(tmp_path / "inflate_check")
    src = os.path.join(ROOT, "zpix_amd", "csrc")
    subprocess.run([GXX, "-O1", "-g", "-std=c++17", "-march=x86-64-v3", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-I", src, os.path.join(ROOT, "tests", "inflate_check.cpp"),
                    os.path.join(src, "inflate_fast.cpp"), "-lpthread", "-o", exe], check=True, timeout=300)
    return exe


class _Bits:
    """LSB-first DEFLATE bit writer (Huffman codes are given MSB-first)."""

    def __init__(self):
        self.v, self.n = 0, 0

    def put(self, val, nbits):
        self.v |= val << self.n
        self.n += nbits

    def code(self, c, nbits):  # a Huffman code, most significant bit first
        self.put(int(format(c, f"0{nbits}b")[::-1], 2), nbits)

    def data(self):
        return self.v.to_bytes((self.n + 7) // 8, "little")


def _fixed_bad_distance():
    """zlib header + one fixed-Huffman block: literal 'a', then a length-3
    match at distance 4 -- past the output's start (RFC 1951 3.2.6 codes)."""
    b = _Bits()
    b.put(1, 1)  # BFINAL
    b.put(1, 2)  # BTYPE = 01, fixed codes
    b.code(0x30 + ord("a"), 8)  # literal 'a'
    b.code(1, 7)  # length code 257: length 3
    b.code(3, 5)  # distance code 3: distance 4
    b.code(0, 7)  # end of block
    return b"\x78\x9c" + b.data() + b"\x00\x00\x00\x00"


@pytest.mark.skipif(GXX is None, reason="g++ not available")
def test_inflate_sanitized_malformed_pairs(tmp_path):
    """inflate_fast_pair on malformed streams, each paired with valid ones
    and with each other: its careful path's distance and overrun
    checks, a stored block whose length check fails, a last block ending
    short of want, one stream failing while the other goes on alone -- every
    ok / produced / byte equal to inflate_fast's on the stream alone, under
    ASan / UBSan."""
    exe = _build(tmp_path)
    rng = np.random.default_rng(9)
    noise = (128 + rng.normal(0, 12, 400_000)).clip(0, 255).astype(np.uint8).tobytes()
    smooth = np.repeat(rng.integers(0, 256, 4_000, dtype=np.uint8), 50).tobytes()
    raw = noise[:200_000] + smooth + noise[200_000:]
    want = len(raw)
    good = zlib.compress(raw, 6)
    stored = zlib.compress(raw[:150_000], 0)
    streams = [good, zlib.compress(raw, 1), good[:len(good) // 2], good[:len(good) - 9], good[:3],
               zlib.compress(raw[:want - 5000], 6),  # the last block ends short of want
               stored, stored[:70_000],
               _fixed_bad_distance()]
    bad_stored = bytearray(stored)
    bad_stored[2 + 3] ^= 0xff  # the first stored block's NLEN no longer complements LEN
    streams.append(bytes(bad_stored))
    for pos in (11, len(good) // 3, len(good) // 2, len(good) - 40):
        f = bytearray(good)
        f[pos] ^= 0x10
        streams.append(bytes(f))
    files = []
    for i, z in enumerate(streams):
        p = tmp_path / f"s{i}.z"
        p.write_bytes(z)
        files.append(str(p))
    r = subprocess.run([exe, "pairs", str(want)] + files, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stderr[-3000:]
    accepted = int(r.stdout.split()[1])
    assert 2 <= accepted < len(streams), r.stdout


@pytest.mark.skipif(GXX is None, reason="g++ not available")
def test_inflate_sanitized_growing_chunks(tmp_path):
    exe = _build(tmp_path)
    for name, raw, level in _streams():
        z = zlib.compress(raw, level)
        zp, rp = tmp_path / f"{name}.z", tmp_path / f"{name}.raw"
        zp.write_bytes(z)
        rp.write_bytes(raw)
        r = subprocess.run([exe, str(zp), str(rp)], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0 and r.stdout.strip() == "ok", (name, r.stderr[-3000:])
