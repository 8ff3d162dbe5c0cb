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


@pytest.mark.skipif(GXX is None, reason="g++ not available")
def test_inflate_sanitized_growing_chunks(tmp_path):
    exe = str(tmp_path / "inflate_check")
    src = os.path.join(ROOT, "zpix_amd", "csrc")
    subprocess.run([GXX, "-O1", "-g", "-std=c++17", "-march=x86-64-v3", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-I", src, os.path.join(ROOT, "tests", "inflate_check.cpp"),
                    os.path.join(src, "inflate_fast.cpp"), "-lpthread", "-o", exe], check=True, timeout=300)
    for name, raw, level in _streams():
        z = zlib.compress(raw, level)
        zp, rp = tmp_path / f"{name}.z", tmp_path / f"{name}.raw"
        zp.write_bytes(z)
        rp.write_bytes(raw)
        r = subprocess.run([exe, str(zp), str(rp)], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0 and r.stdout.strip() == "ok", (name, r.stderr[-3000:])
