"""A/B of the host progressive entropy decode (zpx_jpeg_entropy_decode on the
bench's 4096^2 progressive 4:4:4 frame) between library builds: best of N
decodes per build, builds alternating.  Usage: python3 tools/prog_ab.py lib1 lib2 ..."""
import ctypes as C
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(lib, path, n=5):
    L = C.CDLL(lib)
    L.zpx_jpeg_entropy_decode.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_void_p)]
    L.zpx_jpeg_coeffs_free.argtypes = [C.c_void_p]
    data = open(path, "rb").read()
    best = 1e9
    for _ in range(n):
        h = C.c_void_p()
        t = time.perf_counter()
        assert L.zpx_jpeg_entropy_decode(data, len(data), C.byref(h)) == 0
        best = min(best, time.perf_counter() - t)
        L.zpx_jpeg_coeffs_free(h)
    return 4096 * 4096 / best / 1e6


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        print(round(one(sys.argv[2], sys.argv[3]), 1))
        sys.exit(0)
    sys.path.insert(0, ROOT)
    from tools import synthetic as S
    path = "/tmp/prog_ab_444.jpg"
    open(path, "wb").write(S.jpeg_progressive_444(1000, 4096, 4096))
    for r in range(3):
        for lib in sys.argv[1:]:
            out = subprocess.run([sys.executable, __file__, "--one", lib, path], capture_output=True, text=True)
            print(r, os.path.basename(lib), out.stdout.strip() or out.stderr[-300:], flush=True)
