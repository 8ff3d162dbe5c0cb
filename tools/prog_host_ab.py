"""A/B of the bench's progressive host entropy measurement (configs[4]:
jpeg.Coefficients of the 4096^2 progressive 4:4:4 frame, best of three, as
bench.py times it) between library builds, each in its own process, rounds
alternating.  Usage: python tools/prog_host_ab.py lib1 lib2 ..."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(path):
    sys.path[:0] = [ROOT]
    from zpix_amd import jpeg
    d = open(path, "rb").read()
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        jpeg.Coefficients(d)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return 4096 * 4096 / best / 1e6


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        print(round(one(sys.argv[2]), 1))
        sys.exit(0)
    sys.path.insert(0, ROOT)
    from tools import synthetic as S
    path = "/tmp/prog_host_ab.jpg"
    open(path, "wb").write(S.jpeg_progressive_444(1000, 4096, 4096))
    for r in range(4):
        for lib in sys.argv[1:]:
            env = dict(os.environ, ZPX_LIB_PATH=os.path.abspath(lib))
            out = subprocess.run([sys.executable, __file__, "--one", path], capture_output=True, text=True, env=env)
            print(r, os.path.basename(lib), out.stdout.strip() or out.stderr[-300:], flush=True)
