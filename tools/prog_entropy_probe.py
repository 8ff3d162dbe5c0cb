"""Times the host entropy stage on configs[4]'s 4K progressive 4:4:4 frame (debug aid; ZPX_JPEG_PROG_TRACE=1 prints per-scan times)."""
import sys, time, os
import os; R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0] = [R, os.path.join(R, 'tests')]
from tools import synthetic as S
from zpix_amd import jpeg, _lib
import numpy as np
d = S.jpeg_progressive_444(1000, 4096, 4096)
import oracle_py as O
for rep in range(3):
    t0 = time.perf_counter(); co = jpeg.Coefficients(d); t = time.perf_counter() - t0
    print(f"entropy {t*1e3:.1f} ms  {4096*4096/t/1e6:.1f} MPix/s bits={co.frame.coeff_bits} narrow={co.frame.narrow} par_prog={_lib.lib().zpx_debug_jpeg_parallel_progressive()}")
if len(sys.argv) > 1:
    oc = O.jpeg_coefficients(d)
    for c in range(3):
        n = co.coeff_bytes[c]
        import ctypes as C
        dt = {8: np.int8, 16: np.int16, 32: np.int32}[co.frame.coeff_bits]
        g = np.ctypeslib.as_array(C.cast(co.frame.coeffs[c], C.POINTER(C.c_uint8)), shape=(n,)).view(dt).astype(np.int32)
        print(c, np.array_equal(g.reshape(-1), np.asarray(oc.grids[c]).reshape(-1)))
