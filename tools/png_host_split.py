"""PNG host stage split on one 4K tc8 image: the serial fast inflate of the zlib stream alone
against zpx_png_inflate (chunk walk, CRC, IDAT concatenation, inflate), best of 5.
Run with ZPX_INFLATE_THREADS=1."""
import sys, time, ctypes as C, struct, zlib
import os; sys.path[:0]=[os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import numpy as np
from tools import synthetic as S
from zpix_amd import _lib
L=_lib.lib()
d=S.png_tc8_mixed(1, 4096, 4096)
# zlib stream
p=8; z=b''
while p < len(d):
    n=struct.unpack('>I', d[p:p+4])[0]; t=d[p+4:p+8]
    if t==b'IDAT': z+=d[p+8:p+8+n]
    p+=n+12
raw_len = 4096*(1+4096*3)
out=np.zeros(raw_len+64, np.uint8)
def t_inflate():
    t=time.perf_counter(); ok=L.zpx_debug_inflate_parallel(z, len(z), out.ctypes.data, raw_len, 1); return time.perf_counter()-t, ok
def t_parse():
    h=C.c_void_p(); t=time.perf_counter(); rc=L.zpx_png_inflate(d, len(d), C.byref(h)); dt=time.perf_counter()-t; L.zpx_png_stream_free(h); return dt, rc
for r in range(3):
    a=min(t_inflate()[0] for _ in range(5)); b=min(t_parse()[0] for _ in range(5))
    print(f"inflate only {a*1e3:.1f} ms   png_inflate (CRC + copy + inflate) {b*1e3:.1f} ms   len(z)={len(z)/1e6:.1f} MB")
