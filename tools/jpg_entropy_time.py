import ctypes as C, time, sys
sys.path[:0]=[__import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__)))]
from tools import synthetic as S
L=C.CDLL(sys.argv[1])
data=S.jpeg_420(0,4096,4096,75)
L.zpx_jpeg_entropy_decode_pieces.argtypes=[C.c_char_p,C.c_size_t,C.POINTER(C.c_void_p)]
L.zpx_jpeg_coeffs_free.argtypes=[C.c_void_p]
best=1e9
for i in range(7):
    h=C.c_void_p(); t=time.perf_counter(); r=L.zpx_jpeg_entropy_decode_pieces(data,len(data),C.byref(h)); dt=time.perf_counter()-t
    assert r==0, r
    L.zpx_jpeg_coeffs_free(h); best=min(best,dt)
print(f'jpeg pieces entropy: {best*1e3:.1f} ms  ({len(data)/1e6:.2f} MB)')
