"""Host JPEG entropy time of the bench frame (4K q75 4:2:0), pieces and grids,
best of 15, for the library ZPX_LIB_PATH names (A/B of host decoder builds)."""
import sys, time, os
sys.path[:0]=[os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
from tools import synthetic as S
from zpix_amd import jpeg
d = S.jpeg_420(0, 4096, 4096)
for pz in (True, False):
    best=1e9
    for i in range(15):
        t=time.perf_counter(); c=jpeg.Coefficients(d, pieces=pz); dt=time.perf_counter()-t; best=min(best,dt)
    print(os.path.basename(os.environ.get('ZPX_LIB_PATH','cur')), 'pieces' if pz else 'grids', f"{best*1e3:.1f} ms")
