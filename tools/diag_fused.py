import sys, glob, os, numpy as np
sys.path.insert(0,'tests'); sys.path.insert(0,'.')
import oracle_py as O
import zpix_amd
from zpix_amd import jpeg as J
for n in ['video-001.jpeg','video-001.q50.420.jpeg','video-001.q50.422.jpeg','padded_rst.jpeg','video-005.gray.jpeg','video-001.rgb.jpeg']:
    d = open('tests/golden/testdata/'+n,'rb').read()
    o = O.jpeg_decode(d); want = o.rgba_pixels().reshape(o.height, o.width, 4).astype(int)
    got = J.decode_rgba(d).astype(int)
    diff = np.abs(got-want)
    print(n, o.kind, o.subsample, 'maxdiff per ch', diff.reshape(-1,4).max(0), 'frac', (diff.sum(-1)>0).mean())
    if o.kind == 'YCbCr':
        y, cb, cr = o.planes()
        print('  Y00 Cb00 Cr00', y[0], cb[0], cr[0], 'got', got[0,0], 'want', want[0,0])
        # where do diffs occur
        ys, xs = np.nonzero(diff.sum(-1))
        if len(ys): print('  first diff at', ys[0], xs[0], 'rows', np.unique(ys)[:10], 'cols', np.unique(xs)[:10])
