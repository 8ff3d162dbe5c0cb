"""Decode the multi-band PNG fixtures one by one (GPU debug aid for the
band hand-off): prints each file's result against the oracle."""
import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import oracle_py as O  # noqa: E402
import zpix_amd  # noqa: E402
from tools import synthetic as S  # noqa: E402

items = [(p, open(p, "rb").read()) for p in sorted(glob.glob(os.path.join(ROOT, "tests/golden/testdata/*.png")))]
items += [("tc8_301x97", S.png_tc8_mixed(8, 301, 97)), ("tc8_1024x300", S.png_tc8_mixed(3, 1024, 300))]
if len(sys.argv) > 1:
    items.append(("tc8_4096", S.png_tc8_mixed(0, 4096, 4096)))
for name, data in items:
    try:
        got = zpix_amd.png.decode(data)
        ref = O.png_decode(data)
        ok = got.kind == ref.kind and np.array_equal(got.pixels, ref.pixels)
        print(os.path.basename(name), "ok" if ok else "MISMATCH", flush=True)
    except Exception as e:  # noqa: BLE001
        print(os.path.basename(name), "ERROR", e, flush=True)
