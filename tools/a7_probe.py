"""Adam7 RGBA16 probe (diagnostic): ms per launch of 64 x 4K Adam7 RGBA16
images, the plan's two launches together (HIP events), for the library at
ZPX_LIB_PATH (default: the in-tree build).  Usage: python tools/a7_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import torch  # noqa: E402

from tools import synthetic as S  # noqa: E402
from tools.png_probe import timed  # noqa: E402
from zpix_amd import device, png  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
d = S.png_rgba16_adam7(2000, size, size)
pb = device.PngBatch([png.Stream(d)], slots=[0] * 64)
print(os.environ.get("ZPX_LIB_PATH", "in-tree"), "adam7 rgba16 ms:", round(timed(pb), 3), round(timed(pb), 3), flush=True)
