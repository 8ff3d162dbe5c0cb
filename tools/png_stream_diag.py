"""Diagnostic: the bench's tc8 PNG batch from the inflated stream (the
paired-row kernel's stream instance), checked image by image against the
generator's pixels; prints the mismatching rows (band, lane, half) and the
plan's status word.  Usage: python3 tools/png_stream_diag.py [launches]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tools import synthetic as S  # noqa: E402
from zpix_amd import device, png  # noqa: E402

W = H = 4096
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
streams = [png.Stream(S.png_tc8_mixed(i, W, H)) for i in range(4)]
slots = [i % 4 for i in range(64)]
sb = device.PngBatch(streams, slots=slots, layout="stream")
ref = device.PngBatch(streams, slots=list(range(4)))  # host slab: the reference output here
ref.launch(torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
want = [ref.output_tensor(i).cpu().numpy().reshape(H, W, 4) for i in range(4)]
for it in range(n):
    sb.launch(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    bad = 0
    for s in range(64):
        got = sb.output_tensor(s).cpu().numpy().reshape(H, W, 4)
        rows = np.nonzero((got != want[slots[s]]).any(axis=(1, 2)))[0]
        if rows.size:
            bad += 1
            if bad <= 4:
                cols = np.nonzero((got[rows[0]] != want[slots[s]][rows[0]]).any(axis=1))[0]
                print(f"launch {it} slot {s}: {rows.size} bad rows, first {rows[:8].tolist()} (band {rows[0] // 128}, "
                      f"row-in-band {rows[0] % 128}); first row bad cols {cols[:6].tolist()}..{cols[-3:].tolist()} "
                      f"({cols.size})", flush=True)
    try:
        sb.status(torch.cuda.current_stream().cuda_stream)
        st = "ok"
    except Exception as e:  # noqa: BLE001
        st = repr(e)
    print(f"launch {it}: {bad} of 64 images differ; status {st}", flush=True)
