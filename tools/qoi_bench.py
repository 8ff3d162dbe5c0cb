"""Times the GPU QOI encoder (device form, inputs resident in HBM) on a
4096^2 RGBA frame against the oracle's serial encoder; prints one JSON line."""
import json
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle_py as O  # noqa: E402
from tools import synthetic as S  # noqa: E402
from zpix_amd import context  # noqa: E402
from zpix_amd import qoi as Q  # noqa: E402


def main():
    w = h = int(os.environ.get("QOI_SIZE", "4096"))
    px = S.content(3, w, h, 4)
    px[100:900, 200:3000 % w] = px[100:900, 200 % w:200 % w + 1]
    desc = Q.Desc(w, h, 4, 0)
    cap = Q.encode_bound(desc)
    d_px = torch.from_numpy(px.reshape(-1)).cuda()
    d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx = context.default()
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    for _ in range(3):
        Q.encode_device(d_px.data_ptr(), desc, d_out.data_ptr(), cap, d_len.data_ptr(), st.cuda_stream, ctx)
    torch.cuda.synchronize()
    reps = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        Q.encode_device(d_px.data_ptr(), desc, d_out.data_ptr(), cap, d_len.data_ptr(), st.cuda_stream, ctx)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    n = int(d_len.item())
    t = time.perf_counter()
    ref = O.qoi_encode(px, w, h, 4, 0)
    cpu_s = time.perf_counter() - t
    ok = bytes(d_out[:n].cpu().numpy()) == ref
    print(json.dumps({"qoi_encode": {"size": w, "ms": round(ms, 4), "mpix_s": round(w * h / ms / 1e3, 1),
                                     "in_gb_s": round(w * h * 4 / ms / 1e6, 1), "bytes_out": n,
                                     "cpu_oracle_ms": round(cpu_s * 1e3, 2), "match": ok,
                                     "segment": os.environ.get("ZPX_QOI_SEGMENT", "128")}}))


if __name__ == "__main__":
    main()
