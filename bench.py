"""Benchmark: MPixels/sec decoded, 4K baseline JPEG 4:2:0, fused dequant + IDCT
+ upsample + YCbCr->RGBA on MI355X (BASELINE.json configs[1]).

A step = one launch of the device plan over the batch (64 synthetic 4096x4096
q75 4:2:0 frames per GPU, coefficient grids resident in HBM, RGBA written to
HBM).  Host entropy decoding happens before the timed region (it is reported
separately as host_entropy_mpix_s).  Multi-GPU: one process per GPU
(torch.distributed over RCCL), each rank decodes its own 64 frames (weak
scaling, no data-path collective).

configs[3] is the "end_to_end" line: this rank's shard of the mixed
JPEG+PNG batch (image i -> rank i mod N) from encoded bytes in host memory
to RGBA8 in HBM, then (N > 1) ONE RCCL gather of every rank's RGBA arena to
rank 0, timed and reported apart ("gather"); zpix_amd/shard.py holds the
placement, shared with tests/test_distributed.py.

The PNG workload (configs[2]: 64 x 4096^2 tc8, mixed Sub/Up/Avg/Paeth rows)
is measured in the same run and reported under "png" (disable: --no-png):
from the inflated stream in HBM, as parseIdat hands it to readImagePass,
with the host-built band slab as its "slab_input" sub-line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

PEAK_HBM_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
MEASURED_COPY_GBS = 6290.0  # float4 copy measured on MI355X (same guide)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--images", type=int, default=64, help="frames per GPU")
    ap.add_argument("--distinct", type=int, default=4, help="distinct synthetic frames per GPU (slots cycle them)")
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--quality", type=int, default=75)
    ap.add_argument("--no-png", action="store_true")
    ap.add_argument("--png-only", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=16.0, help="bound on the CPU baseline samples (JPEG + PNG)")
    ap.add_argument("--no-gather", action="store_true",
                    help="N>1: skip the RCCL gather of the end-to-end batch's RGBA to rank 0")
    ap.add_argument("--no-adam7", action="store_true", help="configs[4]: progressive JPEG line only (A/B runs)")
    ap.add_argument("--no-config5", action="store_true",
                    help="skip configs[4]: progressive 4:4:4 JPEG + Adam7 RGBA16 PNG (worst-case control flow)")
    ap.add_argument("--no-planar", action="store_true",
                    help="skip the planar line (jpeg.load: the headline frames into Y/Cb/Cr planes)")
    ap.add_argument("--no-pieces", action="store_true", help="skip the pieces-transport lines")
    ap.add_argument("--no-strip", action="store_true",
                    help="skip the odd-width line (4094-wide 4:2:0 frames: block kernel, and the strip-kernel fallback forced)")
    ap.add_argument("--gather-chunks", type=int, default=8,
                    help="N>1: the end-to-end gather moves each rank's shard in this many chunks, each as soon "
                         "as it is decoded (1: one gather after the whole decode)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the end-to-end streaming line (host entropy threads + H2D + kernels)")
    ap.add_argument("--e2e-images", type=int, default=64,
                    help="encoded images per GPU in the end-to-end batch (configs[3]: 512 over 8 GPUs)")
    ap.add_argument("--host-threads", type=int, default=0,
                    help="host entropy/inflate threads per rank (end-to-end); 0 = this rank's share of the host")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="per-launch HBM bytes measured by rocprofv3 --pmc (see profiles/)")
    return ap.parse_args()


def traffic_of(args, line: str):
    """HBM bytes per launch of a bench line's plan from rocprofv3 --pmc
    (tools/pmc_summary.py writes profiles/traffic.json: FETCH_SIZE x2 +
    WRITE_SIZE, summed over the plan's kernels), or None when not measured
    for this workload."""
    try:
        tj = json.load(open(args.traffic_json))
        if tj.get("images") == args.images and tj.get("size") == args.size and line in tj:
            return tj[line]["hbm_bytes_per_launch"]
    except Exception:
        pass
    return None


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def shard_images(total: int, rank: int, ws: int) -> list[int]:
    """Global image ids owned by `rank`: image i -> GPU i mod N."""
    from zpix_amd.shard import shard_images as f

    return f(total, rank, ws)


def e2e_is_jpeg(i: int, ws: int) -> bool:
    """configs[3]'s mix: image i is a 4K JPEG 4:2:0 when its index within its
    rank's shard (i // N) is even, else a 4K tc8 PNG -- every shard is half
    and half at every N (an even/odd split by global index would hand all
    JPEGs to even ranks and all PNGs to odd ones)."""
    return (i // ws) % 2 == 0


def max_over_ranks(dist, value: float, device) -> float:
    """The slowest rank's wall time (the whole job ends when it does)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    import torch

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_steps(torch, dist, launch, steps, warmup, ws):
    """W untimed steps; K timed steps bracketed by barrier + synchronize; HIP
    events on the launch stream give the average per-launch kernel time."""
    # a dedicated (non-null) stream: the plan launches on it and the HIP events
    # are recorded on it, so the event time is the kernels' time
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    for _ in range(warmup):
        launch(stream.cuda_stream)
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        launch(stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = e0.elapsed_time(e1) / steps
    return max_over_ranks(dist, wall, "cuda"), kern_ms


def cpu_info() -> dict:
    from zpix_amd.shard import host_cpu_budget

    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "budget": host_cpu_budget(),
            "cpu_model": model}


def _all_cores(fn, threads: int, seconds: float, t_one: float):
    """fn() on `threads` threads (ctypes drops the GIL inside the oracle), each
    repeating it to fill about `seconds`; returns (pixels, wall)."""
    per_thread = max(1, int(seconds / max(t_one, 1e-3) / 1.5))
    done = [0] * threads

    def worker(i):
        for _ in range(per_thread):
            done[i] += fn()

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return sum(done), time.perf_counter() - t0, per_thread


def cpu_baseline(jpeg_data: bytes, png_data: bytes | None, seconds: float) -> dict:
    """The oracle (C restatement of the reference algorithm, gcc -O2, scalar,
    one image per thread) timed on this box's host cores on bounded samples
    of the bench's own 4K inputs:

    - JPEG (the headline's metric): jpeg.decode + Image.rgbaPixels of one
      4096^2 q75 4:2:0 frame, on 1 core with the stage split entropy
      (processSos, decoder.zig:1148-1455) / reconstruct (reconstructBlock,
      :1553-1634) / rgbaPixels (image.zig:103-130), then on every usable core;
    - PNG: png.decode of one 4096^2 tc8 mixed-filter image, on 1 core split
      into inflate+chunks (png/decoder.zig:404-545) / unfilter+store
      (:649-1149), then on every usable core."""
    import numpy as np
    import oracle_py as O

    O.lib()
    info = cpu_info()
    cores = info["budget"]
    out = {"unit": "MPixels/sec", "cores": cores, "kind": "port", **info}
    # ---- JPEG, 1 core, stage split
    t0 = time.perf_counter()
    co = O.jpeg_coefficients(jpeg_data)
    t_ent = time.perf_counter() - t0
    from zpix_amd.device import jpeg_layout as _lay  # makeImg geometry (host arithmetic only)

    class _F:  # the frame fields jpeg_layout reads
        n_comp, mxx, myy, h, v = co.n_comp, co.mxx, co.myy, co.h, co.v

    lay = _lay(_F)
    planes_buf = np.zeros(lay.total, np.uint8)
    planes = [planes_buf[0:], planes_buf[lay.cb_off:], planes_buf[lay.cr_off:]][:co.n_comp]
    strides = [lay.y_stride] + [lay.c_stride] * (co.n_comp - 1)
    qts = [co.quant_zigzag[co.tq[c]] for c in range(co.n_comp)]
    tr = []
    O.reconstruct_grids(co.n_comp, co.width, co.height, co.h, co.v, co.mxx, co.myy, co.grids, qts,
                        co.progressive, planes, strides, timing=tr)
    t_rec = tr[0]
    img = O.jpeg_decode(jpeg_data)
    t0 = time.perf_counter()
    img.rgba_pixels()
    t_rgba = time.perf_counter() - t0
    px = img.width * img.height
    t1 = t_ent + t_rec + t_rgba

    def jpeg_one():
        im = O.jpeg_decode(jpeg_data)
        im.rgba_pixels()
        return im.width * im.height

    share = seconds / 2 if png_data is not None else seconds
    pix, wall, per = _all_cores(jpeg_one, cores, share, t1)
    out["value"] = round(pix / wall / 1e6, 2)
    out["sample"] = (f"JPEG: {cores} threads x {per} oracle jpeg.decode+rgbaPixels of one 4096x4096 q75 4:2:0 frame "
                     f"({wall:.1f}s); 1-core stage split on the same frame")
    out["jpeg"] = {"all_cores_mpix_s": out["value"], "single_core_mpix_s": round(px / t1 / 1e6, 2),
                   "stages_ms_1core": {"entropy": round(t_ent * 1e3, 1), "reconstruct": round(t_rec * 1e3, 1),
                                       "rgba_pixels": round(t_rgba * 1e3, 1)}}
    # ---- PNG, 1 core, stage split
    if png_data is not None:
        O.png_unfilter_seconds()
        t0 = time.perf_counter()
        pim = O.png_decode(png_data)
        t_all = time.perf_counter() - t0
        t_unf = O.png_unfilter_seconds()
        ppx = pim.width * pim.height

        def png_one():
            return O.png_decode(png_data).width * pim.height

        pix, wall, per = _all_cores(png_one, cores, share, t_all)
        out["png"] = {"all_cores_mpix_s": round(pix / wall / 1e6, 2), "single_core_mpix_s": round(ppx / t_all / 1e6, 2),
                      "stages_ms_1core": {"inflate_and_chunks": round((t_all - t_unf) * 1e3, 1),
                                          "unfilter_and_store": round(t_unf * 1e3, 1)},
                      "sample": f"{cores} threads x {per} oracle png.decode of one 4096x4096 tc8 mixed-filter PNG "
                                f"({wall:.1f}s)"}
    return out


def bench_config5(args, torch, dist, ws, rank, ctx, S, device, jpeg, png):
    """configs[4]: 4096^2 progressive 4:4:4 JPEG (fused kernel, 786,432 blocks
    per frame) and 4096^2 Adam7 RGBA16 PNG (7 passes scattered into NRGBA64),
    each as a resident batch of `images` slots; parity of slot 0 vs the oracle."""
    import numpy as np
    import oracle_py as O

    W = H = args.size
    out = {}
    d = S.jpeg_progressive_444(1000 + rank, W, H, args.quality)
    # host entropy: the best of three decodes (the first also starts the
    # decoder's worker threads)
    t_ent = None
    for _ in range(3):
        t0 = time.perf_counter()
        co = jpeg.Coefficients(d)
        dt = time.perf_counter() - t0
        t_ent = dt if t_ent is None else min(t_ent, dt)
    jb = device.JpegBatch([co], slots=[0] * args.images, output="rgba", ctx=ctx)
    if rank == 0:
        jb.launch(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        want = O.jpeg_decode(d).rgba_pixels()
        if not torch.equal(jb.output_tensor(0).reshape(-1).cpu(), torch.from_numpy(want)):
            raise SystemExit("parity failure: progressive 4:4:4 JPEG != oracle")
    steps = max(3, args.steps // 2)
    wall, kern_ms = timed_steps(torch, dist, jb.launch, steps, args.warmup, ws)
    out["jpeg_progressive_444"] = {
        "value": round(jb.pixels * ws * steps / wall / 1e6, 1), "unit": "MPixels/sec",
        "kernel_ms_per_launch": round(kern_ms, 3),
        "roofline": {"bound": "hbm", "achieved": round(jb.bytes / (kern_ms * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(jb.bytes / (kern_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                     "traffic": traffic_of(args, "progressive_444") if int(co.frame.coeff_bits) == 8 else None,
                     "algorithmic_bytes_per_launch": jb.bytes},
        "host_entropy_mpix_s": round(W * H / t_ent / 1e6, 1),
        "config": {"workload": f"{args.images}x {W}x{H} progressive 4:4:4 JPEG -> RGBA, configs[4]"}}
    del jb
    if args.no_adam7:
        return out
    pd = S.png_rgba16_adam7(2000 + rank, W, H)
    t0 = time.perf_counter()
    st = png.Stream(pd)
    t_inf = time.perf_counter() - t0
    pb = device.PngBatch([st], slots=[0] * args.images, ctx=ctx)
    if rank == 0:
        pb.launch(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        want = O.png_decode(pd).pixels
        got = pb.output_tensor(0).cpu().numpy()
        if not np.array_equal(got.reshape(-1)[:want.size], want.reshape(-1)):
            raise SystemExit("parity failure: Adam7 RGBA16 PNG != oracle")
    wall, kern_ms = timed_steps(torch, dist, pb.launch, steps, args.warmup, ws)
    pb.status(torch.cuda.current_stream().cuda_stream)  # raises "Hip" if any timed launch timed out
    abytes = pb.bytes
    slab_line = {
        "value": round(pb.pixels * ws * steps / wall / 1e6, 1), "kernel_ms_per_launch": round(kern_ms, 3),
        "frac": round(abytes / (kern_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
        "traffic": traffic_of(args, "adam7_rgba16_slab_input"),
        "note": "the band slab built on the host (zpx_png_stream_slab) and uploaded -> the slab instance"}
    del pb
    torch.cuda.empty_cache()
    # the line: from the inflated stream, the paired-row kernel's stream
    # instance (both launches) -- the path png.decode and the batch pipeline take
    sb = device.PngBatch([st], slots=[0] * args.images, ctx=ctx, layout="stream")
    if rank == 0:
        sb.launch(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        if not np.array_equal(sb.output_tensor(0).cpu().numpy().reshape(-1)[:want.size], want.reshape(-1)):
            raise SystemExit("parity failure: Adam7 RGBA16 PNG from the stream != oracle")
    swall, skern = timed_steps(torch, dist, sb.launch, steps, args.warmup, ws)
    sb.status(torch.cuda.current_stream().cuda_stream)
    out["png_adam7_rgba16"] = {
        "value": round(sb.pixels * ws * steps / swall / 1e6, 1), "unit": "MPixels/sec",
        "kernel_ms_per_launch": round(skern, 3),
        "roofline": {"bound": "hbm", "achieved": round(abytes / (skern * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(abytes / (skern * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                     "traffic": traffic_of(args, "adam7_rgba16_stream"), "algorithmic_bytes_per_launch": abytes,
                     "kernel": "png_pair_kernel<TCA16> (stream instance, two launches)"},
        "host_inflate_mpix_s": round(W * H / t_inf / 1e6, 1),
        "config": {"workload": f"{args.images}x {W}x{H} Adam7 RGBA16 PNG -> NRGBA64 from the inflated stream, "
                               "configs[4]"},
        "slab_input": slab_line}
    del sb
    torch.cuda.empty_cache()
    # Image.rgbaPixels of that NRGBA64 output (image.zig:103-130, the
    # premultiply of color.zig:73-89), resident batch, one plan launch
    import zpix_amd

    img = zpix_amd.from_buffer(pd)
    rb = device.RgbaBatch([img], slots=[0] * args.images, ctx=ctx)
    if rank == 0:
        rb.launch(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        if not np.array_equal(rb.output_tensor(0).cpu().numpy().reshape(-1), O.png_decode(pd).rgba_pixels()):
            raise SystemExit("parity failure: rgbaPixels of NRGBA64 != oracle")
    wall, kern_ms = timed_steps(torch, dist, rb.launch, steps, args.warmup, ws)
    ach = rb.bytes / (kern_ms * 1e-3) / 1e9
    out["rgba_pixels_nrgba64"] = {
        "value": round(rb.pixels * ws * steps / wall / 1e6, 1), "unit": "MPixels/sec",
        "kernel_ms_per_launch": round(kern_ms, 3),
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(ach / PEAK_HBM_GBS, 4), "kernel": "rgba_batch_kernel<NRGBA64>",
                     "traffic": traffic_of(args, "rgba_pixels_nrgba64"), "algorithmic_bytes_per_launch": rb.bytes},
        "config": {"workload": f"{args.images}x {W}x{H} NRGBA64 -> RGBA8 (Image.rgbaPixels), configs[4]'s Adam7 output"}}
    del rb
    torch.cuda.empty_cache()
    return out


def bench_planar(args, torch, dist, ws, rank, ctx, device, jpeg, datas):
    """jpeg.load's output (SURVEY §8(d) "2-planar"): the headline's frames
    reconstructed into makeImg's Y/Cb/Cr planes (reconstructBlock,
    src/jpeg/decoder.zig:1553-1634, :361-370) by the planar block kernel,
    resident batch of `images` slots, int8 and int16 transports; slot 0
    checked against the oracle's jpeg.decode planes before timing."""
    out = {}
    for bits in (8, 16):
        cos = [jpeg.Coefficients(d).widen(bits) for d in datas]
        if any(int(c.frame.coeff_bits) != bits for c in cos):
            continue
        slots = [i % len(cos) for i in range(args.images)]
        jb = device.JpegBatch(cos, slots=slots, output="planes", ctx=ctx)
        if rank == 0:
            import oracle_py as O

            jb.launch(torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            want = torch.from_numpy(O.jpeg_decode(datas[0]).pixels)
            if not torch.equal(jb.output_tensor(0).cpu(), want):
                raise SystemExit(f"parity failure: planar int{bits} planes != oracle")
        wall, kern_ms = timed_steps(torch, dist, jb.launch, args.steps, args.warmup, ws)
        ach = jb.bytes / (kern_ms * 1e-3) / 1e9
        out[f"int{bits}"] = {
            "value": round(jb.pixels * ws * args.steps / wall / 1e6, 1), "unit": "MPixels/sec",
            "kernel_ms_per_launch": round(kern_ms, 4),
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(ach / PEAK_HBM_GBS, 4), "kernel": "jpeg_plane_block_kernel",
                         "traffic": None, "algorithmic_bytes_per_launch": jb.bytes},
            "config": {"workload": f"{args.images}x {args.size}x{args.size} baseline 4:2:0 JPEG -> Y/Cb/Cr planes "
                                   f"(jpeg.load), int{bits} coefficients"}}
        out[f"int{bits}"]["roofline"]["traffic"] = traffic_of(args, f"planar_int{bits}")
        del jb
        torch.cuda.empty_cache()
    return out


def bench_pieces(args, torch, dist, ws, rank, ctx, device, jpeg, datas):
    """The headline's frames in the batch pipeline's compact transport
    (ZPX_COEFFS_PIECES: each block's coefficients in zig-zag order up to its
    last nonzero one, in 16-byte pieces, plus a uint32 index word a block;
    SURVEY §8(f)1), read straight into the block kernels' coefficient image --
    no dense grid is written or read back.  RGBA (the fused kernel) and
    jpeg.load's planes (the planar kernel); slot 0 of each checked against the
    oracle before timing.  Algorithmic bytes: the pieces + index words read,
    the output written."""
    import oracle_py as O

    out = {}
    cos = [jpeg.Coefficients(d, pieces=True) for d in datas]
    if not all(c.is_pieces for c in cos):
        return {"skipped": "frames not decoded into pieces"}
    bits = int(cos[0].frame.coeff_bits)
    slots = [i % len(cos) for i in range(args.images)]
    dense_int8 = sum(c.frame.mxx * c.frame.myy * 6 * 64 for c in (cos[i] for i in slots))
    for output, line in (("rgba", "rgba"), ("planes", "planes")):
        jb = device.JpegBatch(cos, slots=slots, output=output, ctx=ctx)
        if rank == 0:
            jb.launch(torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            ref = O.jpeg_decode(datas[0])
            want = torch.from_numpy(ref.rgba_pixels() if output == "rgba" else ref.pixels)
            if not torch.equal(jb.output_tensor(0).reshape(-1).cpu(), want.reshape(-1)):
                raise SystemExit(f"parity failure: pieces {output} != oracle")
        wall, kern_ms = timed_steps(torch, dist, jb.launch, args.steps, args.warmup, ws)
        ach = jb.bytes / (kern_ms * 1e-3) / 1e9
        kernel = "jpeg_block_kernel<pieces>" if output == "rgba" else "jpeg_plane_block_kernel<pieces>"
        pieces_bytes = sum(int(cos[i].frame.pieces_bytes) for i in slots)
        out[line] = {
            "value": round(jb.pixels * ws * args.steps / wall / 1e6, 1), "unit": "MPixels/sec",
            "kernel_ms_per_launch": round(kern_ms, 4),
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(ach / PEAK_HBM_GBS, 4), "kernel": kernel,
                         "traffic": traffic_of(args, f"pieces_{line}"), "algorithmic_bytes_per_launch": jb.bytes},
            "coefficient_bytes_per_launch": {"pieces": pieces_bytes,
                                             "index": sum(sum(cos[i].coeff_bytes) for i in slots),
                                             "dense_int8_grids": dense_int8},
            "config": {"workload": f"{args.images}x {args.size}x{args.size} baseline 4:2:0 JPEG from pieces -> "
                                   + ("RGBA" if output == "rgba" else "Y/Cb/Cr planes (jpeg.load)")
                                   + f", int{bits} pieces"}}
        del jb
        torch.cuda.empty_cache()
    return out


class _Regeom:
    """A host-decoded frame's coefficient grids under another MCU geometry
    (the same bytes: for 4:1:1 at 4096^2 the luma grid keeps its 512 x 512
    blocks and the 65,536 chroma blocks of each 4:2:0 grid become 128 x 512)."""

    def __init__(self, co, h, v, mxx, myy):
        import ctypes as C

        from zpix_amd import _lib

        self.frame = _lib.zpx_jpeg_frame()
        C.pointer(self.frame)[0] = co.frame
        for c in range(3):
            self.frame.h[c], self.frame.v[c] = h[c], v[c]
        self.frame.mxx, self.frame.myy = mxx, myy
        self.coeff_bytes = list(co.coeff_bytes)
        for c in range(3):
            assert self.coeff_bytes[c] == mxx * h[c] * myy * v[c] * 64 * int(co.frame.coeff_bits) // 8
        self._co = co  # (the grids' host memory)


def bench_odd_geometry(args, torch, dist, ws, rank, ctx, device, jpeg, datas):
    """4:1:1 frames (h0 = 4: the MCU is 4 luma blocks wide), the geometry
    the strip kernel took until round 4, now on the block kernel: the
    headline frame's grids re-read as 4:1:1 (_Regeom), `images` slots, slot
    0 checked against the oracle's reconstructBlock (decoder.zig:1553-1634)
    + Image.rgbaPixels (image.zig:103-130, cOffset for Ratio411)."""
    import ctypes as C

    import numpy as np
    import oracle_py as O

    W = H = args.size
    co = jpeg.Coefficients(datas[0])
    fr = _Regeom(co, [4, 1, 1], [1, 1, 1], W // 32, H // 8)
    jb = device.JpegBatch([fr], slots=[0] * args.images, output="rgba", ctx=ctx)
    if rank == 0:
        jb.launch(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        f = fr.frame
        dt = {8: np.int8, 16: np.int16}[int(f.coeff_bits)]
        grids = [np.ctypeslib.as_array(C.cast(f.coeffs[c], C.POINTER(C.c_uint8)), shape=(fr.coeff_bytes[c],))
                 .view(dt).astype(np.int32).reshape(-1, 64) for c in range(3)]
        unzig = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
                 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45,
                 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63]
        qz = [np.array([f.qt[c][unzig[z]] for z in range(64)], np.int32) for c in range(3)]
        strides = [f.mxx * 4 * 8, f.mxx * 8, f.mxx * 8]
        planes = [np.zeros(strides[c] * f.myy * 8, np.uint8) for c in range(3)]
        O.reconstruct_grids(3, W, H, [4, 1, 1], [1, 1, 1], f.mxx, f.myy, grids, qz, False, planes, strides)
        buf = np.concatenate(planes)
        img = O.ZoImage(kind=2, min_x=0, min_y=0, max_x=W, max_y=H, y_off=0, cb_off=planes[0].size,
                        cr_off=planes[0].size + planes[1].size, y_stride=strides[0], c_stride=strides[1], subsample=4)
        img.pixels = buf.ctypes.data_as(C.POINTER(C.c_uint8))
        img.pixels_len = buf.size
        want = np.zeros(W * H * 4, np.uint8)
        O.lib().zo_rgba_pixels(C.byref(img), want.ctypes.data)
        if not np.array_equal(jb.output_tensor(0).reshape(-1).cpu().numpy(), want):
            raise SystemExit("parity failure: 4:1:1 frame on the block kernel != oracle")
    steps = max(3, args.steps // 2)
    wall, kern_ms = timed_steps(torch, dist, jb.launch, steps, args.warmup, ws)
    ach = jb.bytes / (kern_ms * 1e-3) / 1e9
    out = {"value": round(jb.pixels * ws * steps / wall / 1e6, 1), "unit": "MPixels/sec",
           "kernel_ms_per_launch": round(kern_ms, 3),
           "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": round(ach / PEAK_HBM_GBS, 4), "kernel": "jpeg_block_kernel<4,1,1,1>",
                        "algorithmic_bytes_per_launch": jb.bytes},
           "coeff_bits": int(fr.frame.coeff_bits),
           "config": {"workload": f"{args.images}x {W}x{H} 4:1:1 JPEG -> RGBA (the headline frames' grids as "
                                  "4:1:1 MCUs), block kernel"}}
    del jb
    torch.cuda.empty_cache()
    return out


def bench_strip(args, torch, dist, ws, rank, ctx, S, device, jpeg):
    """4094x4096 4:2:0 frames (width % 4 != 0: rows only dword aligned, each
    row's last 4-pixel piece partial), `images` slots of one frame, slot 0
    checked against the oracle: on the block kernel (its partial-piece path),
    and -- the fused path's fallback, what every frame the block kernel
    refuses (int32, non-narrow, 4:1:1, 2x2 chroma) takes -- on the strip
    kernel through the test switch "jpeg_strip" (zpx_debug_option).  The
    reference runs reconstructBlock on every frame shape
    (decoder.zig:1553-1634)."""
    from zpix_amd import _lib

    W, H = args.size - 2, args.size
    d = S.jpeg_420(3000 + rank, W, H, args.quality)
    co = jpeg.Coefficients(d)
    out = None
    for kernel, strip in (("jpeg_block_kernel", 0), ("jpeg_rgba_kernel", 1)):
        prev = _lib.lib().zpx_debug_option(b"jpeg_strip", strip)
        try:
            jb = device.JpegBatch([co], slots=[0] * args.images, output="rgba", ctx=ctx)
            if rank == 0:
                import oracle_py as O

                jb.launch(torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                want = O.jpeg_decode(d).rgba_pixels()
                if not torch.equal(jb.output_tensor(0).reshape(-1).cpu(), torch.from_numpy(want)):
                    raise SystemExit(f"parity failure: {kernel} on a width % 4 != 0 JPEG != oracle")
            steps = max(3, args.steps // 2)
            wall, kern_ms = timed_steps(torch, dist, jb.launch, steps, args.warmup, ws)
        finally:
            _lib.lib().zpx_debug_option(b"jpeg_strip", prev)
        ach = jb.bytes / (kern_ms * 1e-3) / 1e9
        line = {"value": round(jb.pixels * ws * steps / wall / 1e6, 1), "unit": "MPixels/sec",
                "kernel_ms_per_launch": round(kern_ms, 3),
                "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": round(ach / PEAK_HBM_GBS, 4), "kernel": kernel,
                             "algorithmic_bytes_per_launch": jb.bytes},
                "coeff_bits": int(co.frame.coeff_bits),
                "config": {"workload": f"{args.images}x {W}x{H} baseline 4:2:0 JPEG -> RGBA (width % 4 != 0) "
                                       f"through {kernel}"}}
        del jb
        torch.cuda.empty_cache()
        if out is None:
            out = line
        else:
            out["strip_kernel"] = line
    return out


def bench_e2e(args, torch, dist, ws, rank, ctx, S, threads):
    """configs[3], end to end from encoded bytes in host memory: this rank's
    shard of the mixed JPEG+PNG batch (image i -> rank i mod N) through
    zpx_batch_decode_rgba -- host entropy/inflate workers overlapped with
    pinned H2D copies and the kernels -- into this rank's RGBA8 arena in HBM,
    and (N > 1) every arena gathered to rank 0 over RCCL in --gather-chunks
    chunks, each as soon as this rank has decoded it (batch.start_rgba +
    zpx_batch_wait_prefix), so the gather overlaps the decode of later
    chunks.  The placement is zpix_amd.shard's (shared with the gloo test).
    Never `value`: it is bound by the host's serial Huffman/inflate work."""
    from zpix_amd import batch, shard

    W = H = args.size
    total = args.e2e_images * ws
    uniq = {True: S.jpeg_420(0, W, H, args.quality), False: S.png_tc8_mixed(1, W, H)}
    bufs = [uniq[e2e_is_jpeg(i, ws)] for i in range(total)]
    gather = ws > 1 and not args.no_gather
    plan = shard.ShardPlan([(W, H)] * total, ws, chunks=max(1, args.gather_chunks) if gather else 1)

    def decode_fn(my_bufs, dsts):
        res, st = batch.decode_rgba(my_bufs, host_threads=threads, ctx=ctx, dst=dsts, with_stats=True)
        return [r.status for r in res], st

    # warm-up (code objects, and the pinned host buffer pool at the steady
    # state of a long-running decoder: one untimed pass over this rank's
    # whole shard, so the timed pass does not pin fresh pages for every
    # in-flight image)
    mine = [bufs[i] for i in plan.owned[rank]]
    warm = torch.empty(len(mine) * W * H * 4, dtype=torch.uint8, device="cuda")
    decode_fn(mine, [warm[k * W * H * 4:(k + 1) * W * H * 4].view(H, W, 4) for k in range(len(mine))])
    del warm
    def start_fn(my_bufs, dsts):
        return batch.start_rgba(my_bufs, host_threads=threads, ctx=ctx, dst=dsts)

    r = shard.decode_and_gather(bufs, plan, rank, dist if ws > 1 else None, decode_fn, "cuda", gather=gather,
                                sync=torch.cuda.synchronize, start_fn=start_fn if plan.chunks > 1 else None)
    wall = max_over_ranks(dist, r.decode_s, "cuda")
    bad = sorted({s for s in r.statuses.values() if s != "Ok"})
    if bad:
        raise SystemExit(f"end-to-end batch failed: {bad[:3]}")
    st = r.stats
    out = {"value": round(total * W * H / wall / 1e6, 1), "unit": "MPixels/sec",
           "per_gpu_mpix_s": round(total * W * H / wall / 1e6 / ws, 1),
           "images": total, "images_per_gpu": len(plan.owned[rank]), "host_threads_per_rank": st.host_threads,
           "depth": st.depth, "decode_wall_s": round(wall, 3), "host_cpu_s_rank0": round(st.host_s, 3),
           "host_cpu_s_by_stage_rank0": {
               "jpeg_entropy": round(st.host_jpeg_s, 3), "jpeg_items": st.jpeg_items,
               "png_inflate": round(st.host_png_s, 3), "png_items": st.png_items},
           "h2d_gb_rank0": round(st.h2d_bytes / 1e9, 3),
           "config": {"workload": f"{total}x {W}x{H} JPEG 4:2:0 / tc8 PNG (half each per shard), encoded bytes in "
                                  f"host memory -> RGBA8 in HBM (zpx_batch_decode_rgba), image i -> GPU i mod {ws}"
                                  + (", RCCL gather to rank 0" if gather else ""), "configs": "configs[3]"}}
    if gather:
        gs = max_over_ranks(dist, r.gather_s, "cuda")
        job = max_over_ranks(dist, r.wall_s, "cuda")
        tail = max_over_ranks(dist, r.tail_s, "cuda")
        out["with_gather"] = {"value": round(total * W * H / job / 1e6, 1), "unit": "MPixels/sec",
                              "wall_s": round(job, 3), "note": "decode + the gather's tail: every image on rank 0"}
        out["gather"] = {"bytes": plan.gather_bytes, "seconds": round(gs, 4), "tail_s": round(tail, 4),
                         "chunks": plan.chunks, "GB_s": round(plan.gather_bytes / gs / 1e9, 1),
                         "collective": f"torch.distributed.gather (RCCL), {plan.chunks} chunks overlapped with decode"}
        if rank == 0:  # spot-check the gathered placement: one image of every rank against its source
            import numpy as np
            import oracle_py as O

            want = {k: O.decode(uniq[k]).rgba_pixels() for k in (True, False)}
            for q in range(ws):
                i = plan.owned[q][-1]
                got = r.image(plan, i).reshape(-1).cpu().numpy()
                if not np.array_equal(got, want[e2e_is_jpeg(i, ws)]):
                    raise SystemExit(f"gather parity failure: image {i} from rank {q}")
    del r
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    ws, rank, local = dist_env()
    import numpy as np
    import torch

    dist = None
    if ws > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    # this rank's share of the host (entropy threads + the CPUs they run on)
    from zpix_amd.shard import rank_cpus

    local_ws = int(os.environ.get("LOCAL_WORLD_SIZE", str(ws)))
    threads, cpus = rank_cpus(local, local_ws)
    if args.host_threads:
        threads = args.host_threads
    if ws > 1:
        os.sched_setaffinity(0, cpus)

    from tools import synthetic as S

    import zpix_amd
    from zpix_amd import device, jpeg, png

    ctx = zpix_amd.context.default(dev)
    W = H = args.size
    result = {}
    pdatas = []
    # ------------------------------------------------------------ JPEG (headline)
    if not args.png_only:
        t0 = time.perf_counter()
        mine = shard_images(args.images * ws, rank, ws)  # this rank's global image ids
        # the first `distinct` ids of the shard are synthesised (seed = image id); slots cycle them
        datas = [S.jpeg_420(i, W, H, args.quality) for i in mine[:args.distinct]]
        t_gen = time.perf_counter() - t0
        t0 = time.perf_counter()
        coeffs = [jpeg.Coefficients(d) for d in datas]
        t_ent = time.perf_counter() - t0
        host_entropy = args.distinct * W * H / t_ent / 1e6
        log(f"[rank {rank}] generated {args.distinct} frames in {t_gen:.1f}s; host entropy "
            f"{host_entropy:.1f} MPix/s (1 thread)")
        slots = [i % args.distinct for i in range(args.images)]
        batch = device.JpegBatch(coeffs, slots=slots, output="rgba", ctx=ctx)
        # parity gate before timing: slot 0 vs the oracle (rank 0, cheap at 4K)
        if rank == 0 and not os.environ.get("ZPX_BENCH_TIMING_ONLY"):  # (timing-only A/B builds skip the gate)
            import oracle_py as O

            batch.launch(torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            want = O.jpeg_decode(datas[0]).rgba_pixels()
            ok = torch.equal(batch.output_tensor(0).reshape(-1).cpu(), torch.from_numpy(want))
            if not ok:
                raise SystemExit("parity failure: GPU RGBA != oracle for frame 0")
        wall, kern_ms = timed_steps(torch, dist, batch.launch, args.steps, args.warmup, ws)
        px_per_step = batch.pixels * ws
        value = px_per_step * args.steps / wall / 1e6
        launch_bytes = batch.bytes
        achieved = launch_bytes / (kern_ms * 1e-3) / 1e9
        jkernel = "jpeg_block_kernel"  # the kernel the plan runs on these frames (jpeg_kernels.hip)
        coeff_bits = int(coeffs[0].frame.coeff_bits)
        traffic = traffic_of(args, "headline") if coeff_bits == 8 else None
        # the same frames through the int16 transport (what a frame with any
        # |coefficient| > 127 takes), for comparison: kernel time only
        int16 = None
        if coeff_bits < 16 and os.environ.get("ZPX_BENCH_NO_INT16", "0") != "1":
            del batch
            torch.cuda.empty_cache()
            for co in coeffs:
                co.widen(16)
            batch = device.JpegBatch(coeffs, slots=slots, output="rgba", ctx=ctx)
            _, k16 = timed_steps(torch, dist, batch.launch, args.steps, args.warmup, ws)
            a16 = batch.bytes / (k16 * 1e-3) / 1e9
            int16 = {"kernel_ms_per_launch": round(k16, 4), "algorithmic_bytes_per_launch": batch.bytes,
                     "mpix_s_kernel_only": round(batch.pixels * ws / (k16 * 1e-3) / 1e6, 1),
                     "achieved": round(a16, 1), "frac": round(a16 / PEAK_HBM_GBS, 4),
                     "traffic": traffic_of(args, "int16")}
        result = {
            "metric": "MPixels/sec decoded (4K baseline JPEG 4:2:0) at 1/8 GPU; % HBM roofline",
            "value": round(value, 1),
            "unit": "MPixels/sec",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": f"int32 (int{coeff_bits} coefficients in, u8 RGBA out)",
            "data": f"synthetic: {args.images} x {W}x{H} q{args.quality} 4:2:0 baseline JPEG per GPU "
                    f"({args.distinct} distinct frames, Pillow), host-entropy-decoded before timing, "
                    "coefficients resident in HBM",
            "config": {"workload": f"{args.images}x {W}x{H} baseline 4:2:0 JPEG -> RGBA (fused dequant+IDCT+"
                                   "upsample+YCbCr->RGB), configs[1]",
                       "images_per_gpu": args.images, "width": W, "height": H, "quality": args.quality,
                       "coeff_bits": coeff_bits, "parallelism": f"image-sharded x{ws}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                         "frac_of_measured_copy": round(achieved / MEASURED_COPY_GBS, 4),
                         "kernel": jkernel, "kernel_ms_per_launch": round(kern_ms, 4),
                         "algorithmic_bytes_per_launch": launch_bytes},
            "host_entropy_mpix_s": round(host_entropy, 1),
        }
        if int16:
            result["int16_transport"] = int16
        del batch
        torch.cuda.empty_cache()
    # ------------------------------------------------------------ PNG (configs[2])
    if not args.no_png:
        from zpix_amd import _lib
        t0 = time.perf_counter()
        mine = shard_images(args.images * ws, rank, ws)
        pdatas = [S.png_tc8_mixed(i, W, H) for i in mine[:args.distinct]]
        t_gen = time.perf_counter() - t0
        t0 = time.perf_counter()
        streams = [png.Stream(d) for d in pdatas]
        t_inf = time.perf_counter() - t0
        t0 = time.perf_counter()
        for st in streams:  # the paired-row kernel's band slab (host, png_slab.cpp; PngBatch reuses it)
            st.slab()
        t_slab = time.perf_counter() - t0
        log(f"[rank {rank}] PNG generated in {t_gen:.1f}s, host inflate {args.distinct * W * H / t_inf / 1e6:.1f} MPix/s")
        slots = [i % args.distinct for i in range(args.images)]
        pb = device.PngBatch(streams, slots=slots, ctx=ctx)
        if rank == 0:
            raw, _ = S.png_filtered_tc8(0, W, H)
            pb.launch(torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            got = pb.output_tensor(0).cpu().numpy().reshape(H, W, 4)
            if not np.array_equal(got[..., :3], raw.reshape(H, W, 3)):
                raise SystemExit("parity failure: GPU PNG unfilter != source pixels")
        wall, kern_ms = timed_steps(torch, dist, pb.launch, max(3, args.steps // 2), args.warmup, ws)
        pb.status(torch.cuda.current_stream().cuda_stream)  # raises "Hip" if any timed launch timed out
        steps = max(3, args.steps // 2)
        pv = pb.pixels * ws * steps / wall / 1e6
        ach = pb.bytes / (kern_ms * 1e-3) / 1e9
        pkernel = "png_pair_kernel<TC8>"
        slab_traffic = traffic_of(args, "png_slab_input")
        slab_line = {
            "value": round(pv, 1), "unit": "MPixels/sec", "kernel_ms_per_launch": round(kern_ms, 3),
            "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": slab_traffic,
                         "kernel": pkernel + " (slab instance)", "algorithmic_bytes_per_launch": pb.bytes},
            "host_slab_mpix_s": round(args.distinct * W * H / t_slab / 1e6, 1),
            "note": "the band slab built on the host (zpx_png_stream_slab, png_slab.cpp) and uploaded; the kernel "
                    "reads 1 KiB contiguous per load instruction"}
        del pb
        torch.cuda.empty_cache()

        # the line: the images from the inflated stream (what parseIdat hands
        # readImagePass, png/decoder.zig:516-523), read as is by the
        # paired-row kernel's stream instance -- the path png.decode and the
        # batch pipeline take.  Beside it the round-4 path: a band slab built
        # on the device at every launch (png_slab_kernels.hip), then the slab
        # instance (test switch png_device_slab)
        def stream_line(dev_slab):
            prev = _lib.lib().zpx_debug_option(b"png_device_slab", int(dev_slab))
            try:
                sb = device.PngBatch(streams, slots=slots, ctx=ctx, layout="stream")
            finally:
                _lib.lib().zpx_debug_option(b"png_device_slab", prev)
            if rank == 0:
                sb.launch(torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                got = sb.output_tensor(0).cpu().numpy().reshape(H, W, 4)
                if not np.array_equal(got[..., :3], raw.reshape(H, W, 3)):
                    raise SystemExit("parity failure: GPU PNG from the stream != source pixels")
            swall, skern = timed_steps(torch, dist, sb.launch, steps, args.warmup, ws)
            sb.status(torch.cuda.current_stream().cuda_stream)  # raises "Hip" if any timed launch timed out
            r = (sb.pixels * ws * steps / swall / 1e6, swall, skern, sb.bytes)
            del sb
            torch.cuda.empty_cache()
            return r

        sv, swall, skern, sbytes = stream_line(False)
        sach = sbytes / (skern * 1e-3) / 1e9
        dv, _, dkern, _ = stream_line(True)
        dach = sbytes / (dkern * 1e-3) / 1e9
        dtraffic = traffic_of(args, "png_slab_build")
        pres = {"metric": "MPixels/sec decoded (4K truecolor-8 PNG, mixed Sub/Up/Avg/Paeth)", "value": round(sv, 1),
                "unit": "MPixels/sec", "steps": steps, "ms_per_step": round(swall / steps * 1e3, 3),
                "config": {"workload": f"{args.images}x {W}x{H} tc8 PNG unfilter -> RGBA from the inflated stream, "
                                       "configs[2]"},
                "roofline": {"bound": "hbm", "achieved": round(sach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": round(sach / PEAK_HBM_GBS, 4), "traffic": traffic_of(args, "png_stream"),
                             "kernel": pkernel + " (stream instance)", "kernel_ms_per_launch": round(skern, 3),
                             "algorithmic_bytes_per_launch": sbytes},
                "note": "inflated stream in HBM -> unfilter -> RGBA: one kernel, the whole device path",
                "host_inflate_mpix_s": round(args.distinct * W * H / t_inf / 1e6, 1),
                "slab_input": slab_line,
                "device_slab": {
                    "value": round(dv, 1), "kernel_ms_per_launch": round(dkern, 3),
                    "frac": round(dach / PEAK_HBM_GBS, 4), "kernel": "png_slab_kernel<12> + " + pkernel,
                    "traffic": dtraffic + slab_traffic if dtraffic and slab_traffic else None,
                    "note": "the stream with the band slab built on the device at every launch, then the slab "
                            "instance (test switch png_device_slab)"}}
        if result:
            result["png"] = pres
        else:
            result = dict(pres, n_gpus=ws, warmup=args.warmup, higher_is_better=True, scaling="weak", vs_baseline=None,
                          dtype="u8", data="synthetic PNG")
    # ------------------------------------------------------------ planar (jpeg.load)
    if not args.no_planar and not args.png_only:
        result["planar"] = bench_planar(args, torch, dist, ws, rank, ctx, device, jpeg, datas)
    # ------------------------------------------------------------ the compact (pieces) transport
    if not args.no_pieces and not args.png_only:
        result["pieces"] = bench_pieces(args, torch, dist, ws, rank, ctx, device, jpeg, datas)
    # ------------------------------------------------------------ configs[4] and end to end
    if not args.no_config5 and not args.png_only:
        result["config5"] = bench_config5(args, torch, dist, ws, rank, ctx, S, device, jpeg, png)
    if not args.no_strip and not args.png_only:
        result["odd_width"] = bench_strip(args, torch, dist, ws, rank, ctx, S, device, jpeg)
        result["odd_width"]["ratio411"] = bench_odd_geometry(args, torch, dist, ws, rank, ctx, device, jpeg, datas)
    if not args.no_e2e and not args.png_only:
        result["end_to_end"] = bench_e2e(args, torch, dist, ws, rank, ctx, S, threads)
    # ------------------------------------------------------------ CPU baseline (rank 0, N=1)
    if rank == 0 and ws == 1 and not args.no_cpu_baseline and not args.png_only:
        result["cpu_baseline"] = cpu_baseline(datas[0], pdatas[0] if pdatas else None, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
