"""Benchmark: MPixels/sec decoded, 4K baseline JPEG 4:2:0, fused dequant + IDCT
+ upsample + YCbCr->RGBA on MI355X (BASELINE.json configs[1]).

A step = one launch of the device plan over the batch (64 synthetic 4096x4096
q75 4:2:0 frames per GPU, coefficient grids resident in HBM, RGBA written to
HBM).  Host entropy decoding happens before the timed region (it is reported
separately as host_entropy_mpix_s).  Multi-GPU: one process per GPU
(torch.distributed over RCCL), each rank decodes its own 64 frames (weak
scaling, no data-path collective); `--gather` adds an RCCL gather of every
rank's RGBA to rank 0, timed separately.

The PNG workload (configs[2]: 64 x 4096^2 tc8, mixed Sub/Up/Avg/Paeth rows)
is measured in the same run and reported under "png" (disable: --no-png).
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
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bound on the CPU baseline sample")
    ap.add_argument("--gather", action="store_true", help="RCCL-gather all RGBA outputs to rank 0 (timed apart)")
    ap.add_argument("--no-config5", action="store_true",
                    help="skip configs[4]: progressive 4:4:4 JPEG + Adam7 RGBA16 PNG (worst-case control flow)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the end-to-end streaming line (host entropy threads + H2D + kernels)")
    ap.add_argument("--e2e-images", type=int, default=64,
                    help="encoded images per GPU in the end-to-end batch (configs[3]: 512 over 8 GPUs)")
    ap.add_argument("--host-threads", type=int, default=16, help="host entropy/inflate threads (end-to-end)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="per-launch HBM bytes measured by rocprofv3 --pmc (see profiles/)")
    return ap.parse_args()


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def shard_images(total: int, rank: int, ws: int) -> list[int]:
    """Global image ids owned by `rank`: image i -> GPU i mod N.
    Images are independent, so the shards share nothing."""
    return [i for i in range(total) if i % ws == rank]


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


def cpu_baseline_jpeg(data: bytes, seconds: float):
    """The oracle (C restatement of the reference algorithm, -O2, scalar) on a
    bounded sample: full jpeg.decode + Image.rgbaPixels of the same 4K frame,
    on all host cores (one frame per thread) and on one core."""
    import numpy as np  # noqa: F401
    import oracle_py as O

    O.lib()
    cores = min(16, os.cpu_count() or 1)

    def one():
        img = O.jpeg_decode(data)
        img.rgba_pixels()
        return img.width * img.height

    t0 = time.perf_counter()
    px1 = one()
    t1 = time.perf_counter() - t0
    single = px1 / t1 / 1e6
    # all cores: threads (ctypes releases the GIL inside the oracle)
    budget = max(seconds - t1, 1.0)
    per_thread = max(1, int(budget / t1 / 1.5))
    done = [0] * cores

    def worker(i):
        for _ in range(per_thread):
            done[i] += one()

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(cores)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    tm = time.perf_counter() - t0
    multi = sum(done) / tm / 1e6
    return {"value": round(multi, 2), "unit": "MPixels/sec", "cores": cores, "kind": "port",
            "sample": f"{cores * per_thread + 1} x oracle jpeg.decode+rgbaPixels of one 4096x4096 q75 4:2:0 frame "
                      f"({tm + t1:.1f}s)", "single_core_mpix_s": round(single, 2)}


def bench_config5(args, torch, dist, ws, rank, ctx, S, device, jpeg, png):
    """configs[4]: 4096^2 progressive 4:4:4 JPEG (fused kernel, 786,432 blocks
    per frame) and 4096^2 Adam7 RGBA16 PNG (7 passes scattered into NRGBA64),
    each as a resident batch of `images` slots; parity of slot 0 vs the oracle."""
    import numpy as np
    import oracle_py as O

    W = H = args.size
    out = {}
    d = S.jpeg_progressive_444(1000 + rank, W, H, args.quality)
    t0 = time.perf_counter()
    co = jpeg.Coefficients(d)
    t_ent = time.perf_counter() - t0
    jb = device.JpegBatch([co], slots=[0] * args.images, output="rgba", ctx=ctx)
    if rank == 0:
        jb.launch(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        want = O.jpeg_decode(d).rgba_pixels()
        if not torch.equal(jb.output_tensor(0).reshape(-1).cpu(), torch.from_numpy(want)):
            raise SystemExit("parity failure: progressive 4:4:4 JPEG != oracle")
    steps = max(3, args.steps // 2)
    wall, kern_ms = timed_steps(torch, dist, jb.launch, steps, 1, ws)
    out["jpeg_progressive_444"] = {
        "value": round(jb.pixels * ws * steps / wall / 1e6, 1), "unit": "MPixels/sec",
        "kernel_ms_per_launch": round(kern_ms, 3),
        "roofline": {"bound": "hbm", "achieved": round(jb.bytes / (kern_ms * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(jb.bytes / (kern_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                     "algorithmic_bytes_per_launch": jb.bytes},
        "host_entropy_mpix_s": round(W * H / t_ent / 1e6, 1),
        "config": {"workload": f"{args.images}x {W}x{H} progressive 4:4:4 JPEG -> RGBA, configs[4]"}}
    del jb
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
    wall, kern_ms = timed_steps(torch, dist, pb.launch, steps, 1, ws)
    out["png_adam7_rgba16"] = {
        "value": round(pb.pixels * ws * steps / wall / 1e6, 1), "unit": "MPixels/sec",
        "kernel_ms_per_launch": round(kern_ms, 3),
        "roofline": {"bound": "hbm", "achieved": round(pb.bytes / (kern_ms * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(pb.bytes / (kern_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                     "algorithmic_bytes_per_launch": pb.bytes},
        "host_inflate_mpix_s": round(W * H / t_inf / 1e6, 1),
        "config": {"workload": f"{args.images}x {W}x{H} Adam7 RGBA16 PNG -> NRGBA64, configs[4]"}}
    del pb
    torch.cuda.empty_cache()
    return out


def bench_e2e(args, torch, dist, ws, rank, ctx, S):
    """End to end, from encoded bytes in host memory: zpx_batch_decode_rgba
    with a pool of host entropy/inflate threads overlapped with pinned H2D
    copies and the kernels, RGBA8 into device memory (configs[3]'s per-GPU
    shard: alternating 4096^2 JPEG 4:2:0 and tc8 PNG).  Never `value`."""
    from zpix_amd import batch

    W = H = args.size
    mine = shard_images(args.e2e_images * ws, rank, ws)
    uniq = {0: S.jpeg_420(0, W, H, args.quality), 1: S.png_tc8_mixed(1, W, H)}
    bufs = [uniq[i % 2] for i in mine]
    batch.decode_rgba(bufs[:2], host_threads=args.host_threads, ctx=ctx)  # warm-up (pools, code objects)
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    t0 = time.perf_counter()
    res, st = batch.decode_rgba(bufs, host_threads=args.host_threads, ctx=ctx, with_stats=True)
    torch.cuda.synchronize()
    wall = max_over_ranks(dist, time.perf_counter() - t0, "cuda")
    bad = [r.status for r in res if r.status != "Ok"]
    if bad:
        raise SystemExit(f"end-to-end batch failed: {bad[:3]}")
    return {"value": round(len(bufs) * ws * W * H / wall / 1e6, 1), "unit": "MPixels/sec",
            "images_per_gpu": len(bufs), "host_threads": st.host_threads, "depth": st.depth,
            "wall_s": round(wall, 3), "host_cpu_s": round(st.host_s, 3),
            "h2d_gb": round(st.h2d_bytes / 1e9, 3),
            "config": {"workload": f"{len(bufs)}x {W}x{H} alternating JPEG 4:2:0 / tc8 PNG, encoded bytes in host "
                                   "memory -> RGBA8 in HBM (zpx_batch_decode_rgba), configs[3] shard"}}


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

    from tools import synthetic as S

    import zpix_amd
    from zpix_amd import device, jpeg, png

    ctx = zpix_amd.context.default(dev)
    W = H = args.size
    result = {}
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
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                if tj.get("images") == args.images and tj.get("size") == args.size and tj.get("kernel", "").startswith("jpeg_rgba"):
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        gather = None
        if args.gather and ws > 1:
            out = batch.out_arena
            bufs = [torch.empty_like(out) for _ in range(ws)] if rank == 0 else None
            torch.cuda.synchronize()
            dist.barrier()
            g0 = time.perf_counter()
            dist.gather(out, gather_list=bufs, dst=0)
            torch.cuda.synchronize()
            gt = time.perf_counter() - g0
            gather = {"bytes": int(out.numel() * (ws - 1)), "seconds": round(gt, 4),
                      "GB_s": round(out.numel() * (ws - 1) / gt / 1e9, 1)}
        coeff_bits = int(coeffs[0].frame.coeff_bits)
        if traffic is not None and tj.get("coeff_bits", 16) != coeff_bits:
            traffic = None  # measured on the other coefficient transport
        # the same frames through the int16 transport (what a frame with any
        # |coefficient| > 127 takes), for comparison: kernel time only
        int16 = None
        if coeff_bits < 16 and not os.environ.get("ZPX_BENCH_NO_INT16"):
            del batch
            torch.cuda.empty_cache()
            for co in coeffs:
                co.widen(16)
            batch = device.JpegBatch(coeffs, slots=slots, output="rgba", ctx=ctx)
            _, k16 = timed_steps(torch, dist, batch.launch, args.steps, args.warmup, ws)
            a16 = batch.bytes / (k16 * 1e-3) / 1e9
            int16 = {"kernel_ms_per_launch": round(k16, 4), "algorithmic_bytes_per_launch": batch.bytes,
                     "mpix_s_kernel_only": round(batch.pixels * ws / (k16 * 1e-3) / 1e6, 1),
                     "achieved": round(a16, 1), "frac": round(a16 / PEAK_HBM_GBS, 4), "traffic": None}
            t16 = os.path.join(os.path.dirname(args.traffic_json), "traffic_int16.json")
            try:
                tj16 = json.load(open(t16))
                if tj16.get("images") == args.images and tj16.get("size") == args.size:
                    int16["traffic"] = tj16.get("hbm_bytes_per_launch")
            except Exception:
                pass
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
                         "kernel": "jpeg_rgba_kernel", "kernel_ms_per_launch": round(kern_ms, 4),
                         "algorithmic_bytes_per_launch": launch_bytes},
            "host_entropy_mpix_s": round(host_entropy, 1),
        }
        if gather:
            result["gather"] = gather
        if int16:
            result["int16_transport"] = int16
        del batch
        torch.cuda.empty_cache()
    # ------------------------------------------------------------ PNG (configs[2])
    if not args.no_png:
        t0 = time.perf_counter()
        mine = shard_images(args.images * ws, rank, ws)
        pdatas = [S.png_tc8_mixed(i, W, H) for i in mine[:args.distinct]]
        t_gen = time.perf_counter() - t0
        t0 = time.perf_counter()
        streams = [png.Stream(d) for d in pdatas]
        t_inf = time.perf_counter() - t0
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
        wall, kern_ms = timed_steps(torch, dist, pb.launch, max(3, args.steps // 2), 1, ws)
        steps = max(3, args.steps // 2)
        pv = pb.pixels * ws * steps / wall / 1e6
        ach = pb.bytes / (kern_ms * 1e-3) / 1e9
        ptraffic = None
        try:
            tp = json.load(open(args.traffic_json)).get("png_unfilter", {})
            if tp.get("images") == args.images and tp.get("size") == args.size:
                ptraffic = tp.get("hbm_bytes_per_launch")
        except Exception:
            ptraffic = None
        pres = {"metric": "MPixels/sec decoded (4K truecolor-8 PNG, mixed Sub/Up/Avg/Paeth)", "value": round(pv, 1),
                "unit": "MPixels/sec", "steps": steps, "ms_per_step": round(wall / steps * 1e3, 3),
                "config": {"workload": f"{args.images}x {W}x{H} tc8 PNG unfilter -> RGBA, configs[2]"},
                "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": ptraffic, "kernel": "png_unfilter_kernel",
                             "kernel_ms_per_launch": round(kern_ms, 3), "algorithmic_bytes_per_launch": pb.bytes},
                "host_inflate_mpix_s": round(args.distinct * W * H / t_inf / 1e6, 1)}
        if result:
            result["png"] = pres
        else:
            result = dict(pres, n_gpus=ws, warmup=1, higher_is_better=True, scaling="weak", vs_baseline=None,
                          dtype="u8", data="synthetic PNG")
        del pb
    # ------------------------------------------------------------ configs[4] and end to end
    if not args.no_config5 and not args.png_only:
        result["config5"] = bench_config5(args, torch, dist, ws, rank, ctx, S, device, jpeg, png)
    if not args.no_e2e and not args.png_only:
        result["end_to_end"] = bench_e2e(args, torch, dist, ws, rank, ctx, S)
    # ------------------------------------------------------------ CPU baseline (rank 0, N=1)
    if rank == 0 and ws == 1 and not args.no_cpu_baseline and not args.png_only:
        result["cpu_baseline"] = cpu_baseline_jpeg(datas[0], args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
