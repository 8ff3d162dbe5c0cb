"""configs[3]: a batch of independent images sharded one-per-GPU, RGBA gathered to rank 0.

Image i goes to rank i mod N; a rank decodes its shard with
no data-path collective, then ONE gather moves every rank's RGBA arena to
rank 0 over RCCL (xGMI).  The reference has no counterpart -- zpix is
single-threaded and its facade decodes one image per call (src/root.zig:24-40)
-- so per image the result is `zpix.fromBuffer` + `Image.rgbaPixels`
(src/image/image.zig:103-130), and the batch adds only placement.

Two forms of the same placement:

- one process per GPU (what bench.py runs, torch.distributed: backend "nccl"
  is RCCL on ROCm): `ShardPlan` is the bookkeeping every rank derives
  identically from the host-only header sizes of the whole batch (decodeConfig
  is cheap): which images a rank owns, where each sits in the rank's RGBA
  arena, the arena size every rank pads to so one fixed-size gather moves them
  all, and where each image lands in rank 0's gathered buffer.
  `decode_and_gather()` runs a rank's shard through a decode function and
  gathers -- chunk by chunk while later chunks still decode, when the decode
  runs asynchronously (batch.start_rgba).  The CPU `gloo` test drives these
  same functions;
- one process, many GPUs: `decode_sharded()` over the C-ABI
  zpx_batch_decode_sharded (a pipeline thread per device, RCCL gather).
"""
from __future__ import annotations

import ctypes as C
import math
import os
import time
from dataclasses import dataclass, field

ALIGN = 256


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


def shard_images(total: int, rank: int, ws: int) -> list[int]:
    """Global image ids owned by `rank`: image i -> GPU i mod N."""
    return [i for i in range(total) if i % ws == rank]


@dataclass
class ShardPlan:
    """Placement of a batch of RGBA8 results across `ws` ranks.

    dims[i] = (width, height) of image i (None: the header did not parse --
    the image still belongs to its rank, which reports its error, but takes
    no arena space).

    chunks > 1 splits every rank's shard into that many consecutive runs of
    its images; an arena is laid out chunk after chunk, each chunk padded to
    the largest rank's bytes for it, so chunk c of every rank is one
    fixed-size gather that can run while chunk c+1 still decodes.  With
    chunks == 1 this is one gather of the whole arena."""

    dims: list
    ws: int
    chunks: int = 1
    owned: list = field(init=False)        # owned[r]: image ids of rank r, in order
    offset: dict = field(init=False)       # image id -> byte offset in its rank's arena
    arena_bytes: list = field(init=False)  # bytes rank r's images occupy (end of its last image)
    slot_bytes: int = field(init=False)    # the padded arena size every rank allocates
    per_chunk: int = field(init=False)     # images of a rank per chunk
    chunk_base: list = field(init=False)   # chunk c's byte offset in every arena
    chunk_bytes: list = field(init=False)  # chunk c's padded size (the largest rank's)

    def __post_init__(self):
        self.owned = [shard_images(len(self.dims), r, self.ws) for r in range(self.ws)]
        most = max((len(o) for o in self.owned), default=0)
        self.chunks = max(1, min(self.chunks, most)) if most else 1
        self.per_chunk = max(1, math.ceil(most / self.chunks)) if most else 1
        self.chunk_bytes = []
        for c in range(self.chunks):
            lo, hi = c * self.per_chunk, (c + 1) * self.per_chunk
            self.chunk_bytes.append(max(sum(_align(self.nbytes(i)) for i in o[lo:hi]) for o in self.owned))
        self.chunk_base = []
        acc = 0
        for nb in self.chunk_bytes:
            self.chunk_base.append(acc)
            acc += nb
        self.offset = {}
        self.arena_bytes = []
        for r in range(self.ws):
            end = 0
            for k, i in enumerate(self.owned[r]):
                c = k // self.per_chunk
                off = self.chunk_base[c] if k % self.per_chunk == 0 else end
                self.offset[i] = off
                end = off + _align(self.nbytes(i))
            self.arena_bytes.append(end)
        self.slot_bytes = max(ALIGN, acc)

    def nbytes(self, i: int) -> int:
        d = self.dims[i]
        return 0 if d is None else d[0] * d[1] * 4

    def owner(self, i: int) -> int:
        return i % self.ws

    def chunk_of(self, i: int) -> int:
        return (i // self.ws) // self.per_chunk

    def chunk_images(self, c: int, rank: int) -> tuple[int, int]:
        """Positions lo..hi-1 in rank `rank`'s shard that chunk c holds."""
        n = len(self.owned[rank])
        return min(n, c * self.per_chunk), min(n, (c + 1) * self.per_chunk)

    def gathered_offset(self, i: int) -> int:
        """Byte offset of image i in rank 0's gathered buffer (ws x slot_bytes,
        chunk-major: chunk c of rank q at ws * chunk_base[c] + q * chunk_bytes[c])."""
        c = self.chunk_of(i)
        return self.ws * self.chunk_base[c] + self.owner(i) * self.chunk_bytes[c] + self.offset[i] - self.chunk_base[c]

    @property
    def gather_bytes(self) -> int:
        """Bytes the gather moves into rank 0 (every other rank's slot)."""
        return (self.ws - 1) * self.slot_bytes


def rgba_view(arena, off: int, dims):
    """(H, W, 4) uint8 view of an arena at byte offset `off`."""
    w, h = dims
    return arena[off:off + w * h * 4].view(h, w, 4)


@dataclass
class ShardResult:
    statuses: dict             # image id -> error name ("Ok", ...), every image on rank 0, own ones elsewhere
    decode_s: float            # this rank's decode wall time
    gather_s: float | None     # from the first gather posted to the last complete (None: no gather ran)
    gathered: object = None    # rank 0: uint8 tensor (ws * slot_bytes) holding every image
    arena: object = None       # this rank's arena
    stats: object = None       # whatever decode_fn returned besides the statuses
    wall_s: float = 0.0        # decode start -> every gather complete (the job's end on this rank)
    tail_s: float = 0.0        # wall_s - decode_s: the gather not hidden behind the decode

    def image(self, plan: ShardPlan, i: int):
        """Rank 0, after a gather: image i's RGBA (H, W, 4)."""
        return rgba_view(self.gathered, plan.gathered_offset(i), plan.dims[i])


class ThreadedDecode:
    """The start protocol of decode_and_gather (wait / statuses / finish) for
    a per-image decode function on a Python thread: decode_one(buf, dst) ->
    error name.  What the CPU tests drive; the GPU path's counterpart is
    zpix_amd.batch.start_rgba (a native pipeline)."""

    def __init__(self, decode_one, bufs, dsts):
        import threading

        self._st = [None] * len(bufs)
        self._done = 0
        self._cv = threading.Condition()

        def run():
            for k, (b, d) in enumerate(zip(bufs, dsts)):
                s = decode_one(b, d)
                with self._cv:
                    self._st[k] = s
                    self._done = k + 1
                    self._cv.notify_all()

        self._th = threading.Thread(target=run, daemon=True)
        self._th.start()

    def wait(self, n: int) -> int:
        with self._cv:
            self._cv.wait_for(lambda: self._done >= n or not self._th.is_alive())
            return self._done

    def statuses(self, lo: int, hi: int) -> list:
        return self._st[lo:hi]

    def finish(self):
        self._th.join()
        return list(self._st), None


def decode_and_gather(buffers, plan: ShardPlan, rank: int, dist, decode_fn=None, device="cuda", gather: bool = True,
                      sync=None, start_fn=None) -> ShardResult:
    """Decode rank `rank`'s shard of `buffers` (the whole batch, indexed by
    global image id) into its arena, and gather every arena to rank 0.

    decode_fn(bufs, dsts) -> (statuses, stats): decodes bufs[k] into the
    (H, W, 4) tensor dsts[k] and returns one error name per image; the gather
    follows the whole decode.
    start_fn(bufs, dsts) -> a running decode with wait(n) / statuses(lo, hi) /
    finish() -> (statuses, stats) (batch.start_rgba, ThreadedDecode): chunk c
    of every rank is gathered (async) as soon as this rank's images of it are
    final, overlapping the decode of the chunks after it.
    sync(): waits for the device (torch.cuda.synchronize) before the clocks.
    """
    import torch

    ws = plan.ws
    mine = plan.owned[rank]
    arena = torch.empty(plan.slot_bytes, dtype=torch.uint8, device=device)
    dsts = [rgba_view(arena, plan.offset[i], plan.dims[i]) if plan.dims[i] is not None else None for i in mine]
    do_gather = gather and dist is not None and ws > 1
    gathered = None
    if do_gather and rank == 0:
        gathered = torch.empty(ws * plan.slot_bytes, dtype=torch.uint8, device=device)
    if sync:
        sync()
    if dist is not None and ws > 1:
        dist.barrier()
    works = []
    t_first = None

    def post(c):  # the async gather of chunk c of every rank into rank 0's chunk-major buffer
        nonlocal t_first
        base, nb = plan.chunk_base[c], plan.chunk_bytes[c]
        if nb == 0:
            return
        if t_first is None:
            t_first = time.perf_counter()
        glist = list(gathered[ws * base:ws * (base + nb)].view(ws, nb)) if rank == 0 else None
        works.append(dist.gather(arena[base:base + nb], gather_list=glist, dst=0, async_op=True))

    t0 = time.perf_counter()
    my_bufs = [buffers[i] for i in mine]
    if start_fn is not None:
        run = start_fn(my_bufs, dsts)
        for c in range(plan.chunks):
            _, hi = plan.chunk_images(c, rank)
            run.wait(hi)  # (its RGBA is complete in the arena: no device-wide sync, which would
            if do_gather:  # also wait for the decode kernels of the later chunks)
                post(c)
        statuses, stats = run.finish()
    else:
        statuses, stats = decode_fn(my_bufs, dsts)
    if sync:
        sync()
    decode_s = time.perf_counter() - t0
    result = ShardResult({i: s for i, s in zip(mine, statuses)}, decode_s, None, None, arena, stats, decode_s, 0.0)
    if not do_gather:
        if ws == 1:
            result.gathered = arena
        return result
    if start_fn is None:
        for c in range(plan.chunks):
            post(c)
    for w in works:
        w.wait()
    if sync:
        sync()
    t_end = time.perf_counter()
    result.gather_s = t_end - (t_first if t_first is not None else t_end)
    result.wall_s = t_end - t0
    result.tail_s = result.wall_s - decode_s
    # statuses travel as small ints (one per owned slot); error names are few,
    # and every rank agrees on their codes through a gather of names
    codes = {"Ok": 0}
    names = {0: "Ok"}
    per_rank = max(len(o) for o in plan.owned)
    st = torch.full((per_rank,), -1, dtype=torch.int32, device=device)
    for k, s in enumerate(statuses):
        st[k] = codes.setdefault(s, len(codes))
        names[codes[s]] = s
    name_list = [None] * ws if rank == 0 else None
    dist.gather_object(names, name_list, dst=0)
    gst = torch.empty(ws * per_rank, dtype=torch.int32, device=device) if rank == 0 else None
    dist.gather(st, gather_list=list(gst.view(ws, per_rank)) if rank == 0 else None, dst=0)
    if rank == 0:
        result.gathered = gathered
        table = gst.view(ws, per_rank).cpu().tolist()
        for r in range(ws):
            for k, i in enumerate(plan.owned[r]):
                result.statuses[i] = name_list[r][table[r][k]]
    return result


def host_cpu_budget() -> int:
    """CPUs this process may use: its affinity set, capped by a cgroup v2 CPU
    quota (a GPU box shares its host: nproc alone overstates it)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, math.ceil(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def rank_cpus(local_rank: int, local_ws: int) -> tuple[int, list[int]]:
    """This rank's share of the host: (entropy threads, CPUs to pin to).
    The budget splits evenly over the node's ranks, and each rank is pinned
    to its own contiguous block of the affinity set (threads the native pool
    creates inherit the calling thread's affinity)."""
    budget = host_cpu_budget()
    cpus = sorted(os.sched_getaffinity(0))
    threads = max(1, budget // max(1, local_ws))
    if len(cpus) >= local_ws > 1:
        per = len(cpus) // local_ws
        cpus = cpus[local_rank * per:(local_rank + 1) * per]
    return threads, cpus


def decode_sharded(buffers, ctxs, dst, host_threads: int = 0, depth: int = 0):
    """zpx_batch_decode_sharded: image i on ctxs[i % len(ctxs)], every result
    gathered into dst[i] (device tensors on ctxs[0]'s GPU).  Returns
    (statuses, zpx_batch_stats, zpx_gather_stats)."""
    from . import _lib

    n = len(buffers)
    items = (_lib.zpx_batch_item * max(1, n))()
    keep = [bytes(b) for b in buffers]
    for i, b in enumerate(keep):
        it = items[i]
        it.buf = C.cast(C.c_char_p(b), C.c_void_p)
        it.len = len(b)
        it.dst = dst[i].data_ptr()
        it.dst_capacity = dst[i].numel()
        it.dst_stride = 0
    handles = (C.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
    opts = _lib.zpx_batch_opts(host_threads, depth, 0)
    st = _lib.zpx_batch_stats()
    gs = _lib.zpx_gather_stats()
    _lib.check(_lib.lib().zpx_batch_decode_sharded(handles, len(ctxs), items, n, C.byref(opts), C.byref(st),
                                                   C.byref(gs)), ctxs[0].handle)
    return [_lib.error_name(items[i].status) for i in range(n)], st, gs
