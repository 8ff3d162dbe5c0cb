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
  gathers.  The CPU `gloo` test drives these same two functions;
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
    no arena space)."""

    dims: list
    ws: int
    owned: list = field(init=False)        # owned[r]: image ids of rank r, in order
    offset: dict = field(init=False)       # image id -> byte offset in its rank's arena
    arena_bytes: list = field(init=False)  # bytes rank r's images occupy
    slot_bytes: int = field(init=False)    # the padded arena size every rank allocates

    def __post_init__(self):
        self.owned = [shard_images(len(self.dims), r, self.ws) for r in range(self.ws)]
        self.offset = {}
        self.arena_bytes = []
        for r in range(self.ws):
            off = 0
            for i in self.owned[r]:
                self.offset[i] = off
                off += _align(self.nbytes(i))
            self.arena_bytes.append(off)
        self.slot_bytes = max(ALIGN, max(self.arena_bytes) if self.arena_bytes else 0)

    def nbytes(self, i: int) -> int:
        d = self.dims[i]
        return 0 if d is None else d[0] * d[1] * 4

    def owner(self, i: int) -> int:
        return i % self.ws

    def gathered_offset(self, i: int) -> int:
        """Byte offset of image i in rank 0's gathered buffer (ws x slot_bytes)."""
        return self.owner(i) * self.slot_bytes + self.offset[i]

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
    gather_s: float | None     # gather wall time (None: no gather ran)
    gathered: object = None    # rank 0: uint8 tensor (ws * slot_bytes) holding every image
    arena: object = None       # this rank's arena
    stats: object = None       # whatever decode_fn returned besides the statuses

    def image(self, plan: ShardPlan, i: int):
        """Rank 0, after a gather: image i's RGBA (H, W, 4)."""
        return rgba_view(self.gathered, plan.gathered_offset(i), plan.dims[i])


def decode_and_gather(buffers, plan: ShardPlan, rank: int, dist, decode_fn, device, gather: bool = True,
                      sync=None) -> ShardResult:
    """Decode rank `rank`'s shard of `buffers` (the whole batch, indexed by
    global image id) into its arena, then gather every arena to rank 0.

    decode_fn(bufs, dsts) -> (statuses, stats): decodes bufs[k] into the
    (H, W, 4) tensor dsts[k] and returns one error name per image.
    sync(): waits for the device (torch.cuda.synchronize) before the clocks.
    """
    import torch

    ws = plan.ws
    mine = plan.owned[rank]
    arena = torch.empty(plan.slot_bytes, dtype=torch.uint8, device=device)
    dsts = [rgba_view(arena, plan.offset[i], plan.dims[i]) if plan.dims[i] is not None else None for i in mine]
    if sync:
        sync()
    if dist is not None and ws > 1:
        dist.barrier()
    t0 = time.perf_counter()
    statuses, stats = decode_fn([buffers[i] for i in mine], dsts)
    if sync:
        sync()
    decode_s = time.perf_counter() - t0
    codes = {"Ok": 0}
    names = {0: "Ok"}
    result = ShardResult({i: s for i, s in zip(mine, statuses)}, decode_s, None, None, arena, stats)
    if not gather or dist is None or ws == 1:
        if ws == 1:
            result.gathered = arena
        return result
    # statuses travel as small ints next to the pixels (one per owned slot)
    per_rank = max(len(o) for o in plan.owned)
    st = torch.full((per_rank,), -1, dtype=torch.int32, device=device)
    for k, s in enumerate(statuses):
        st[k] = codes.setdefault(s, len(codes))
        names[codes[s]] = s
    # error names are few; every rank agrees on their codes through a gather of names too
    name_list = [None] * ws if rank == 0 else None
    dist.gather_object(names, name_list, dst=0)
    gathered = torch.empty(ws * plan.slot_bytes, dtype=torch.uint8, device=device) if rank == 0 else None
    gst = torch.empty(ws * per_rank, dtype=torch.int32, device=device) if rank == 0 else None
    if sync:
        sync()
    dist.barrier()
    t0 = time.perf_counter()
    dist.gather(arena, gather_list=list(gathered.view(ws, plan.slot_bytes)) if rank == 0 else None, dst=0)
    if sync:
        sync()
    result.gather_s = time.perf_counter() - t0
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
