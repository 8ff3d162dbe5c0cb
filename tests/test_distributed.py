"""The N>1 path of bench.py on CPU: world_size-2 `gloo` ranks.

configs[3]: images shard one-per-rank (image i -> rank i mod N)
with no data-path collective; each rank decodes its shard into its RGBA arena,
then one gather moves every arena to rank 0.  These tests drive the SAME
functions bench.py's end-to-end line uses -- zpix_amd.shard.ShardPlan (the
placement every rank derives from the header sizes), decode_and_gather (the
shard decode + arena gather + status gather) and bench.max_over_ranks -- with
a CPU decode function in place of the GPU pipeline: here each rank decodes
its images with the oracle (test infrastructure: the device decode itself is
covered by -m gpu), and rank 0 checks every gathered image, byte for byte,
against an unsharded decode, plus the error status of a corrupt image.
"""
import ast
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import bench  # noqa: E402
from zpix_amd import shard  # noqa: E402

N_IMAGES = 7
CORRUPT = 5  # a truncated JPEG: its rank reports the reference's error name


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _image(i: int, ws: int) -> bytes:
    from tools import synthetic as S

    if bench.e2e_is_jpeg(i, ws):
        d = S.jpeg_420(i, 48 + 8 * i, 40)
        return d[: len(d) // 2] if i == CORRUPT else d
    return S.png_tc8_mixed(i, 40 + 8 * i, 24)


def _dims(data: bytes):
    import oracle_py as O

    try:
        im = O.decode(data)
        return (im.width, im.height)
    except O.OracleError:
        # header-only size, as the GPU path gets it (decodeConfig, host-only):
        # a truncated scan still has its SOF
        from zpix_amd.batch import _probe_dims

        return _probe_dims(data)


def _oracle_decode_fn(bufs, dsts):
    """decode_fn for decode_and_gather: the oracle into the (H, W, 4) views."""
    import oracle_py as O

    statuses = []
    for b, d in zip(bufs, dsts):
        try:
            px = O.decode(b).rgba_pixels()
        except O.OracleError as e:
            statuses.append(e.name)
            continue
        d.copy_(torch.from_numpy(px).view(d.shape))
        statuses.append("Ok")
    return statuses, None


def _oracle_one(b, d):
    """decode_one for shard.ThreadedDecode: the oracle into one (H, W, 4) view."""
    statuses, _ = _oracle_decode_fn([b], [d])
    return statuses[0]


def _worker(rank, ws, port, out_dir, chunks):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        bufs = [_image(i, ws) for i in range(N_IMAGES)]
        plan = shard.ShardPlan([_dims(b) for b in bufs], ws, chunks=chunks)
        if chunks == 1:  # the whole shard, then one gather
            r = shard.decode_and_gather(bufs, plan, rank, dist, _oracle_decode_fn, "cpu", gather=True)
        else:  # chunk c gathered while the later chunks still decode
            r = shard.decode_and_gather(bufs, plan, rank, dist, device="cpu", gather=True,
                                        start_fn=lambda b, d: shard.ThreadedDecode(_oracle_one, b, d))
        slowest = bench.max_over_ranks(dist, float(rank + 1), "cpu")
        if rank == 0:
            got = {i: (r.statuses[i], r.image(plan, i).reshape(-1).numpy().tobytes().hex()
                       if r.statuses[i] == "Ok" else None) for i in range(N_IMAGES)}
            timing_ok = r.gather_s is not None and r.wall_s >= r.decode_s and abs(r.tail_s - (r.wall_s - r.decode_s)) < 1e-9
            with open(os.path.join(out_dir, "result.txt"), "w") as f:
                f.write(repr((got, slowest, timing_ok, plan.slot_bytes, plan.chunks)))
    finally:
        dist.destroy_process_group()


def test_shard_images_partition():
    for ws in (1, 2, 4, 8):
        shards = [bench.shard_images(512, r, ws) for r in range(ws)]
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(512))
        assert all(len(s) == 512 // ws for s in shards)  # weak scaling: 64 per GPU at N=8


def test_e2e_mix_is_half_and_half_on_every_rank():
    for ws in (1, 2, 4, 8):
        for r in range(ws):
            mine = bench.shard_images(64 * ws, r, ws)
            kinds = [bench.e2e_is_jpeg(i, ws) for i in mine]
            assert sum(kinds) == len(mine) // 2, (ws, r)


def test_shard_plan_placement():
    dims = [(16, 8), None, (4, 4), (100, 3), (7, 9)]
    p = shard.ShardPlan(dims, 2)
    assert p.owned == [[0, 2, 4], [1, 3]]
    # arena offsets are 256-aligned, non-overlapping, and fit the padded slot
    for r in range(2):
        spans = sorted((p.offset[i], p.offset[i] + p.nbytes(i)) for i in p.owned[r])
        assert all(a % 256 == 0 for a, _ in spans)
        assert all(spans[k][1] <= spans[k + 1][0] for k in range(len(spans) - 1))
        assert spans[-1][1] <= p.slot_bytes
    assert p.slot_bytes == max(p.arena_bytes)
    assert p.gathered_offset(3) == p.slot_bytes + p.offset[3]
    assert p.gather_bytes == p.slot_bytes


def test_rank_cpus_split():
    threads, cpus = shard.rank_cpus(0, 1)
    assert threads == shard.host_cpu_budget() and set(cpus) == set(os.sched_getaffinity(0))
    n = len(os.sched_getaffinity(0))
    if n >= 2:
        t0, c0 = shard.rank_cpus(0, 2)
        t1, c1 = shard.rank_cpus(1, 2)
        assert not set(c0) & set(c1) and len(c0) == len(c1) == n // 2
        assert t0 == t1 == max(1, shard.host_cpu_budget() // 2)


def test_max_over_ranks_single_process():
    assert bench.max_over_ranks(None, 1.5, "cpu") == 1.5


def test_shard_plan_chunks():
    """Chunked placement: each chunk is one fixed-size gather (chunk c of every
    rank padded to the largest), images never overlap in an arena or in rank
    0's gathered buffer, and a chunk's images are consecutive in their shard."""
    dims = [(16, 8), None, (4, 4), (100, 3), (7, 9), (3, 3), (5, 5), (64, 64), (1, 1)]
    for chunks in (1, 2, 3, 5, 50):
        p = shard.ShardPlan(dims, 3, chunks=chunks)
        assert p.chunks == min(chunks, 3)
        assert sum(p.chunk_bytes) == p.slot_bytes or p.slot_bytes == 256
        spans = []
        for r in range(3):
            for k, i in enumerate(p.owned[r]):
                c = p.chunk_of(i)
                lo, hi = p.chunk_images(c, r)
                assert lo <= k < hi
                assert p.chunk_base[c] <= p.offset[i] and p.offset[i] + p.nbytes(i) <= p.chunk_base[c] + p.chunk_bytes[c]
                if p.nbytes(i):
                    g = p.gathered_offset(i)
                    spans.append((g, g + p.nbytes(i)))
        spans.sort()
        assert all(spans[k][1] <= spans[k + 1][0] for k in range(len(spans) - 1))
        assert spans[-1][1] <= 3 * p.slot_bytes


@pytest.mark.parametrize("chunks", [1, 3])
def test_gloo_world2_sharded_decode_and_gather(tmp_path, chunks):
    import oracle_py as O

    ws = 2
    mp.spawn(_worker, args=(ws, _free_port(), str(tmp_path), chunks), nprocs=ws, join=True)
    got, slowest, timing_ok, slot, nchunks = ast.literal_eval(open(tmp_path / "result.txt").read())
    assert slowest == float(ws) and timing_ok and slot % 256 == 0 and nchunks == chunks
    assert sorted(got) == list(range(N_IMAGES))
    for i in range(N_IMAGES):
        data = _image(i, ws)
        if i == CORRUPT:
            with pytest.raises(O.OracleError) as e:
                O.decode(data)
            assert got[i] == (e.value.name, None)
            continue
        want = O.decode(data).rgba_pixels()
        assert got[i][0] == "Ok", i
        assert np.array_equal(np.frombuffer(bytes.fromhex(got[i][1]), np.uint8), want), i
