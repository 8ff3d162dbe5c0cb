"""The N>1 path of bench.py on CPU: world_size-2 `gloo` ranks.

Images shard one-per-rank (image i -> rank i mod N) with no
data-path collective; each rank decodes its shard independently; the only
collectives are the max-over-ranks wall time and the optional gather of
results to rank 0.  Here each rank decodes a small sharded batch with the
oracle (CPU test infrastructure, the GPU path is covered by -m gpu) and rank 0
checks that the gathered per-image checksums equal an unsharded decode — a
checksum of checksums, independent of N.
"""
import ast
import os
import socket
import zlib

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import bench  # noqa: E402

N_IMAGES = 6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _decode_checksum(i: int) -> int:
    import oracle_py as O
    from tools import synthetic as S

    data = S.jpeg_420(i, 48 + 8 * i, 40) if i % 2 == 0 else S.png_tc8_mixed(i, 40 + 8 * i, 24)
    return zlib.crc32(O.decode(data).rgba_pixels().tobytes())


def _worker(rank, ws, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        mine = bench.shard_images(N_IMAGES, rank, ws)
        sums = torch.tensor([[i, _decode_checksum(i)] for i in mine], dtype=torch.int64)
        # ranks may own different counts: pad to the max shard size
        n = torch.tensor([len(mine)])
        dist.all_reduce(n, op=dist.ReduceOp.MAX)
        pad = torch.full((int(n.item()) - len(mine), 2), -1, dtype=torch.int64)
        sums = torch.cat([sums, pad])
        bufs = [torch.empty_like(sums) for _ in range(ws)] if rank == 0 else None
        dist.gather(sums, gather_list=bufs, dst=0)
        slowest = bench.max_over_ranks(dist, float(rank + 1), "cpu")
        if rank == 0:
            got = {int(i): int(c) for b in bufs for i, c in b.tolist() if i >= 0}
            with open(os.path.join(out_dir, "result.txt"), "w") as f:
                f.write(repr((got, slowest)))
    finally:
        dist.destroy_process_group()


def test_shard_images_partition():
    for ws in (1, 2, 4, 8):
        shards = [bench.shard_images(512, r, ws) for r in range(ws)]
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(512))
        assert all(len(s) == 512 // ws for s in shards)  # weak scaling: 64 per GPU at N=8


def test_max_over_ranks_single_process():
    assert bench.max_over_ranks(None, 1.5, "cpu") == 1.5


def test_gloo_world2_sharded_decode(tmp_path):
    ws = 2
    mp.spawn(_worker, args=(ws, _free_port(), str(tmp_path)), nprocs=ws, join=True)
    got, slowest = ast.literal_eval(open(tmp_path / "result.txt").read())
    assert slowest == float(ws)
    assert sorted(got) == list(range(N_IMAGES))
    for i in range(N_IMAGES):
        assert got[i] == _decode_checksum(i), i
