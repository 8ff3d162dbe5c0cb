"""GPU parity of the batch / streaming pipeline (zpx_batch_decode_rgba).

Every item must equal zpix.fromBuffer + Image.rgbaPixels of the same bytes
through the CPU oracle, bit-exact, whatever the mix of formats, the number of
host threads and staging slots, the destination (device or host memory) and
its row stride; a malformed item carries the reference's error name for it
and the rest of the batch is unaffected.
"""
import ctypes as C
import glob

import numpy as np
import pytest

import oracle_py as O
from conftest import golden, read
from tools import synthetic as S

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import zpix_amd  # noqa: E402
from zpix_amd import _lib, batch  # noqa: E402

FIXTURES = sorted(glob.glob(golden("testdata", "*.jpeg")) + glob.glob(golden("testdata", "*.jpg")) +
                  glob.glob(golden("testdata", "*.png")) + glob.glob(golden("pngsuite", "*.png")))


def oracle_rgba(data):
    """fromBuffer + rgbaPixels through the oracle (src/root.zig:34-40 probes PNG, then JPEG)."""
    if data[:8] != b"\x89PNG\r\n\x1a\n" and data[:2] != b"\xff\xd8":
        return None, "UnknownImageFormat"
    try:
        img = O.decode(data)
    except O.OracleError as e:
        return None, e.name
    return img.rgba_pixels().reshape(img.height, img.width, 4), "Ok"


def mixed_buffers():
    bufs = [open(p, "rb").read() for p in FIXTURES]
    bufs += [S.jpeg_420(7, 333, 211), S.png_tc8_mixed(8, 301, 97), S.jpeg_progressive_444(9, 130, 77),
             S.png_rgba16_adam7(10, 77, 45), S.png_generic(11, 190, 123, 8, 2, interlace=1),
             S.png_generic(12, 67, 90, 8, 6, interlace=1)]  # Adam7 through the staged passes (RGBA16, RGB8, RGBA8)
    bufs += [bufs[0][:len(bufs[0]) // 2], b"not an image at all", b""]  # malformed items
    return bufs


def check_results(bufs, res):
    assert len(res) == len(bufs)
    for data, r in zip(bufs, res):
        want, status = oracle_rgba(data)
        if status != "Ok":
            # the batch reports the image's own error (fromBuffer's, incl. UnknownImageFormat)
            assert r.status == status, (r.status, status)
            assert r.rgba is None
            continue
        assert r.status == "Ok", r.status
        got = r.rgba.cpu().numpy() if hasattr(r.rgba, "cpu") else r.rgba
        assert got.shape == want.shape
        assert np.array_equal(got, want)


@pytest.mark.parametrize("threads,depth", [(1, 1), (4, 3), (0, 0)])
def test_batch_device_dst(threads, depth):
    bufs = mixed_buffers()
    res = batch.decode_rgba(bufs, host_threads=threads, depth=depth)
    check_results(bufs, res)


@pytest.mark.parametrize("pair,makespan", [(0, 1), (1, 1), (1, 0)])
def test_batch_inflate_pair_switch(pair, makespan):
    """Workers inflating two PNGs in one loop ("inflate_pair", the default)
    or one at a time give the oracle's results, with a token budget of two
    (a pair takes both) and malformed PNGs among the pairs; with the pairs
    planned against the batch's remaining time ("batch_makespan", the
    default: PNGs of very different sizes, so late ones run alone) or formed
    whenever items are to spare."""
    L = _lib.lib()
    prev = L.zpx_debug_option(b"inflate_pair", pair)
    prev_m = L.zpx_debug_option(b"batch_makespan", makespan)
    try:
        bufs = mixed_buffers() + [S.png_tc8_mixed(20 + i, 257 + i, 129) for i in range(12)]
        bufs += [S.png_tc8_mixed(40, 64, 64)[:-30], S.png_generic(41, 99, 77, 16, 2)]
        bufs += [S.png_tc8_mixed(60 + i, 700 if i % 3 == 0 else 90, 300) for i in range(9)]
        res = batch.decode_rgba(bufs, host_threads=3, depth=3)
        check_results(bufs, res)
    finally:
        L.zpx_debug_option(b"inflate_pair", prev)
        L.zpx_debug_option(b"batch_makespan", prev_m)


def test_batch_host_dst():
    bufs = mixed_buffers()
    res, st = batch.decode_rgba(bufs, on_host=True, host_threads=3, with_stats=True)
    check_results(bufs, res)
    ok = [r for r in res if r.status == "Ok"]
    assert st.pixels == sum(r.width * r.height for r in ok)
    assert st.failed == len(bufs) - len(ok)
    assert st.d2h_bytes == st.pixels * 4


def test_batch_padded_stride_and_short_capacity():
    """dst_stride > 4W writes rows at the caller's pitch and leaves the pad
    alone; a destination that is too small fails only its own item."""
    data = [S.jpeg_420(3, 100, 37), S.png_tc8_mixed(4, 61, 29), read("pngsuite", "basn3p08.png")]
    c = zpix_amd.context.default()
    items = (_lib.zpx_batch_item * 4)()
    bufs = data + [data[0]]
    dsts, pitches = [], []
    for i, d in enumerate(bufs):
        want, _ = oracle_rgba(d)
        h, w = want.shape[:2]
        pitch = w * 4 + 52 if i < 3 else w * 4
        t = torch.full((h * pitch,), 0xAB, dtype=torch.uint8, device="cuda")
        dsts.append(t)
        pitches.append(pitch)
        items[i].buf = C.cast(C.c_char_p(d), C.c_void_p)
        items[i].len = len(d)
        items[i].dst = t.data_ptr()
        items[i].dst_stride = pitch
        items[i].dst_capacity = t.numel() if i < 3 else t.numel() - 1
    torch.cuda.synchronize()
    opts = _lib.zpx_batch_opts(2, 2, 0)
    _lib.check(_lib.lib().zpx_batch_decode_rgba(c.handle, items, 4, C.byref(opts), None), c.handle)
    for i in range(3):
        want, _ = oracle_rgba(bufs[i])
        h, w = want.shape[:2]
        got = dsts[i].cpu().numpy().reshape(h, pitches[i])
        assert items[i].status == 0
        assert np.array_equal(got[:, :w * 4].reshape(h, w, 4), want)
        assert (got[:, w * 4:] == 0xAB).all()
    assert _lib.error_name(items[3].status) == "InvalidArgument"


def test_batch_async_start_wait():
    bufs = [S.jpeg_420(i, 160 + 16 * i, 90) for i in range(5)] + [S.png_tc8_mixed(5, 200, 64)]
    c = zpix_amd.context.default()
    items = (_lib.zpx_batch_item * len(bufs))()
    outs = []
    for i, d in enumerate(bufs):
        want, _ = oracle_rgba(d)
        arr = np.zeros_like(want)
        outs.append((arr, want))
        items[i].buf = C.cast(C.c_char_p(d), C.c_void_p)
        items[i].len = len(d)
        items[i].dst = arr.ctypes.data
        items[i].dst_capacity = arr.nbytes
    opts = _lib.zpx_batch_opts(2, 0, 1)
    h = C.c_void_p()
    _lib.check(_lib.lib().zpx_batch_start(c.handle, items, len(bufs), C.byref(opts), C.byref(h)))
    st = _lib.zpx_batch_stats()
    _lib.check(_lib.lib().zpx_batch_wait(h, C.byref(st)), c.handle)
    assert st.failed == 0
    for i, (arr, want) in enumerate(outs):
        assert items[i].status == 0
        assert np.array_equal(arr, want)


def test_batch_empty():
    assert batch.decode_rgba([]) == []


def test_batch_4k_pair_matches_oracle():
    """One bench-size JPEG and PNG through the streaming path (device dst)."""
    bufs = [S.jpeg_420(0, 4096, 4096), S.png_tc8_mixed(0, 4096, 4096)]
    res = batch.decode_rgba(bufs, host_threads=2)
    check_results(bufs, res)


# ---------------------------------------------------------------- configs[3]: zpx_batch_decode_sharded
@pytest.mark.parametrize("ndev", [1, 2])
def test_batch_decode_sharded_matches_oracle(ndev):
    """Image i on context i mod ndev, every result gathered into its
    destination on context 0's device.  On a one-GPU box the second context
    shares device 0 (its shard decodes into staging on its own streams and
    travels by a device copy; between distinct GPUs the same code path sends
    over RCCL)."""
    from zpix_amd import shard

    bufs = mixed_buffers()[-10:]
    ctxs = [zpix_amd.context.default(0)] + [zpix_amd.Context(0) for _ in range(ndev - 1)]
    dims = [batch._probe_dims(b) or (1, 1) for b in bufs]
    dst = [torch.full((h, w, 4), 0x5a, dtype=torch.uint8, device="cuda:0") for w, h in dims]
    torch.cuda.synchronize()
    statuses, st, gs = shard.decode_sharded(bufs, ctxs, dst, host_threads=3)
    assert gs.ndev == ndev and gs.decode_s > 0
    ok = 0
    for i, data in enumerate(bufs):
        want, status = oracle_rgba(data)
        assert statuses[i] == status, (i, statuses[i], status)
        if status == "Ok":
            ok += 1
            assert np.array_equal(dst[i].cpu().numpy(), want), i
    assert st.pixels == sum(dims[i][0] * dims[i][1] for i in range(len(bufs)) if statuses[i] == "Ok")
    if ndev > 1:  # every successful image of the second shard travelled
        moved = sum(dims[i][0] * dims[i][1] * 4 for i in range(1, len(bufs), 2) if statuses[i] == "Ok")
        assert gs.gather_bytes == moved
    assert ok >= 6


@pytest.mark.parametrize("ndev", [2, 3])
def test_batch_decode_sharded_fake_comm_send_recv(ndev):
    """configs[3]'s communicator branch on the one-GPU box: with the in-process
    fake communicator (zpx_debug_shard_fake_comm: RCCL's grouped send/recv
    semantics, one rank per context) every context is its own rank, so every
    remote result travels by ncclSend/ncclRecv on the gather streams, posted
    as each image finishes.  Bit-exact against the oracle; the communicators
    are created once (comm_setup_s is 0 on the second call)."""
    from zpix_amd import shard

    bufs = mixed_buffers()[-9:]
    ctxs = [zpix_amd.context.default(0)] + [zpix_amd.Context(0) for _ in range(ndev - 1)]
    dims = [batch._probe_dims(b) or (1, 1) for b in bufs]
    prev = _lib.lib().zpx_debug_shard_fake_comm(1)
    try:
        for call in range(2):
            dst = [torch.full((h, w, 4), 0x5a, dtype=torch.uint8, device="cuda:0") for w, h in dims]
            torch.cuda.synchronize()
            statuses, st, gs = shard.decode_sharded(bufs, ctxs, dst, host_threads=2)
            assert gs.ndev == ndev and gs.comm_ranks == ndev
            if call == 1:
                assert gs.comm_setup_s == 0.0 or gs.comm_setup_s < 1e-3
            assert abs(st.wall_s - (gs.decode_s + gs.tail_s)) < 1e-6
            moved = 0
            for i, data in enumerate(bufs):
                want, status = oracle_rgba(data)
                assert statuses[i] == status, (i, statuses[i], status)
                if status == "Ok":
                    assert np.array_equal(dst[i].cpu().numpy(), want), (call, i)
                    if i % ndev:
                        moved += dims[i][0] * dims[i][1] * 4
            assert gs.gather_bytes == moved and moved > 0
            assert gs.gather_s > 0
    finally:
        _lib.lib().zpx_debug_shard_fake_comm(prev)


@pytest.mark.parametrize("ndev", [2, 3])
def test_batch_decode_sharded_real_rccl_self_send(ndev):
    """configs[3]'s gather through the real RCCL on the one-GPU box (test
    switch shard_rccl_self): every context shares device 0, so the
    communicator set is one rank (ncclCommInitAll over device 0, from the
    dlopen'd librccl.so.1) and each remote shard's results travel as grouped
    ncclSend / ncclRecv to rank 0 itself on the gather stream.  Bit-exact
    against the oracle on two calls, the second reusing the cached
    communicator; closing the contexts destroys it (zpx_ctx_destroy ->
    shard_release_comms), and a later call builds a new one."""
    from zpix_amd import shard

    bufs = mixed_buffers()[-9:]
    dims = [batch._probe_dims(b) or (1, 1) for b in bufs]
    prev = _lib.lib().zpx_debug_option(b"shard_rccl_self", 1)
    try:
        for life in range(2):
            ctxs = [zpix_amd.Context(0) for _ in range(ndev)]
            for call in range(2):
                dst = [torch.full((h, w, 4), 0x5a, dtype=torch.uint8, device="cuda:0") for w, h in dims]
                torch.cuda.synchronize()
                statuses, st, gs = shard.decode_sharded(bufs, ctxs, dst, host_threads=2)
                assert gs.ndev == ndev and gs.comm_ranks == 1
                if call == 1:
                    assert gs.comm_setup_s < 1e-3  # the cached communicator
                moved = 0
                for i, data in enumerate(bufs):
                    want, status = oracle_rgba(data)
                    assert statuses[i] == status, (life, call, i, statuses[i], status)
                    if status == "Ok":
                        assert np.array_equal(dst[i].cpu().numpy(), want), (life, call, i)
                        if i % ndev:
                            moved += dims[i][0] * dims[i][1] * 4
                assert gs.gather_bytes == moved and moved > 0
            for c in ctxs:
                c.close()
    finally:
        _lib.lib().zpx_debug_option(b"shard_rccl_self", prev)


def test_batch_decode_sharded_concurrent_calls_share_comms():
    """Two threads run sharded decodes at once, each on its own contexts but
    on the same device set, so both use the one cached communicator set: a
    call checks the set out for its whole gather (RCCL forbids one
    communicator on two threads at once), so the calls take turns and both
    results are exact."""
    import threading

    from zpix_amd import shard

    bufs = mixed_buffers()[-6:]
    dims = [batch._probe_dims(b) or (1, 1) for b in bufs]
    want = [oracle_rgba(d) for d in bufs]
    prev = _lib.lib().zpx_debug_shard_fake_comm(1)
    results = {}
    try:
        def run(t):
            ctxs = [zpix_amd.Context(0), zpix_amd.Context(0)]
            dst = [torch.full((h, w, 4), 0x5a, dtype=torch.uint8, device="cuda:0") for w, h in dims]
            statuses, _, gs = shard.decode_sharded(bufs, ctxs, dst, host_threads=2)
            torch.cuda.synchronize()
            results[t] = (statuses, [d.cpu().numpy() for d in dst], gs.gather_bytes)
            for c in ctxs:
                c.close()

        ths = [threading.Thread(target=run, args=(t,)) for t in range(2)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
    finally:
        _lib.lib().zpx_debug_shard_fake_comm(prev)
    assert sorted(results) == [0, 1]
    for t in range(2):
        statuses, got, moved = results[t]
        assert moved > 0
        for i, (w, status) in enumerate(want):
            assert statuses[i] == status, (t, i)
            if status == "Ok":
                assert np.array_equal(got[i], w), (t, i)


def test_batch_decode_sharded_rejects_host_dst():
    """Results gather into device memory: dst_on_host is an invalid argument."""
    ctxs = [zpix_amd.context.default(0)]
    items = (_lib.zpx_batch_item * 1)()
    handles = (C.c_void_p * 1)(ctxs[0].handle.value)
    opts = _lib.zpx_batch_opts(1, 0, 1)
    code = _lib.lib().zpx_batch_decode_sharded(handles, 1, items, 1, C.byref(opts), None, None)
    assert _lib.error_name(code) == "InvalidArgument"


def test_batch_start_wait_prefix():
    """zpx_batch_wait_prefix: the leading images are final (status and RGBA)
    before the batch ends; the chunked gather of configs[3] moves them then."""
    bufs = mixed_buffers()[-8:]
    run = batch.start_rgba(bufs, host_threads=2)
    k = run.wait(3)
    assert k >= 3
    early = run.statuses(0, 3)
    res, st = run.finish()
    assert run.wait(len(bufs)) == len(bufs)
    assert early == [r.status for r in res[:3]]
    check_results(bufs, res)


def test_batch_png_band_too_wide_rejected():
    """A pass whose 64-row band exceeds the kernel's 2 GiB band range is
    refused with Unsupported (never silently decoded with zero rows past
    2 GiB): checked on the plan, from the frame descriptor alone."""
    ctx = zpix_amd.context.default(0)
    f = _lib.zpx_png_frame()
    f.width, f.height, f.depth = 1 << 22, 64, 15  # RGBA16: 33.5 MB rows, a 2.1 GB band
    dummy = torch.empty(256, dtype=torch.uint8, device="cuda")
    f.filtered = dummy.data_ptr()
    f.out = dummy.data_ptr()
    f.out_stride = f.width * 8
    h = C.c_void_p()
    code = _lib.lib().zpx_png_plan_create(ctx.handle, C.byref(f), 1, C.byref(h))
    assert _lib.error_name(code) == "Unsupported"


def test_plan_status_ok_and_stall_times_out_once():
    """zpx_plan_status reports a good launch as Ok; a producer that never
    publishes makes the bounded boundary wait give up, the launch report
    Hip, and costs about one spin limit, not one per step."""
    from zpix_amd import device, png as P

    data = S.png_tc8_mixed(3, 301, 200)
    pb = device.PngBatch([P.Stream(data)])
    for _ in range(3):
        pb.launch()
    pb.status()  # Ok: no raise
    ctx = zpix_amd.context.default(0)
    secs = C.c_double()
    code = _lib.lib().zpx_debug_png_stall(ctx.handle, 4096, C.byref(secs))
    assert _lib.error_name(code) == "Hip"
    assert b"timed out" in _lib.lib().zpx_last_error(ctx.handle)
    assert secs.value < 2.0, secs.value
    # the stall did not poison later launches of other plans
    pb.launch()
    pb.status()


def test_batch_sparse_coefficient_upload():
    """Baseline 3-component JPEGs travel as sparse coefficient records
    (SURVEY §8(f)1), expanded on the device: bit-exact results and fewer H2D
    bytes than the dense int8 grids."""
    bufs = [S.jpeg_420(20 + i, 256 + 8 * i, 192) for i in range(4)] + [S.jpeg_subsampled(30, 200, 120, 0),
                                                                       S.jpeg_subsampled(31, 96, 64, 1)]
    res, st = batch.decode_rgba(bufs, host_threads=2, with_stats=True)
    check_results(bufs, res)
    dense = 0
    for data in bufs:
        c = O.jpeg_coefficients(data)
        dense += sum(np.asarray(g).size for g in c.grids if g is not None)  # int8 bytes
    assert 0 < st.h2d_bytes < 0.8 * dense, (st.h2d_bytes, dense)


def test_batch_dense_coefficient_upload():
    """The test switch "jpeg_sparse" = 0 keeps the dense-grid upload; same pixels."""
    prev = _lib.lib().zpx_debug_option(b"jpeg_sparse", 0)
    try:
        bufs = mixed_buffers()
        check_results(bufs, batch.decode_rgba(bufs, host_threads=3))
    finally:
        _lib.lib().zpx_debug_option(b"jpeg_sparse", prev)


def test_batch_slot_cache_reuse_and_trim():
    """A finished batch's slots are cached per device and reused by the next
    batch (zpx_batch_cache_trim frees them): the mixed batch decodes the same
    with the cache off, through slots cached by a batch of other formats and
    sizes (JPEG-only, then PNG-only, then the mix), and after a trim."""
    L = _lib.lib()
    bufs = mixed_buffers()
    prev = L.zpx_debug_option(b"batch_slot_cache", 0)
    try:
        L.zpx_batch_cache_trim()
        check_results(bufs, batch.decode_rgba(bufs, host_threads=3, depth=4))
        assert L.zpx_batch_cache_trim() == 0  # (nothing cached with the switch off)
        L.zpx_debug_option(b"batch_slot_cache", 1)
        jpegs = [b for b in bufs if b[:2] == b"\xff\xd8"]
        pngs = [b for b in bufs if b[:8] == b"\x89PNG\r\n\x1a\n"]
        check_results(jpegs, batch.decode_rgba(jpegs, host_threads=2, depth=3))
        check_results(pngs, batch.decode_rgba(pngs, host_threads=3, depth=5))  # 3 cached slots + 2 new
        check_results(bufs, batch.decode_rgba(bufs, host_threads=3, depth=6))
        check_results(bufs, batch.decode_rgba(bufs, host_threads=2, depth=2))
        assert L.zpx_batch_cache_trim() > 0
        assert L.zpx_batch_cache_trim() == 0
        check_results(bufs, batch.decode_rgba(bufs, host_threads=3, depth=4))
    finally:
        L.zpx_debug_option(b"batch_slot_cache", prev)
