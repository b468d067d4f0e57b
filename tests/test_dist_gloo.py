"""Multi-rank channel sharding + gather of the batched STFT (SURVEY.md §8e,
config 5) on CPU with the gloo backend, world_size 2 and 3.

Each rank computes its channel shard's spectrogram with the oracle (the CPU
restatement; these tests exercise the layout and the collective, not the GPU
kernels) and `vvdsp_dist.gather_rows` assembles them on rank 0, which checks
the result against the unsharded oracle computation bit for bit.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vv-dsp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import vvdsp_dist  # noqa: E402

NS, NFFT, HOP = 6000, 256, 64


def _signals(nch):
    rng = np.random.default_rng(11)
    return rng.uniform(-1, 1, (nch, NS)).astype(np.float32)


def _worker(rank, world, nch, port, q, slab=None):
    if slab is not None:   # gather in slabs of `slab` bytes (one channel's rows per collective)
        vvdsp_dist.GATHER_SLAB_BYTES = slab
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vvapi import Oracle
        orc = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
        x = _signals(nch)
        lo, hi = vvdsp_dist.channel_shard(nch, world, rank)
        rows = [orc.spectrogram(x[c], NFFT, HOP) for c in range(lo, hi)]
        local = torch.from_numpy(np.stack(rows)) if rows else \
            torch.zeros((0,) + orc.spectrogram(x[0], NFFT, HOP).shape)
        full = vvdsp_dist.gather_rows(local, nch, dst=0)
        if rank == 0:
            ref = np.stack([orc.spectrogram(x[c], NFFT, HOP) for c in range(nch)])
            q.put(bool(np.array_equal(full.numpy(), ref)) and tuple(full.shape) == ref.shape)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _half_worker(rank, world, nch, port, q):
    """gather_rows_half: ranks send bins 0..NFFT/2 of their rows; rank 0
    expands by mirror symmetry.  pack / unpack here are torch slices on CPU
    tensors (the layout under test); on the GPU they are the library kernels
    (tests/test_gpu_shard.py pins those)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vvapi import Oracle
        orc = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
        x = _signals(nch)
        lo, hi = vvdsp_dist.channel_shard(nch, world, rank)
        local = torch.from_numpy(np.stack([orc.spectrogram(x[c], NFFT, HOP) for c in range(lo, hi)]))
        h = NFFT // 2 + 1
        mirror = torch.tensor([k if k < h else NFFT - k for k in range(NFFT)])

        def unpack(t, o):
            o.copy_(t[..., mirror])

        full = vvdsp_dist.gather_rows_half(local, nch, NFFT, dst=0, pack=lambda t: t[..., :h].contiguous(),
                                           unpack=unpack)
        if rank == 0:
            ref = np.stack([orc.spectrogram(x[c], NFFT, HOP) for c in range(nch)])
            ref = ref[..., mirror.numpy()]
            q.put(bool(np.array_equal(full.numpy(), ref)) and tuple(full.shape) == ref.shape)
        else:
            q.put(full is None)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _frame_worker(rank, world, port, q):
    """One long signal split by frame ranges (config 3 sharded): each rank
    transforms its input slice (frame0's first sample on, as
    vv_dsp_stft_frames_range_device does), rank 0 gathers the rows."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vvapi import Oracle
        orc = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
        x = _signals(1)[0]
        frames = 1 + (NS - NFFT + HOP) // HOP
        lo, hi = vvdsp_dist.frame_shard(frames, world, rank)
        if hi > lo:
            local = torch.from_numpy(np.ascontiguousarray(orc.spectrogram(x[lo * HOP:], NFFT, HOP)[:hi - lo]))
        else:
            local = torch.zeros((0, NFFT))
        full = vvdsp_dist.gather_frames(local, frames, dst=0)
        if rank == 0:
            ref = orc.spectrogram(x, NFFT, HOP)
            q.put(bool(np.array_equal(full.numpy(), ref)) and tuple(full.shape) == ref.shape)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _stream_worker(rank, world, nch, port, q, slab):
    """gather_rows_stream: rank 0 never allocates the [nch, ...] result on the
    device; slabs of `slab` bytes per rank go through one staging buffer into a
    host tensor (host_sink), uneven shards included."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vvapi import Oracle
        orc = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
        x = _signals(nch)
        lo, hi = vvdsp_dist.channel_shard(nch, world, rank)
        shape = orc.spectrogram(x[0], NFFT, HOP).shape
        local = torch.from_numpy(np.stack([orc.spectrogram(x[c], NFFT, HOP) for c in range(lo, hi)])) \
            if hi > lo else torch.zeros((0,) + shape)
        out = torch.full((nch,) + shape, -1.0) if rank == 0 else None
        seen = []

        def sink(first, block):
            seen.append((first, block.shape[0]))
            vvdsp_dist.host_sink(out)(first, block)

        vvdsp_dist.gather_rows_stream(local, nch, sink if rank == 0 else None, dst=0, slab_bytes=slab)
        if rank == 0:
            ref = np.stack([orc.spectrogram(x[c], NFFT, HOP) for c in range(nch)])
            rows = sorted(f + i for f, k in seen for i in range(k))
            q.put(bool(np.array_equal(out.numpy(), ref)) and rows == list(range(nch)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,nch,slab", [(2, 5, None), (3, 5, None), (2, 6, None), (3, 6, None), (2, 6, 1),
                                            (3, 9, 100000)])
def test_sharded_spectrogram_gather_gloo(world, nch, slab):
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        pytest.skip("oracle not built (make -C oracle)")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, nch, port, q, slab)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


@pytest.mark.parametrize("world", [2, 3])
def test_frame_sharded_spectrogram_gather_gloo(world):
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        pytest.skip("oracle not built (make -C oracle)")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_frame_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


@pytest.mark.parametrize("world,nch", [(2, 4), (3, 6)])
def test_half_bin_gather_gloo(world, nch):
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        pytest.skip("oracle not built (make -C oracle)")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_half_worker, args=(r, world, nch, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert all(q.get(timeout=5) is True for _ in range(world))


@pytest.mark.parametrize("world,nch,slab", [(2, 5, 1), (3, 7, 100000), (2, 6, 1 << 30)])
def test_streaming_gather_gloo(world, nch, slab):
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        pytest.skip("oracle not built (make -C oracle)")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stream_worker, args=(r, world, nch, port, q, slab)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_shard_range_c_matches_python():
    """vv_dsp_shard_range (vv_dsp_amd.h, pure host arithmetic) is the same split
    as vvdsp_dist.channel_shard."""
    import ctypes as C
    L = C.CDLL(os.path.join(ROOT, "vv-dsp_amd", "lib", "libvvdsp_amd.so"))
    L.vv_dsp_shard_range.argtypes = [C.c_size_t] * 3 + [C.POINTER(C.c_size_t)] * 2
    for total in (0, 1, 7, 256, 1001):
        for world in (1, 2, 3, 8):
            for r in range(world):
                a, b = C.c_size_t(), C.c_size_t()
                assert L.vv_dsp_shard_range(total, world, r, C.byref(a), C.byref(b)) == 0
                assert (a.value, a.value + b.value) == vvdsp_dist.channel_shard(total, world, r)
    a, b = C.c_size_t(), C.c_size_t()
    assert L.vv_dsp_shard_range(4, 2, 2, C.byref(a), C.byref(b)) == 3        # OUT_OF_RANGE
    assert L.vv_dsp_shard_range(4, 0, 0, C.byref(a), C.byref(b)) == 3
    assert L.vv_dsp_shard_range(4, 2, 0, None, C.byref(b)) == 1              # NULL_POINTER


def test_frame_shard_layout():
    for frames in (0, 1, 2, 5, 11247, 11248):
        for world in (1, 2, 3, 8):
            spans = [vvdsp_dist.frame_shard(frames, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == frames
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert all(lo % 2 == 0 for lo, hi in spans if hi > lo)   # whole frame pairs per rank
    assert vvdsp_dist.frame_shard_sizes(11248, 8) == [1406] * 8


def test_channel_shard_layout():
    for total in (0, 1, 7, 256):
        for world in (1, 2, 3, 8):
            spans = [vvdsp_dist.channel_shard(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    assert vvdsp_dist.channel_shard(256, 8, 3) == (96, 128)   # config 5: 32 ch per GPU
    with pytest.raises(ValueError):
        vvdsp_dist.channel_shard(4, 2, 2)
