"""The plain-C multi-GPU layer (include/vv_dsp/vv_dsp_dist.h, csrc/host/dist.c)
and the Python gathers (vvdsp_dist.py) on a world-1 nccl (= RCCL) process group.

What runs where:
* two or more visible GPUs (skipped on the one-GPU test box):
  `test_rccl_two_devices` -- ncclCommInitAll over devices 0 and 1, 7 uneven
  channels, roots 0 and 1, full and half rows, 256 MiB and 1500 KiB slabs:
  the grouped ncclSend / ncclRecv slabs (dist.c, "the transfers of this slab")
  against the single-call rows, bit for bit; and a stream on the wrong device
  refused;
* one GPU: RCCL communicators of ONE rank (ncclCommInitAll over device 0, and
  ncclGetUniqueId + ncclCommInitRank): the sharded STFT and the gather return
  before any ncclSend / ncclRecv (a world of one has no peer), so these cover the
  communicator set-up and the root's own rows only -- RCCL refuses two ranks
  on one device ("Duplicate GPU detected"), so no send / receive runs here;
* loopback contexts of 2 and 3 ranks on device 0 (the same slab / offset /
  pack-unpack logic with device copies in place of ncclSend/ncclRecv): uneven
  channel shards (vv_dsp_shard_range), roots 0 and world-1, small slabs;
* config 2 / config 4 shard helpers (batch shards of an FFT, channel shards of
  the FIR) against the unsharded calls, bit for bit.
Reference semantics: stft.c:112-144 (rows), SURVEY.md 8e (shards + gather)."""
import os
import socket

import numpy as np
import pytest
import vvdsp_amd as vv

pytestmark = pytest.mark.gpu

NCH, N = 7, 48000 * 20 + 333     # 7 channels: shards 4/3 (world 2), 3/2/2 (world 3)


@pytest.fixture(scope="module")
def job():
    import torch
    g = torch.Generator(device="cuda").manual_seed(5)
    sig = torch.rand(NCH, N, device="cuda", generator=g) * 2 - 1
    st = vv.Stft(1024, 256)
    ref = st.spectrogram(sig).clone()
    torch.cuda.synchronize()
    return sig, st, ref


def _shards(total, world):
    return [vv.shard_range(total, world, r) for r in range(world)]


def _sharded_rows(d, sig, st, world, kind=0):
    import torch
    fr = st.frames(N)
    width = 1024 if kind != 2 else 513
    dt = torch.complex64 if kind == 1 else torch.float32
    sl = _shards(NCH, world)
    rows = [torch.full((c, fr, width), -3.0, device="cuda").to(dt) for (_, c) in sl]
    sigs = [sig[f] for (f, _) in sl]
    assert d.stft(st, sigs, N, NCH, sig.stride(0), rows, out_kind=kind) == fr
    return rows


@pytest.mark.parametrize("how", ["init_all", "init_rank"])
def test_rccl_one_rank_stft_and_gather(job, how):
    import torch
    sig, st, ref = job
    d = vv.Dist.all([0]) if how == "init_all" else vv.Dist.rank(1, 0, vv.Dist.unique_id(), 0)
    assert d.slots == 1 and d.rank_info(0) == (0, 1, 0)
    assert d.comm_count(0) == 1
    rows = _sharded_rows(d, sig, st, 1)
    torch.cuda.synchronize()
    assert torch.equal(rows[0], ref)
    for half in (False, True):
        out = torch.full_like(ref, -1.0)
        d.gather_rows([rows[0]], NCH, ref.shape[1], 1024, out, root=0, half=half)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
    # the root's rows already in place inside the output: nothing moves
    out = ref.clone()
    d.gather_rows([out], NCH, ref.shape[1], 1024, out, root=0, half=True)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_unique_ids_differ():
    a, b = vv.Dist.unique_id(), vv.Dist.unique_id()
    assert len(a) == len(b) == 128 and a != b


def _two_gpus():
    import torch
    return torch.cuda.device_count() >= 2


@pytest.mark.skipif(not _two_gpus(), reason="needs two visible GPUs (RCCL refuses two ranks on one device)")
@pytest.mark.parametrize("root", [0, 1])
@pytest.mark.parametrize("half", [False, True])
@pytest.mark.parametrize("slab_kb", [0, 1500])
def test_rccl_two_devices(job, knob, root, half, slab_kb):
    """ncclCommInitAll over devices 0 and 1: rank 1's shard lives on device 1,
    the sends / receives cross xGMI, and the gathered rows on the root equal the
    unsharded single-call rows bit for bit (1500 KiB slabs end inside a channel)."""
    import torch
    sig, st, ref = job
    if slab_kb:
        knob("DIST_SLAB_KB", slab_kb)
    d = vv.Dist.all([0, 1])
    assert d.slots == 2 and d.comm_count(0) == 2 and d.comm_count(1) == 2
    assert [d.rank_info(s) for s in range(2)] == [(0, 2, 0), (1, 2, 1)]
    sl = _shards(NCH, 2)
    fr = st.frames(N)
    sigs = [sig[sl[0][0]:sl[0][0] + sl[0][1]], sig[sl[1][0]:sl[1][0] + sl[1][1]].to("cuda:1")]
    rows = [torch.full((c, fr, 1024), -3.0, device=f"cuda:{i}") for i, (_, c) in enumerate(sl)]
    assert d.stft(st, sigs, N, NCH, N, rows) == fr
    for i in range(2):
        torch.cuda.synchronize(i)
    for (f, c), r in zip(sl, rows):
        assert torch.equal(r.to("cuda:0"), ref[f:f + c])
    out = torch.full(ref.shape, -1.0, device=f"cuda:{root}")
    d.gather_rows(rows, NCH, fr, 1024, out, root=root, half=half)
    for i in range(2):
        torch.cuda.synchronize(i)
    assert torch.equal(out.to("cuda:0"), ref)


@pytest.mark.skipif(not _two_gpus(), reason="needs two visible GPUs")
def test_rccl_stream_on_wrong_device_refused(job):
    import torch
    sig, st, _ = job
    d = vv.Dist.all([0, 1])
    s0 = torch.cuda.Stream(device=0)
    with pytest.raises(vv.VvError, match="device"):
        d.stft(st, [sig, sig], N, NCH, N, [sig, sig], streams=[s0, s0])


def test_loopback_distinct_streams(job):
    """Each slot writes its rows on its own stream and the gather is enqueued
    right after, with no host synchronisation: the loopback copies run on the
    root's stream after a device-side wait for every slot's stream."""
    import torch
    sig, st, ref = job
    world = 3
    d = vv.Dist.loopback(world)
    streams = [torch.cuda.Stream() for _ in range(world)]
    sl = _shards(NCH, world)
    fr = st.frames(N)
    for half in (False, True):
        rows = [torch.full((c, fr, 1024), -3.0, device="cuda") for (_, c) in sl]
        torch.cuda.synchronize()
        out = torch.full_like(ref, -1.0)
        torch.cuda.synchronize()   # torch's side streams do not wait for the null stream's fills
        d.stft(st, [sig[f] for f, _ in sl], N, NCH, N, rows, streams=streams)
        d.gather_rows(rows, NCH, fr, 1024, out, root=1, half=half, streams=streams)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)


def test_loopback_slot_overwrite_after_gather(job):
    """right after the gather returns, each slot overwrites its rows
    on its OWN stream with no host synchronisation (the next step's rows); the
    gather's reads on the root's stream must come first -- each slot stream
    waits (device side) for the root's stream before the call returns."""
    import torch
    sig, st, ref = job
    world, root = 3, 1
    d = vv.Dist.loopback(world)
    streams = [torch.cuda.Stream() for _ in range(world)]
    sl = _shards(NCH, world)
    fr = st.frames(N)
    for half in (False, True):
        rows = [torch.full((c, fr, 1024), -3.0, device="cuda") for (_, c) in sl]
        out = torch.full_like(ref, -1.0)
        torch.cuda.synchronize()
        d.stft(st, [sig[f] for f, _ in sl], N, NCH, N, rows, streams=streams)
        d.gather_rows(rows, NCH, fr, 1024, out, root=root, half=half, streams=streams)
        for s in range(world):
            if s != root:
                with torch.cuda.stream(streams[s]):
                    rows[s].fill_(-7.0)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
        assert all(bool((rows[s] == -7.0).all()) for s in range(world) if s != root)


def test_half_rows_need_even_width(job):
    d = vv.Dist.loopback(2)
    sig, _, ref = job
    with pytest.raises(vv.VvError):
        d.gather_rows([ref, ref], 2, 1, 513, ref, root=0, half=True)


def test_half_rows_need_two_bins(job):
    d = vv.Dist.loopback(2)
    sig, _, ref = job
    with pytest.raises(vv.VvError):
        d.gather_rows([ref, ref], 2, 1, 1, ref, root=0, half=True)


@pytest.mark.parametrize("world,root,slab_kb", [(2, 0, 0), (3, 0, 0), (3, 2, 0), (3, 1, 1500), (2, 1, 4097)])
@pytest.mark.parametrize("half", [False, True])
def test_loopback_gather_uneven(job, knob, world, root, slab_kb, half):
    """slab_kb: slabs smaller than a channel (15 MB here), ending inside channels"""
    import torch
    sig, st, ref = job
    if slab_kb:
        knob("DIST_SLAB_KB", slab_kb)
    d = vv.Dist.loopback(world)
    assert d.slots == world
    rows = _sharded_rows(d, sig, st, world)
    torch.cuda.synchronize()
    for (f, c), r in zip(_shards(NCH, world), rows):
        assert torch.equal(r, ref[f:f + c])
    out = torch.full_like(ref, -1.0)
    d.gather_rows(rows, NCH, ref.shape[1], 1024, out, root=root, half=half)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_loopback_power_and_complex_rows(job):
    import torch
    sig, st, _ = job
    d = vv.Dist.loopback(3)
    for kind, full in ((2, st.power(sig)), (1, st.spectrogram(sig, complex_out=True))):
        rows = _sharded_rows(d, sig, st, 3, kind)
        torch.cuda.synchronize()
        for (f, c), r in zip(_shards(NCH, 3), rows):
            assert torch.equal(r, full[f:f + c])
        # power rows gather as plain rows (513 floats)
        if kind == 2:
            out = torch.full_like(full, -1.0)
            d.gather_rows(rows, NCH, full.shape[1], 513, out, root=1)
            torch.cuda.synchronize()
            assert torch.equal(out, full)


def test_loopback_fft_and_fir_shards():
    import torch
    total, n = 1001, 1024
    g = torch.Generator(device="cuda").manual_seed(8)
    x = torch.complex(torch.rand(total, n, device="cuda", generator=g) - 0.5,
                      torch.rand(total, n, device="cuda", generator=g) - 0.5)
    ref = vv.FftPlan(n, vv.C2C, vv.FWD, batch=total)(x)
    d = vv.Dist.loopback(3)
    sl = _shards(total, 3)
    y = torch.empty_like(x)
    d.fft(n, vv.C2C, vv.FWD, total, [x[f] for f, _ in sl], [y[f] for f, _ in sl])
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    # config 4's FIR over channel shards
    h = torch.from_numpy(np.hanning(257).astype(np.float32) / 128.0)
    xs = torch.rand(5, 3_000_001, device="cuda", generator=g) * 2 - 1
    plan = vv.FirPlan(h)
    yref = plan(xs)
    ys = torch.empty_like(xs)
    sl = _shards(5, 2)
    d2 = vv.Dist.loopback(2)
    d2.fir([plan, plan], xs.shape[1], 5, [xs[f] for f, _ in sl], xs.stride(0), [ys[f] for f, _ in sl], ys.stride(0))
    torch.cuda.synchronize()
    assert torch.equal(ys, yref)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_torch_nccl_world1_gathers(job):
    """vvdsp_dist.gather_rows_half / gather_rows_stream on a world-1 nccl
    process group (RCCL), i.e. the bench's with_gather path on hardware."""
    import torch
    import torch.distributed as dist
    import vvdsp_dist
    sig, st, ref = job
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        out = vvdsp_dist.gather_rows_half(ref, NCH, 1024, dst=0)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
        host = torch.empty(ref.shape, dtype=ref.dtype).pin_memory()
        vvdsp_dist.gather_rows_stream(ref, NCH, vvdsp_dist.host_sink(host), dst=0, slab_bytes=3 * ref[0].numel() * 4 // 2)
        torch.cuda.synchronize()
        assert torch.equal(host, ref.cpu())
        full = vvdsp_dist.gather_rows(ref, NCH, dst=0)
        assert torch.equal(full, ref)
    finally:
        dist.destroy_process_group()
