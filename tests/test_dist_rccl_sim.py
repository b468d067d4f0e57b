"""The shipped RCCL gather branch of the multi-GPU layer, executed on CPU.

`vv_dsp_dist_gather_rows`'s point-to-point branch (vv-dsp_amd/csrc/host/dist.c:
one ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd group per slab) and the
one-process-per-GPU form (`vv_dsp_dist_unique_id` + `vv_dsp_dist_init_rank`)
need two GPUs, which the one-GPU pool never has.  Here the product's own dist.c
is linked unchanged with CPU stand-ins for the vvhip_* calls it makes
(tests/distsim/vvhip_cpu.c) and runs in 2-3 spawned processes over a host-memory
RCCL stand-in (tests/distsim/fake_rccl.c, soname librccl.so.1) whose receives
check every message's (peer, count, dtype, sequence) against the matching send.

Each rank computes its channel shard's spectrogram rows with the oracle (the
C restatement of /root/reference/src/spectral/stft.c:112-144; frames never span
channels) and the root checks the gathered [channels][frames][nfft] rows bit for
bit against the oracle's unsharded rows (half rows: against those rows made
mirror-symmetric, the rule the STFT kernel's rows obey and the pack / unpack
steps rely on, include/vv_dsp/vv_dsp_dist.h).  The fake's operation log is
compared with the schedule dist.c must produce: per slab one send from each peer
holding rows in it and one receive of the same count on the root.
"""
import ctypes as C
import multiprocessing as mp
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIM = os.path.join(ROOT, "tests", "distsim")
BUILD = os.path.join(SIM, "_build")
FAKE = os.path.join(BUILD, "fake", "librccl.so.1")
LIBS = {"default": os.path.join(BUILD, "libdistsim.so"),      # 256 MiB slabs (dist.c's own)
        "slab4k": os.path.join(BUILD, "libdistsim_slab.so")}  # 4 KiB slabs: many per rank
SLAB_BYTES = {"default": 256 << 20, "slab4k": 4096}
ORACLE = os.path.join(ROOT, "oracle", "liboracle.so")
NS, NFFT, HOP = 3000, 256, 64
FRAMES = 1 + (NS - NFFT + HOP) // HOP   # stft.c:119
vp, sz = C.c_void_p, C.c_size_t


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-s", "-C", SIM], check=True)
    assert os.path.exists(ORACLE), "oracle/liboracle.so missing: run `make -C oracle`"


def _bind(path):
    L = C.CDLL(path)
    L.vv_dsp_dist_unique_id.argtypes = [C.c_char_p]
    L.vv_dsp_dist_init_rank.argtypes = [C.c_int, C.c_int, C.c_char_p, C.c_int, C.POINTER(vp)]
    L.vv_dsp_dist_init_loopback.argtypes = [C.c_int, C.c_int, C.POINTER(vp)]
    L.vv_dsp_dist_destroy.argtypes = [vp]
    L.vv_dsp_dist_comm_count.argtypes = [vp, C.c_int, C.POINTER(C.c_int)]
    L.vv_dsp_dist_gather_rows.argtypes = [vp, C.POINTER(vp), sz, sz, sz, C.c_int, vp, C.c_int, C.POINTER(vp)]
    L.vv_dsp_shard_range.argtypes = [sz, sz, sz, C.POINTER(sz), C.POINTER(sz)]
    L.distsim_stream.restype = vp
    L.distsim_stream.argtypes = [C.c_int, C.c_int]
    L.distsim_waits.argtypes = [C.POINTER(C.c_int), C.c_int]
    L.distsim_live_allocs.restype = C.c_longlong
    L.vvhip_last_error.restype = C.c_char_p
    return L


def _shard(L, total, world, rank):
    f, c = sz(), sz()
    assert L.vv_dsp_shard_range(total, world, rank, C.byref(f), C.byref(c)) == 0
    return f.value, c.value


def _rows(total):
    """the oracle's unsharded rows [total][FRAMES][NFFT], one signal per channel"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from vvapi import Oracle
    orc = Oracle(ORACLE)
    rng = np.random.default_rng(17)
    x = rng.uniform(-1, 1, (total, NS)).astype(np.float32)
    return np.stack([orc.spectrogram(x[c], NFFT, HOP) for c in range(total)]).astype(np.float32)


def _mirror(rows):
    """rows[..., k] for k > NFFT/2 replaced by rows[..., NFFT - k]"""
    m = rows.copy()
    k = np.arange(NFFT // 2 + 1, NFFT)
    m[..., k] = rows[..., NFFT - k]
    return m


def _rank_main(lib_key, world, rank, total, root, half, id_q, res_q):
    try:
        C.CDLL(FAKE, mode=C.RTLD_GLOBAL)   # dist.c's dlopen("librccl.so.1") now resolves to the fake
        L = _bind(LIBS[lib_key])
        if rank == 0:
            uid = C.create_string_buffer(128)
            assert L.vv_dsp_dist_unique_id(uid) == 0, L.vvhip_last_error()
            for _ in range(world - 1):
                id_q.put(uid.raw)
            uid = uid.raw
        else:
            uid = id_q.get(timeout=30)
        d = vp()
        st = L.vv_dsp_dist_init_rank(world, rank, uid, rank, C.byref(d))
        assert st == 0, (st, L.vvhip_last_error())
        cnt_ = C.c_int()
        assert L.vv_dsp_dist_comm_count(d, 0, C.byref(cnt_)) == 0 and cnt_.value == world
        rows = _rows(total)
        src = _mirror(rows) if half else rows
        lo, cnt = _shard(L, total, world, rank)
        local = np.ascontiguousarray(src[lo:lo + cnt]) if cnt else None
        out = np.full((total, FRAMES, NFFT), np.nan, np.float32) if rank == root else None
        ptrs = (vp * 1)(local.ctypes.data if local is not None else None)
        streams = (vp * 1)(L.distsim_stream(rank, 0))
        st = L.vv_dsp_dist_gather_rows(d, ptrs, total, FRAMES, NFFT, half, out.ctypes.data if out is not None else None,
                                       root, streams)
        err = L.vvhip_last_error().decode()
        res = {"rank": rank, "status": st, "err": err, "live_allocs": L.distsim_live_allocs(),
               "dir": uid.split(b"\0", 1)[0].decode()}
        if rank == root and st == 0:
            res["equal"] = bool(np.array_equal(out, src))
            res["bad_rows"] = int(np.sum(~np.all(out == src, axis=-1)))
        assert L.vv_dsp_dist_destroy(d) == 0
        res_q.put(res)
    except BaseException as e:   # report instead of hanging the parent
        res_q.put({"rank": rank, "exception": repr(e)})


def _expected_ops(L, world, total, root, half, lib_key):
    """the per-slab schedule of dist.c: (kind, a, b, count, seq) lines of the fake's log"""
    w = NFFT // 2 + 1 if half else NFFT
    counts = [_shard(L, total, world, r)[1] * FRAMES for r in range(world)]
    cmax = max(counts)
    slab = max(1, min(SLAB_BYTES[lib_key] // (4 * w), cmax))
    ops, seq = [], {}
    for i0 in range(0, cmax, slab):
        for p in range(world):
            if p == root or i0 >= counts[p]:
                continue
            n = min(slab, counts[p] - i0) * w
            s = seq.get(p, 0)
            seq[p] = s + 1
            ops += [("send", p, root, n, s), ("recv", root, p, n, s)]
    return sorted(ops)


def _run(lib_key, world, total, root, half):
    ctx = mp.get_context("spawn")
    id_q, res_q = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(lib_key, world, r, total, root, half, id_q, res_q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in range(world):
            res.append(res_q.get(timeout=90))
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.terminate()
                p.join()
    res.sort(key=lambda r: r["rank"])
    for r in res:
        assert "exception" not in r, r
    d = res[0]["dir"]
    try:
        with open(os.path.join(d, "ops.log")) as f:
            log = [ln.split() for ln in f if ln.strip()]
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return res, log


CASES = [
    # (lib, world, channels, root, half)
    ("slab4k", 2, 5, 0, 0), ("slab4k", 2, 5, 1, 0), ("slab4k", 2, 5, 0, 1), ("slab4k", 2, 5, 1, 1),
    ("slab4k", 3, 5, 0, 0), ("slab4k", 3, 5, 1, 0), ("slab4k", 3, 5, 0, 1), ("slab4k", 3, 5, 1, 1),
    ("slab4k", 3, 2, 1, 1),    # fewer channels than ranks: rank 2 holds nothing
    ("default", 3, 4, 0, 1), ("default", 2, 3, 1, 0),
]


@pytest.mark.parametrize("lib_key,world,total,root,half", CASES)
def test_rccl_gather_branch_multiprocess(lib_key, world, total, root, half):
    res, log = _run(lib_key, world, total, root, half)
    for r in res:
        assert r["status"] == 0, r
        assert r["live_allocs"] == 0, r          # every pack / staging slab freed
    rr = res[root]
    assert rr["equal"], f"{rr['bad_rows']} rows differ from the oracle's unsharded rows"
    L = _bind(LIBS[lib_key])
    got = sorted((k, int(a), int(b), int(n), int(s)) for k, a, b, n, s in log if k != "init")
    want = _expected_ops(L, world, total, root, half, lib_key)
    assert got == want
    assert sorted(int(a) for k, a, *_ in log if k == "init") == list(range(world))
    if lib_key == "slab4k":   # the small slab really splits a rank's rows
        counts = [_shard(L, total, world, r)[1] * FRAMES for r in range(world)]
        w = NFFT // 2 + 1 if half else NFFT
        assert 4096 // (4 * w) < max(counts)
        assert len(want) > 2 * (world - 1)


def test_fake_rejects_unmatched_counts():
    """the fake is not permissive: a receive whose count differs from the send fails"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_mismatch_main, args=(r, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=60) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=10)
    assert res[0][1] != 0          # the receiver saw the mismatch
    shutil.rmtree(res[0][2], ignore_errors=True)


class _UniqueId(C.Structure):   # ncclUniqueId, passed by value
    _fields_ = [("internal", C.c_char * 128)]


def _mismatch_main(rank, q):
    F = C.CDLL(FAKE)
    F.ncclCommInitRank.argtypes = [C.POINTER(vp), C.c_int, _UniqueId, C.c_int]
    F.ncclSend.argtypes = [vp, sz, C.c_int, C.c_int, vp, vp]
    F.ncclRecv.argtypes = [vp, sz, C.c_int, C.c_int, vp, vp]
    path = b"/tmp/fake_rccl_mismatch_%d" % os.getppid()
    os.makedirs(path, exist_ok=True)
    uid = _UniqueId(path)
    c = vp()
    assert F.ncclCommInitRank(C.byref(c), 2, uid, rank) == 0
    buf = np.zeros(64, np.float32)
    ncclFloat32 = 7
    if rank == 1:
        r = F.ncclSend(buf.ctypes.data, 32, ncclFloat32, 0, c, None)
    else:
        r = F.ncclRecv(buf.ctypes.data, 16, ncclFloat32, 1, c, None)
    q.put((rank, r, path.decode()))


def test_half_rows_need_even_width():
    """half = 1 takes mirror-symmetric rows of an even fft_size only: an odd
    row_floats (e.g. 513-float power rows) is INVALID_SIZE, before any transfer"""
    L = _bind(LIBS["default"])
    d = vp()
    assert L.vv_dsp_dist_init_loopback(2, 0, C.byref(d)) == 0
    rows = np.zeros((2, 3, 513), np.float32)
    out = np.zeros_like(rows)
    ptrs = (vp * 2)(rows[0:1].ctypes.data, rows[1:2].ctypes.data)
    streams = (vp * 2)(None, None)
    assert L.vv_dsp_dist_gather_rows(d, ptrs, 2, 3, 513, 1, out.ctypes.data, 0, streams) == 2   # INVALID_SIZE
    assert b"even" in L.vvhip_last_error()
    assert L.vv_dsp_dist_gather_rows(d, ptrs, 2, 3, 513, 0, out.ctypes.data, 0, streams) == 0   # full rows fine
    assert np.array_equal(out, rows)
    assert L.vv_dsp_dist_destroy(d) == 0


@pytest.mark.parametrize("root", [0, 2])
def test_loopback_slot_streams_wait_for_root(root):
    """after a loopback gather every slot stream waits for the root's
    stream (which read d_local[s]), after the root waited for every slot stream"""
    L = _bind(LIBS["default"])
    L.distsim_reset()
    d = vp()
    assert L.vv_dsp_dist_init_loopback(3, 1, C.byref(d)) == 0
    rows = _mirror(np.random.default_rng(2).random((3, 4, NFFT), dtype=np.float32))
    out = np.zeros_like(rows)
    ptrs = (vp * 3)(*[rows[s:s + 1].ctypes.data for s in range(3)])
    streams = (vp * 3)(*[L.distsim_stream(1, s) for s in range(3)])
    for half in (0, 1):
        L.distsim_reset()
        out[:] = 0
        assert L.vv_dsp_dist_gather_rows(d, ptrs, 3, 4, NFFT, half, out.ctypes.data, root, streams) == 0
        assert np.array_equal(out, rows)
        buf = (C.c_int * 64)()
        n = L.distsim_waits(buf, 32)
        waits = [(buf[2 * i], buf[2 * i + 1]) for i in range(n)]
        rid = 16 + root
        others = [16 + s for s in range(3) if s != root]
        assert waits[:2] == [(rid, o) for o in others]    # root waits for the slots
        assert waits[2:] == [(o, rid) for o in others]    # then every slot waits for the root
        assert L.distsim_live_allocs() == 0
    assert L.vv_dsp_dist_destroy(d) == 0
