"""The dynamically scheduled STFT walks (k_stft_pair VAR 4 / VAR 5: persistent
grid, per-(device, stream) work counters that the kernel's last waves reset;
VAR 5 hands out runs of pairs walked on a ring of span chunks) against the
chunked launch they replace for large jobs (knob STFT_DYN=0):
bit-identical rows, repeated launches (the counters must come back to zero),
two streams at once (each its own counter block), the zero-padded tail and a
missing second frame (odd frame count), and sampled rows against NumPy f64 at
the harness tolerance (stft.c:112-144, python/test_fft.py:37-38)."""
import numpy as np
import pytest
import vvdsp_amd as vv

pytestmark = pytest.mark.gpu

NCH = 7
# 78,749 frames per channel (1 + (n - 1024 + 256) // 256): odd, zero-padded tail;
# n a multiple of 4, so the channels are 16 B aligned: the LDS-DMA kernels and
# their dynamic walks (with an odd stride every launch is the register-load VAR 1/2)
N = 7 * 60 * 48000 + 336


@pytest.fixture(scope="module")
def job(vdev):
    import torch
    g = torch.Generator(device="cuda").manual_seed(11)
    sig = torch.rand(NCH, N, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(1024, 256)
    vv.debug_set("STFT_DYN", 0)
    try:
        ref = st.spectrogram(sig).clone()
    finally:
        vv.debug_clear("STFT_DYN")
    torch.cuda.synchronize()
    return sig, st, ref


def test_dynamic_walk_equals_chunked(job):
    import torch
    sig, st, ref = job
    assert ref.shape == (NCH, 78749, 1024) and st.frames(N) == 78749
    out = torch.full_like(ref, -1.0)
    for _ in range(3):   # the counters are reset by each launch's last waves
        out.fill_(-1.0)
        d0 = vv.debug_get("STAT_STFT_DYN")
        st.spectrogram(sig, out=out)
        torch.cuda.synchronize()
        assert vv.debug_get("STAT_STFT_DYN") - d0 == 1   # the dynamic walk ran
        assert torch.equal(out, ref)


def test_dynamic_walk_two_streams(job):
    import torch
    sig, st, ref = job
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    o1, o2 = torch.full_like(ref, -1.0), torch.full_like(ref, -1.0)
    torch.cuda.synchronize()
    for _ in range(2):
        st.spectrogram(sig, out=o1, stream=s1)
        st.spectrogram(sig, out=o2, stream=s2)
    torch.cuda.synchronize()
    assert torch.equal(o1, ref)
    assert torch.equal(o2, ref)


def test_dynamic_walk_rows_vs_numpy(job, orc):
    sig, st, ref = job
    out = st.spectrogram(sig)
    w = orc.window(1, 1024).astype(np.float64)
    for c in (0, NCH - 1):
        x = sig[c].cpu().numpy().astype(np.float64)
        pad = np.concatenate([x, np.zeros(1024)])
        frames = [0, 1, 4097, 39374, 78744, 78747, 78748]   # the last ones run past the end
        X = np.abs(np.fft.fft(np.stack([pad[f * 256:f * 256 + 1024] for f in frames]) * w, axis=1))
        np.testing.assert_allclose(out[c][frames].cpu().numpy(), X, rtol=5e-5, atol=5e-5)


@pytest.mark.parametrize("kind", ["magnitude", "power", "complex"])
def test_dynamic_walk_other_rows(job, kind):
    """knob STFT_DYN=1 forces VAR 4 (one pair per counter value; magnitude rows
    default to VAR 5's runs) and runs power (n/2+1) and complex rows through the
    same walk: rows equal to the chunked launch's, bit for bit."""
    import torch
    sig, st, _ = job
    run = {"magnitude": lambda: st.spectrogram(sig), "power": lambda: st.power(sig),
           "complex": lambda: st.spectrogram(sig, complex_out=True)}[kind]
    vv.debug_set("STFT_DYN", 0)
    try:
        ref = run().clone()
    finally:
        vv.debug_clear("STFT_DYN")
    vv.debug_set("STFT_DYN", 1)
    try:
        for _ in range(2):
            got = run()
            torch.cuda.synchronize()
            assert torch.equal(got, ref)
    finally:
        vv.debug_clear("STFT_DYN")


@pytest.mark.parametrize("run_len", ["1", "3", "4", "16"])
@pytest.mark.parametrize("kind", ["magnitude", "power", "complex"])
def test_dynamic_ring_runs(job, kind, run_len):
    """knob STFT_DYN=2 (VAR 5): the dynamic walk handing out runs of
    knob STFT_RUN pairs, each walked on a ring of 256-float chunks -- runs that
    cross channel ends, a short last run, repeated launches: rows equal to the
    chunked launch's, bit for bit."""
    import torch
    sig, st, ref_mag = job
    run = {"magnitude": lambda: st.spectrogram(sig), "power": lambda: st.power(sig),
           "complex": lambda: st.spectrogram(sig, complex_out=True)}[kind]
    if kind == "magnitude":
        ref = ref_mag
    else:
        vv.debug_set("STFT_DYN", 0)
        try:
            ref = run().clone()
        finally:
            vv.debug_clear("STFT_DYN")
    vv.debug_set("STFT_DYN", 2)
    vv.debug_set("STFT_RUN", int(run_len))
    try:
        for _ in range(2):
            got = run()
            torch.cuda.synchronize()
            assert torch.equal(got, ref)
    finally:
        vv.debug_clear("STFT_DYN")
        vv.debug_clear("STFT_RUN")


@pytest.mark.parametrize("hop", [128, 512])
def test_dynamic_walks_other_hops(vdev, hop):
    """hop 512 (a 6-chunk ring refilled 4 chunks per pair) takes VAR 5, hop 128
    (not whole chunks) VAR 4: rows equal to the chunked launch's, bit for bit,
    for a multi-channel job past the dynamic-walk threshold."""
    import torch
    nch, n = 5, 4 * 60 * 48000 + 4097
    g = torch.Generator(device="cuda").manual_seed(hop)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(1024, hop)
    vv.debug_set("STFT_DYN", 0)
    try:
        ref = st.spectrogram(sig).clone()
    finally:
        vv.debug_clear("STFT_DYN")
    for _ in range(2):
        got = st.spectrogram(sig)
        torch.cuda.synchronize()
        assert torch.equal(got, ref)


def test_dynamic_walks_under_graph_capture(job, vdev, orc):
    """A large STFT and a config-4-sized FIR call captured on a fresh stream
    inside torch.cuda.graph: the capture takes counter blocks of
    its own, zeroed by a captured memset, so every replay starts from zero and
    never shares counters with eager launches on the stream.  Replays, with
    eager launches in between, give the eager rows bit for bit."""
    import torch
    sig, st, ref = job
    h = orc.fir_design_lowpass(257, 0.25, 2)
    plan = vdev.FirPlan(torch.from_numpy(h))
    x = torch.rand(6, 9_000_004, device="cuda") * 2 - 1   # aligned channels: the bulk kernel's dynamic walk
    with vv.knobs(FIR_R32=0):
        yref = plan(x).clone()
    out, y = torch.empty_like(ref), torch.empty_like(x)
    torch.cuda.synchronize()
    d0, f0 = vv.debug_get("STAT_STFT_DYN"), vv.debug_get("STAT_FIR_DYN")
    g = torch.cuda.CUDAGraph()
    with vv.knobs(FIR_R32=0):          # the 16 x 16 x 4 FIR kernel: the one with a dynamic walk
        with torch.cuda.graph(g):      # torch captures on a side stream of its own
            st.spectrogram(sig, out=out)
            plan(x, out=y)
    # the captured launches took the dynamic walks
    assert vv.debug_get("STAT_STFT_DYN") - d0 == 1 and vv.debug_get("STAT_FIR_DYN") - f0 == 1
    for _ in range(3):
        out.fill_(-1.0)
        y.fill_(-1.0)
        g.replay()
        eager = st.spectrogram(sig)      # eager work on the default stream between replays
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
        assert torch.equal(y, yref)
        assert torch.equal(eager, ref)
    del g


def test_capture_blocks_come_back(job):
    """every capture took a counter block for good, so after 256
    captures the dynamic walks silently fell back to the static ones.  A
    capture's block is now tied to its graph (hipGraphRetainUserObject) and
    returns to a free list when the graph is destroyed: 300 capture/destroy
    cycles later a capture still takes the dynamic walk, and its replay gives
    the eager rows."""
    import gc
    import torch
    sig, st, ref = job
    out = torch.empty_like(ref)
    torch.cuda.synchronize()
    for _ in range(300):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            st.spectrogram(sig, out=out)
        del g
        gc.collect()
        torch.cuda.synchronize()
    d0 = vv.debug_get("STAT_STFT_DYN")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        st.spectrogram(sig, out=out)
    assert vv.debug_get("STAT_STFT_DYN") - d0 == 1, "the capture fell back to the static walk"
    out.fill_(-1.0)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    del g


def test_many_streams_each_get_a_block(job):
    """more streams than one chunk of counter blocks (256): each still takes the
    dynamic walk with a block of its own (the pool grows by chunks)"""
    import torch
    sig, st, ref = job
    one = sig[:2]   # 78,750 pairs: enough for the dynamic walk
    ref1 = ref[:2]
    out = torch.empty_like(ref1)
    torch.cuda.synchronize()
    d0 = vv.debug_get("STAT_STFT_DYN")
    streams = [torch.cuda.Stream() for _ in range(300)]
    for s in streams:
        with torch.cuda.stream(s):
            st.spectrogram(one, out=out, stream=s)
        s.synchronize()
    assert vv.debug_get("STAT_STFT_DYN") - d0 == 300
    torch.cuda.synchronize()
    assert torch.equal(out, ref1)
