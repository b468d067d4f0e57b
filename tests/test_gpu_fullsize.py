"""GPU tests at BASELINE.json's full sizes, through size-independent properties
(round trips, Parseval, linearity, shard equivalence) plus oracle/NumPy checks
on sampled rows.  Sizes: config 2 (65536 x 1024 c2c), config 3 (60 s mono
STFT), config 4 (8 ch x 2^24 FIR), config 5 per-GPU shard shape (reduced
channel count)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_config2_c2c_65536x1024(vdev):
    import torch
    B, N = 65536, 1024
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.complex(torch.rand(B, N, device="cuda", generator=g) - 0.5,
                      torch.rand(B, N, device="cuda", generator=g) - 0.5)
    fwd = vdev.FftPlan(N, vdev.C2C, vdev.FWD, batch=B)
    bwd = vdev.FftPlan(N, vdev.C2C, vdev.BWD, batch=B)
    X = fwd(x)
    xr = bwd(X)
    torch.cuda.synchronize()
    # round trip (backward scales 1/N)
    assert (xr - x).abs().max().item() < 2e-6
    # Parseval: sum |X|^2 = N sum |x|^2 per row
    px = (x.abs() ** 2).sum(1).double()
    pX = (X.abs() ** 2).sum(1).double() / N
    assert ((pX - px).abs() / px).max().item() < 1e-5
    # sampled rows vs NumPy f64 at the harness tolerance
    rows = torch.arange(0, B, 1021, device="cuda")
    xs = x[rows].cpu().numpy().astype(np.complex128)
    np.testing.assert_allclose(X[rows].cpu().numpy(), np.fft.fft(xs, axis=1), rtol=5e-5, atol=5e-5)
    # linearity on a slice
    a, b = 0.75, -1.25
    y1 = fwd(x * a + torch.roll(x, 1, 0) * b)
    torch.testing.assert_close(y1, X * a + torch.roll(X, 1, 0) * b, rtol=1e-4, atol=2e-4)


def test_config3_stft_60s(vdev, orc):
    import torch
    n = 60 * 48000
    g = torch.Generator(device="cuda").manual_seed(3)
    sig = torch.rand(n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(1024, 256)
    mag = st.spectrogram(sig)
    assert mag.shape == (11248, 1024)   # stft.c:119 convention
    x = sig.cpu().numpy()
    frames = list(range(0, 11248, 373)) + [11246, 11247]   # last frames are zero-padded
    w = orc.window(1, 1024).astype(np.float64)
    pad = np.concatenate([x.astype(np.float64), np.zeros(1024)])
    ref = np.abs(np.fft.fft(np.stack([pad[f * 256:f * 256 + 1024] for f in frames]) * w, axis=1))
    np.testing.assert_allclose(mag[frames].cpu().numpy(), ref, rtol=5e-5, atol=5e-5)
    # the oracle (Kiss restatement) on a 1 s slice: same frames within 2x the bound
    sl = x[:48000]
    ko = orc.spectrogram(sl, 1024, 256)
    np.testing.assert_allclose(mag[:ko.shape[0] - 4].cpu().numpy(), ko[:-4], rtol=1e-4, atol=1e-4)


def test_config5_shard_shape(vdev):
    """Multi-channel STFT (channel shards): each channel equals its single-channel run."""
    import torch
    nch, n = 4, 10 * 48000
    sig = torch.empty(nch, n, device="cuda")
    for c in range(nch):
        g = torch.Generator(device="cuda").manual_seed(c)
        sig[c] = torch.rand(n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(1024, 256)
    out = st.spectrogram(sig)
    assert out.shape == (nch, 1 + (n - 1024 + 256) // 256, 1024)
    for c in (0, nch - 1):
        assert torch.equal(out[c], st.spectrogram(sig[c].contiguous()))


def test_config4_fir_8ch_2p24(vdev, orc):
    import torch
    nch, n = 8, 1 << 24
    h = orc.fir_design_lowpass(257, 0.25, 2)
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    plan = vdev.FirPlan(torch.from_numpy(h))
    y = plan(x)
    yd = plan(x, direct=True)
    torch.cuda.synchronize()
    err = (y - yd).abs().max().item()
    assert err < 1e-5, err
    # direct form is the reference's summation order: bit-exact on a slice
    xs = x[5, : 200000].cpu().numpy()
    assert np.array_equal(yd[5, : 200000].cpu().numpy(), orc.fir_apply(h, xs))
    # linearity across channels
    y2 = plan(x[:2] * 2.0 - x[2:4])
    torch.testing.assert_close(y2, y[:2] * 2.0 - y[2:4], rtol=1e-4, atol=1e-5)


def test_config5_real_shard_32ch_10min(vdev, orc):
    """Config 5's actual per-GPU shard at 8 GPUs -- 32 ch x 10 min @ 48 kHz
    (28,800,000 samples, 112,498 frames per channel; 3.7 GB in, 14.7 GB out),
    the bench's kernel and walk -- with sampled rows of EVERY channel (first,
    interior, and the zero-padded last frames) against NumPy f64 at the harness
    tolerance (stft.c:112-144, python/test_fft.py:37-38), and one whole channel's
    row sums against the single-channel call (bit-identical)."""
    import torch
    C, n = 32, 10 * 60 * 48000
    sig = torch.empty(C, n, device="cuda")
    for c in range(C):
        g = torch.Generator(device="cuda").manual_seed(c)
        sig[c].uniform_(-1.0, 1.0, generator=g)
    st = vdev.Stft(1024, 256)
    fr = st.frames(n)
    assert fr == 112498
    mag = st.spectrogram(sig)
    w = orc.window(1, 1024).astype(np.float64)
    for c in range(C):
        frames = [0, 1, 2 + 3517 * c, 56249, 91111 - c, fr - 3, fr - 2, fr - 1]
        idx = torch.tensor(frames, device="cuda")
        got = mag[c].index_select(0, idx).cpu().numpy()
        x = sig[c].cpu().numpy().astype(np.float64)
        pad = np.concatenate([x, np.zeros(1024)])
        ref = np.abs(np.fft.fft(np.stack([pad[f * 256:f * 256 + 1024] for f in frames]) * w, axis=1))
        np.testing.assert_allclose(got, ref, rtol=5e-5, atol=5e-5, err_msg=f"channel {c}")
    one = st.spectrogram(sig[17:18])
    assert torch.equal(one[0], mag[17])
    del mag, one, sig
    torch.cuda.empty_cache()
