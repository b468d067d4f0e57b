"""k_stft_r32 (stft_kernels.hip): power rows of nfft 1024 / hop 256 with the
transform split 32 x 32 on half-waves (knob POW_R32 = 1; the default is the
16 x 16 x 4 ring kernel), against NumPy f64 per
bin at the power-row tolerance of test_gpu_parity.test_stft_power_rows, against
the default kernel, and with the path counter proving the kernel ran.  Shapes:
odd channel counts (a frame-pair couple spanning two channels, a missing last
pair), odd frame counts (a pair without its second frame), zero-padded tail
frames (spans staged through LDS), signals shorter than one span, and rows
that are not 16 B aligned (the path takes 8 B aligned channels: even channel
strides, or one channel)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ref_power(x, nfft, hop, fr, w):
    pad = np.concatenate([x.astype(np.float64), np.zeros(nfft + hop)])
    return np.abs(np.fft.rfft(np.stack([pad[f * hop:f * hop + nfft] for f in range(fr)]) * w, axis=1)) ** 2


@pytest.mark.parametrize("nch,n,off", [(3, 48000 + 334, 0), (1, 1280, 0), (1, 701, 1), (1, 48000 + 333, 0),
                                        (5, 1024 + 3 * 256, 0), (4, 20000, 3), (7, 48128, 2), (2, 1024, 0),
                                        (3, 1280 + 2, 0)])
def test_pow_r32_vs_f64(vdev, orc, knob, nch, n, off):
    import torch
    import vvdsp_amd as vv
    nfft, hop = 1024, 256
    g = torch.Generator(device="cuda").manual_seed(n + 17 * nch)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1   # channel stride n: even, or one channel
    st = vdev.Stft(nfft, hop)
    fr, nh = st.frames(n), nfft // 2 + 1
    buf = torch.full((off + nch * fr * nh + 64,), -7.0, device="cuda")
    out = buf[off:off + nch * fr * nh].view(nch, fr, nh)
    knob("POW_R32", 1)
    vv.debug_clear("STAT_POW_R32")
    st.power(sig, out=out)
    torch.cuda.synchronize()
    assert vv.debug_get("STAT_POW_R32") == 1, "k_stft_r32 did not run"
    knob("POW_R32", 0)   # the 16 x 16 x 4 ring kernel (the default)
    ref16 = st.power(sig).cpu().numpy()
    b = buf.cpu().numpy()
    assert np.all(b[:off] == -7.0) and np.all(b[off + nch * fr * nh:] == -7.0), "stores outside the rows"
    pw = out.cpu().numpy()
    assert np.all(np.isfinite(pw))
    w = orc.window(1, nfft).astype(np.float64)
    x = sig.cpu().numpy()
    for c in range(nch):
        ref = _ref_power(x[c], nfft, hop, fr, w)
        scale = np.max(ref, axis=1, keepdims=True)
        assert np.all(np.abs(pw[c] - ref) <= 1e-4 * np.abs(ref) + 1e-4 * scale), (c, np.max(np.abs(pw[c] - ref)))
        # and as close to the default (16 x 16 x 4) kernel as either is to f64
        assert np.all(np.abs(pw[c] - ref16[c]) <= 2e-4 * np.abs(ref) + 2e-4 * scale)


def test_pow_r32_large_sampled_and_repeatable(vdev, orc, knob):
    """32 ch x 60 s: every channel's first, middle and last rows against f64;
    two launches bit-identical (a static walk, no counters)."""
    import torch
    nfft, hop, nch, n = 1024, 256, 32, 60 * 48000
    g = torch.Generator(device="cuda").manual_seed(5)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(nfft, hop)
    fr = st.frames(n)
    knob("POW_R32", 1)
    a = st.power(sig)
    b = st.power(sig)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    w = orc.window(1, nfft).astype(np.float64)
    x = sig.cpu().numpy()
    pw = a.cpu().numpy()
    for c in range(nch):
        for f in (0, 1, fr // 2, fr // 2 + 1, fr - 2, fr - 1):
            seg = np.concatenate([x[c].astype(np.float64), np.zeros(nfft)])[f * hop:f * hop + nfft]
            ref = np.abs(np.fft.rfft(seg * w)) ** 2
            assert np.all(np.abs(pw[c, f] - ref) <= 1e-4 * np.abs(ref) + 1e-4 * ref.max()), (c, f)


@pytest.mark.parametrize("nch,n", [(3, 48000 + 334), (1, 1280), (1, 48000 + 333), (5, 1024 + 3 * 256),
                                   (7, 48128), (2, 1024), (3, 1280 + 2)])
def test_mag_r32_vs_f64(vdev, orc, knob, nch, n):
    """The magnitude rows of the same split (knob MAG_R32 = 1): all 1024 bins,
    the upper half stored from the mirrored registers, against NumPy f64 at the
    harness tolerance (rtol = atol = 5e-5, python/test_fft.py:37-38)."""
    import torch
    import vvdsp_amd as vv
    nfft, hop = 1024, 256
    g = torch.Generator(device="cuda").manual_seed(n + 29 * nch)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(nfft, hop)
    fr = st.frames(n)
    knob("MAG_R32", 1)
    vv.debug_clear("STAT_MAG_R32")
    mag = st.spectrogram(sig)
    torch.cuda.synchronize()
    assert vv.debug_get("STAT_MAG_R32") == 1, "k_stft_r32<0> did not run"
    mag = mag.cpu().numpy()
    w = orc.window(1, nfft).astype(np.float64)
    x = sig.cpu().numpy()
    for c in range(nch):
        pad = np.concatenate([x[c].astype(np.float64), np.zeros(nfft + hop)])
        X = np.fft.fft(np.stack([pad[f * hop:f * hop + nfft] for f in range(fr)]) * w, axis=1)
        np.testing.assert_allclose(mag[c], np.abs(X), rtol=5e-5, atol=5e-5)
