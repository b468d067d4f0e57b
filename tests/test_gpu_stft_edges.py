"""STFT framing edge cases (stft.c:112-144): frames = 1 when n < nfft (the
whole frame zero-padded, n = 0 included), 1 + (n - nfft + hop) / hop
otherwise, the last frame zero-padded past n.  Host entry against the oracle
at the harness tolerance (python/test_fft.py:37-38), and the device entry
writing every element of a sentinel-filled output."""
import numpy as np
import pytest
import vvdsp_amd as vv

pytestmark = pytest.mark.gpu


def _np_frames(x, nfft, hop, w):
    """|FFT| of the reference's framing (stft.c:119-139) in f64"""
    n = len(x)
    frames = 1 if n < nfft else 1 + (n - nfft + hop) // hop
    pad = np.concatenate([x.astype(np.float64), np.zeros(frames * hop + nfft)])
    return np.abs(np.fft.fft(np.stack([pad[f * hop:f * hop + nfft] for f in range(frames)]) * w, axis=1))


@pytest.mark.parametrize("nfft,hop", [(1024, 256), (400, 160), (512, 512), (480, 120), (256, 64), (4096, 1024)])
def test_stft_short_and_ragged_signals(amd, orc, nfft, hop):
    """against NumPy f64 at the harness tolerance (the primary parity rule,
    SURVEY 8c note 5); for pow2 nfft <= 1024 also against the oracle (Kiss)"""
    rng = np.random.default_rng(nfft + hop)
    w = orc.window(1, nfft).astype(np.float64)
    for n in (1, 7, nfft - 1, nfft, nfft + 1, nfft + hop - 1, nfft + hop, 3 * nfft + 5):
        x = (rng.random(n) * 2 - 1).astype(np.float32)
        got = amd.spectrogram(x, nfft, hop)
        ref = _np_frames(x, nfft, hop, w)
        assert got.shape == ref.shape == (1 if n < nfft else 1 + (n - nfft + hop) // hop, nfft)
        np.testing.assert_allclose(got, ref, rtol=5e-5, atol=5e-5)
        if nfft & (nfft - 1) == 0 and nfft <= 1024:   # Kiss itself misses the tolerance above 1024
            np.testing.assert_allclose(got, orc.spectrogram(x, nfft, hop), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("nfft,hop", [(1024, 256), (400, 160)])
def test_stft_device_empty_signal_is_one_zero_frame(vdev, nfft, hop):
    import ctypes as C
    import torch
    st = vdev.Stft(nfft, hop)
    assert st.frames(0) == 1
    buf = torch.full((2, 8), 3.0, device="cuda")   # a valid signal pointer, n = 0 samples per channel
    L = vdev.lib()
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for f, dt in ((L.vv_dsp_stft_spectrogram_device, torch.float32), (L.vv_dsp_stft_spectrum_device, torch.complex64)):
        out = torch.full((2, 1, nfft), 7.0, dtype=dt, device="cuda")
        nf = C.c_size_t(0)
        assert f(st.h, C.c_void_p(buf.data_ptr()), 0, 2, 8, C.c_void_p(out.data_ptr()), nfft, s, C.byref(nf)) == 0
        torch.cuda.synchronize()
        assert nf.value == 1
        assert bool((out == 0).all())


@pytest.mark.parametrize("nfft,hop,n", [(1024, 256, 1), (1024, 256, 1023), (1024, 256, 1300), (400, 160, 399)])
def test_stft_device_short_signal_writes_every_bin(vdev, orc, nfft, hop, n):
    import torch
    st = vdev.Stft(nfft, hop)
    g = torch.Generator(device="cuda").manual_seed(n)
    sig = torch.rand(3, n, device="cuda", generator=g) * 2 - 1
    fr = st.frames(n)
    out = torch.full((3, fr, nfft), float("nan"), device="cuda")
    st.spectrogram(sig, out=out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert np.isfinite(got).all()
    w = orc.window(1, nfft).astype(np.float64)
    for c in range(3):
        np.testing.assert_allclose(got[c], _np_frames(sig[c].cpu().numpy(), nfft, hop, w), rtol=5e-5, atol=5e-5)


@pytest.mark.parametrize("nfft,hop", [(256, 64), (256, 100), (4096, 1024), (4096, 441)])
def test_stft_mirror_through_lds_all_row_kinds(vdev, orc, nfft, hop):
    """nfft 256 / 4096 (the mirror bins read back through LDS; 4096 magnitude rows
    on k_stft_one, its complex and power rows on k_stft_pair_lds):
    magnitude, complex and power rows of a multi-channel ragged job against
    NumPy f64 at the harness tolerance; magnitude rows equal |complex rows|
    and the power rows |complex rows|^2 of bins 0..nfft/2."""
    import torch
    n = 5 * nfft + 3 * hop + 17
    g = torch.Generator(device="cuda").manual_seed(nfft + hop)
    sig = torch.rand(3, n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(nfft, hop)
    mag = st.spectrogram(sig).cpu().numpy()
    cpx = st.spectrogram(sig, complex_out=True).cpu().numpy()
    pw = st.power(sig).cpu().numpy()
    w = orc.window(1, nfft).astype(np.float64)
    for c in range(3):
        x = sig[c].cpu().numpy()
        fr = st.frames(n)
        pad = np.concatenate([x.astype(np.float64), np.zeros(fr * hop + nfft)])
        X = np.fft.fft(np.stack([pad[f * hop:f * hop + nfft] for f in range(fr)]) * w, axis=1)
        np.testing.assert_allclose(mag[c], np.abs(X), rtol=5e-5, atol=5e-5 * np.sqrt(nfft / 1024))
        np.testing.assert_allclose(cpx[c], X, rtol=5e-5, atol=5e-5 * np.sqrt(nfft / 1024))
        np.testing.assert_allclose(pw[c], np.abs(X[:, :nfft // 2 + 1]) ** 2, rtol=1e-4, atol=1e-4 * nfft)
    # nfft 4096 magnitude rows come from k_stft_one (its last-pass twiddles are
    # other f32 roundings of the same values), the complex rows from
    # k_stft_pair_lds: equal up to f32 transform error, not to the last ulp
    mtol = (5e-5, 5e-5) if nfft == 4096 else (2e-6, 1e-6 * np.sqrt(nfft / 1024))
    np.testing.assert_allclose(mag, np.abs(cpx), rtol=mtol[0], atol=mtol[1])
    np.testing.assert_allclose(pw, np.abs(cpx[..., :nfft // 2 + 1]) ** 2, rtol=1e-5, atol=1e-6 * nfft)
