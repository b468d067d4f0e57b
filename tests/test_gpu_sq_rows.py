"""Row emit of the register STFT kernel (mixed_fft.hip k_stft_sq, MODE 1): the
magnitude rows are staged in LDS and flushed per frame pair as 16 B/lane stores
(row length a multiple of 4 floats, output 16 B aligned) or 4 B/lane stores
(441-point rows, or an output view that is not 16 B aligned).  Every flush must
give the same rows as the aligned run, and the rows must match NumPy f64 at the
harness tolerance (python/test_fft.py:37-38) for frames of stft.c:112-144."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LENGTHS = (320, 400, 441, 480, 600, 640, 720, 800, 900, 960)


@pytest.mark.parametrize("nfft", LENGTHS)
def test_unaligned_output_same_rows(vdev, orc, nfft):
    import torch
    hop = nfft // 4
    nch, n = 3, 48000 + 4 * hop + 77   # an odd frame count per channel for some lengths
    g = torch.Generator(device="cuda").manual_seed(nfft)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(nfft, hop)
    fr = st.frames(n)
    ref = st.spectrogram(sig)
    buf = torch.full((nch * fr * nfft + 1,), -1.0, device="cuda")
    out = buf[1:].view(nch, fr, nfft)   # 4 B past a 16 B boundary
    st.spectrogram(sig, out=out)
    torch.cuda.synchronize()
    assert buf[0].item() == -1.0
    assert torch.equal(out, ref)
    # sampled frames of the first and last channel vs NumPy f64
    w = orc.window(1, nfft).astype(np.float64)
    for c in (0, nch - 1):
        x = np.concatenate([sig[c].cpu().numpy().astype(np.float64), np.zeros(nfft)])
        frames = sorted({0, 1, fr // 2, fr - 2, fr - 1})
        X = np.abs(np.fft.fft(np.stack([x[f * hop:f * hop + nfft] for f in frames]) * w, axis=1))
        np.testing.assert_allclose(ref[c][frames].cpu().numpy(), X, rtol=5e-5, atol=5e-5)
