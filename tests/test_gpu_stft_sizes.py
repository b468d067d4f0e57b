"""STFT magnitude rows at the reference's other benchmarked sizes
(/root/reference/bench/bench_stft.c:165: nfft 256, 512, 2048, 4096 at hop
nfft/4; stft.c:112-144 semantics) through the round-6 kernels:
  * nfft 256: k_stft_stage (each wave's four frame pairs as one coalesced span,
    rows staged through LDS) -- bit-identical to k_stft_pair_lds (knob
    STFT_STAGE = 0), which is pinned to f64 by test_gpu_parity.py;
  * nfft 2048: k_stft_pair VAR 0 with the half-size exchange and register
    last-pass twiddles (three waves per SIMD);
  * nfft 256 / 4096: mirror-bin posts (bin N - k from bin k's post);
  * nfft 4096: k_stft_one (one frame pair per transform slot, no loop).
Every case checks sampled rows of every channel against NumPy f64 at the
harness rule (VV_PY_RTOL/ATOL, python/test_fft.py:37-38), channels with odd
pair counts and zero-padded tails included."""
import numpy as np
import pytest
import vvdsp_amd as vv

from conftest import tolerances

pytestmark = pytest.mark.gpu


def _hann64(nfft):
    return np.array([0.5 - 0.5 * np.cos(np.float32(2 * np.pi) / np.float32(nfft - 1) * np.float32(i))
                     for i in range(nfft)], np.float64)


def _check_rows(sig, out, nfft, hop, rows=5):
    rtol, atol = tolerances()
    nch, n = sig.shape
    fr = out.shape[1]
    w = _hann64(nfft)
    s = sig.double().cpu().numpy()
    o = out.cpu().numpy()
    for c in range(nch):
        for f in sorted({0, 1, fr // 2, fr - 2, fr - 1} if fr > 2 else set(range(fr))):
            x = np.zeros(nfft)
            seg = s[c, f * hop: f * hop + nfft]
            x[:len(seg)] = seg
            want = np.abs(np.fft.fft(x * w))
            err = np.abs(o[c, f] - want)
            assert np.all(err <= atol + rtol * np.abs(want)), (c, f, err.max())


@pytest.mark.parametrize("nch,n,hop", [(3, 48000 * 7 + 333, 64), (5, 9_999, 64), (1, 256 * 40 + 17, 32), (2, 300, 64),
                                       (4, 48000 * 3, 128), (7, 123_457, 60), (2, 8 * 64 + 256, 64)])
def test_stft256_stage_equals_pair_lds(nch, n, hop):
    import torch
    g = torch.Generator(device="cuda").manual_seed(nch * 7 + n % 101 + hop)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    st = vv.Stft(256, hop)
    got = st.spectrogram(sig).clone()
    with vv.knobs(STFT_STAGE=0):
        ref = st.spectrogram(sig)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    _check_rows(sig, got, 256, hop)


@pytest.mark.parametrize("nfft", [256, 512, 2048, 4096])
def test_stft_reference_sizes_vs_f64(nfft):
    """8 ch x 20 s @ 48 kHz per size, hop nfft/4 (the bulk kernels of each size)"""
    import torch
    hop = nfft // 4
    nch, n = 8, 20 * 48000 + 77
    g = torch.Generator(device="cuda").manual_seed(nfft)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    out = vv.Stft(nfft, hop).spectrogram(sig)
    torch.cuda.synchronize()
    _check_rows(sig, out, nfft, hop)


@pytest.mark.parametrize("nfft", [256, 4096])
def test_stft_mirror_post_complex_rows(nfft):
    """complex rows (k_stft_pair_lds MODE 1): bin N - k is stored as conj(bin k)"""
    import torch
    hop = nfft // 4
    nch, n = 3, 6 * nfft + 5
    g = torch.Generator(device="cuda").manual_seed(nfft + 1)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    z = vv.Stft(nfft, hop).spectrogram(sig, complex_out=True).cpu().numpy()
    k = np.arange(1, nfft // 2)
    assert np.array_equal(z[..., nfft - k], np.conj(z[..., k]))
    w = _hann64(nfft)
    s = sig.double().cpu().numpy()
    for c in range(nch):
        for f in (0, z.shape[1] - 1):
            x = np.zeros(nfft)
            seg = s[c, f * hop: f * hop + nfft]
            x[:len(seg)] = seg
            want = np.fft.fft(x * w)
            assert np.abs(z[c, f] - want).max() <= 5e-5 + 5e-5 * np.abs(want).max() * 4


@pytest.mark.parametrize("nch,n", [(8, 20 * 48000 + 77), (3, 4096 * 9 + 1), (1, 48000 * 30), (5, 4096 + 1024 * 3),
                                   (2, 5000), (2, 1000), (3, 1), (1, 4096)])
def test_stft4096_one_pair_per_slot(nch, n):
    """nfft 4096 magnitude rows on k_stft_one (one frame pair per transform slot,
    no loop; last-pass twiddles as powers in registers) against k_stft_pair_lds
    (knob STFT_ONE = 0): the same transform and mirror-bin posts, up to f32
    rounding (other roundings of the twiddles, and the compiler may contract the
    window product into the first butterflies differently) -- within 2e-5 of the
    largest bin; and against f64 at the harness rule (zero-padded tails, odd
    pair counts, fewer pairs than the grid's eight XCD ranges)."""
    import torch
    nfft = 4096
    hop = nfft // 4
    g = torch.Generator(device="cuda").manual_seed(nch * 5 + n % 97 + nfft)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    st = vv.Stft(nfft, hop)
    got = st.spectrogram(sig).clone()
    with vv.knobs(STFT_ONE=0):
        ref = st.spectrogram(sig)
    torch.cuda.synchronize()
    assert (got - ref).abs().max().item() <= 2e-5 * ref.abs().max().item()
    _check_rows(sig, got, nfft, hop)
