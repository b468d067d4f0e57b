"""Power rows at a row pitch (vv_dsp_stft_power_pitched_device) and the mel
kernels on pitched rows (vv_dsp_log_mel_pitched_device /
vv_dsp_mfcc_process_pitched_device): the same values as the reference's packed
[frame][nfft/2+1] layout (include/vv_dsp/features/mel.h:156-161, stft.c:112-144
frames), bit for bit, with the pad floats untouched.  Pitch 544 (17 whole
128 B lines for nfft 1024) is the line-aligned layout."""
import numpy as np
import pytest
import vvdsp_amd as vv

pytestmark = pytest.mark.gpu


def _sig(nch, n, seed):
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.rand(nch, n, device="cuda", generator=g) * 2 - 1


@pytest.mark.parametrize("nfft,hop,pitch", [(1024, 256, 544), (1024, 256, 513), (1024, 256, 600), (1024, 128, 544),
                                            (512, 128, 288), (256, 64, 160), (4096, 1024, 2080), (400, 160, 224),
                                            (16, 4, 12)])
@pytest.mark.parametrize("knobs", [{}, {"POW_R32": 1}, {"STFT_RING": 0}])
def test_power_pitched_equals_packed(nfft, hop, pitch, knobs):
    import torch
    st = vv.Stft(nfft, hop)
    for nch, n in ((3, 48000 * 3 + 77), (1, nfft + 5 * hop), (2, nfft // 2)):
        sig = _sig(nch, n, nfft + n)
        with vv.knobs(**knobs):
            ref = st.power(sig)
            out = torch.full((nch, st.frames(n), pitch), -7.0, device="cuda")
            st.power(sig, out=out, pitch=pitch)
        torch.cuda.synchronize()
        nb = nfft // 2 + 1
        assert torch.equal(out[:, :, :nb], ref), (nch, n)
        assert bool((out[:, :, nb:] == -7.0).all()), "pad floats written"


def test_power_pitch_below_row_refused():
    st = vv.Stft(1024, 256)
    with pytest.raises(vv.VvError):
        st.power(_sig(1, 4096, 1), pitch=512)


@pytest.mark.parametrize("pitch", [544, 520, 1024, 70000])
def test_mel_on_pitched_rows(pitch):
    """520 / 544: the kernel reads the pitched rows; 1024 / 70000 (a pad past
    64 floats; 70000 floats would not fit a CU's LDS): packed by a 2-D copy first"""
    import torch
    st = vv.Stft(1024, 256)
    mf = vv.Mfcc(1024, 40, 13, 48000.0, 20.0, 20000.0, lifter=22.0)
    sig = _sig(2, 48000 * 5 + 123, 9)
    packed = st.power(sig)
    pitched = st.power(sig, pitch=pitch)
    assert torch.equal(mf.log_mel(pitched, pitched=True), mf.log_mel(packed))
    assert torch.equal(mf(pitched, pitched=True), mf(packed))
    # and the fused signal -> log-mel / MFCC rows
    assert torch.equal(mf.from_signal(st, sig, log_mel=True), mf.log_mel(pitched, pitched=True))


def test_power_pitched_config5_shard_rows():
    """32 ch x 10 min at pitch 544 (the line-aligned layout) against the packed
    rows on sampled frames of every channel"""
    import torch
    st = vv.Stft(1024, 256)
    nch, n = 32, 600 * 48000
    sig = _sig(nch, n, 5)
    fr = st.frames(n)
    out = torch.empty(nch, fr, 544, device="cuda")
    st.power(sig, out=out, pitch=544)
    rng = np.random.default_rng(0)
    frs = sorted(set([0, 1, fr - 2, fr - 1] + list(rng.integers(0, fr, 16))))
    for c in range(nch):
        ref = st.power(sig[c:c + 1, :])   # one channel packed
        assert torch.equal(out[c, frs, :513], ref[0, frs]), c
