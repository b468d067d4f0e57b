"""Signal -> log-mel / MFCC rows in one launch (vv_dsp_stft_log_mel_device /
vv_dsp_stft_mfcc_device, vv_dsp_amd.h): the power rows of the STFT
(stft.c:112-144 framing, power of bins 0..nfft/2) feed the MFCC plan's
filterbank, log, DCT-II and lifter (src/features/mel.c:208-330) without being
written to HBM.  The contract is equality with the two device steps the
reference's pipeline maps to -- vv_dsp_stft_power_device, then
vv_dsp_log_mel_device / vv_dsp_mfcc_process_device (both pinned against the
reference elsewhere: tests/test_gpu_parity.py mel golden rows) -- bit for bit,
for the fused nfft = 1024 kernel (chunked and dynamic-walk launches) and for
the two-launch path other shapes take."""
import pytest
import vvdsp_amd as vv

pytestmark = pytest.mark.gpu


def _two_step(vdev, st, mf, sig, log_mel):
    pw = st.power(sig)
    return mf.log_mel(pw) if log_mel else mf(pw)


@pytest.mark.parametrize("nfft,hop,sr,n_mels,n_coeffs,nch,n", [
    (1024, 256, 48000, 40, 13, 3, 48000 + 777),     # odd frame count, zero-padded tail
    (1024, 256, 48000, 64, 20, 2, 5 * 48000),
    (1024, 160, 16000, 128, 13, 1, 16000 * 3 + 5),  # M = 128: two filters per lane
    (1024, 512, 44100, 26, 12, 4, 44100),
    (1024, 256, 48000, 40, 13, 1, 700),             # shorter than one frame
    (512, 128, 16000, 40, 13, 3, 16000 * 2 + 3),    # not fused: the two launches
])
@pytest.mark.parametrize("log_mel", [True, False])
def test_stft_mel_equals_two_step(vdev, nfft, hop, sr, n_mels, n_coeffs, nch, n, log_mel):
    import torch
    g = torch.Generator(device="cuda").manual_seed(nfft + n_mels + nch)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(nfft, hop)
    mf = vdev.Mfcc(nfft, n_mels, n_coeffs, float(sr), 20.0, sr / 2.0, lifter=22.0)
    ref = _two_step(vdev, st, mf, sig, log_mel)
    f0, s0 = vv.debug_get("STAT_MEL_FUSED"), vv.debug_get("STAT_MEL_SPLIT")
    got = mf.from_signal(st, sig, log_mel=log_mel)
    torch.cuda.synchronize()
    # the path that ran (vv_dsp_amd.h: one kernel for nfft 1024, hop <= 256 and a
    # multiple of 4, a 16 B aligned signal with a channel stride of 4k floats, and
    # for MFCC at most 60 mel bands; otherwise the two launches)
    fused = nfft == 1024 and hop <= 256 and hop % 4 == 0 and n % 4 == 0 and (log_mel or n_mels <= 60)
    assert (vv.debug_get("STAT_MEL_FUSED") - f0, vv.debug_get("STAT_MEL_SPLIT") - s0) == \
        ((1, 0) if fused else (0, 1))
    assert got.shape == ref.shape
    assert torch.equal(got, ref)
    vv.debug_set("MEL_FUSED", 0)   # the two-launch path of the same entry point
    try:
        two = mf.from_signal(st, sig, log_mel=log_mel)
    finally:
        vv.debug_clear("MEL_FUSED")
    assert torch.equal(two, ref)
    # the 32 x 32 FFT's pipelines (hop 256; knobs POW_R32 = 1 and MEL_R32 = 1):
    # power rows + mel and the fused rows agree with each other bit for bit, and
    # with the default 16 x 16 x 4 path within the FFTs' rounding
    if nfft == 1024 and hop == 256:
        with vv.knobs(POW_R32=1, MEL_R32=1):
            ref16 = _two_step(vdev, st, mf, sig, log_mel)
            got16 = mf.from_signal(st, sig, log_mel=log_mel)
        torch.cuda.synchronize()
        assert torch.equal(got16, ref16)
        assert torch.allclose(got16, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("log_mel", [True, False])
def test_stft_mel_r32_path_taken(vdev, log_mel):
    """knobs POW_R32 = MEL_R32 = 1, hop 256, 8 B aligned channels: the fused rows
    come from k_stft_r32's MEL modes (STAT_MEL_R32), bit-identical to its power
    rows + mel"""
    import torch
    g = torch.Generator(device="cuda").manual_seed(3)
    sig = torch.rand(5, 48000 * 7 + 512, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(1024, 256)
    mf = vdev.Mfcc(1024, 40, 13, 48000.0, 20.0, 20000.0, lifter=22.0)
    with vv.knobs(POW_R32=1, MEL_R32=1):
        vv.debug_clear("STAT_MEL_R32")
        got = mf.from_signal(st, sig, log_mel=log_mel)
        torch.cuda.synchronize()
        assert vv.debug_get("STAT_MEL_R32") == 1
        assert torch.equal(got, _two_step(vdev, st, mf, sig, log_mel))


@pytest.mark.parametrize("log_mel", [True, False])
def test_stft_mel_large_job(vdev, log_mel):
    """Enough pairs for the dynamic walk; channels written at a padded stride."""
    import torch
    nch, n = 3, 6 * 60 * 48000 + 1001
    g = torch.Generator(device="cuda").manual_seed(99)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(1024, 256)
    mf = vdev.Mfcc(1024, 40, 13, 48000.0, 20.0, 20000.0, lifter=22.0)
    ref = _two_step(vdev, st, mf, sig, log_mel)
    fr, width = ref.shape[1], ref.shape[2]
    for _ in range(2):   # repeated launches (the dynamic walk's counters)
        got = mf.from_signal(st, sig, log_mel=log_mel)
        torch.cuda.synchronize()
        assert torch.equal(got, ref)
    # padded channel stride through the C entry point
    import ctypes as C
    pad = fr * width + 37
    buf = torch.full((nch * pad,), -7.0, device="cuda")
    L = vdev.lib()
    f = L.vv_dsp_stft_log_mel_device if log_mel else L.vv_dsp_stft_mfcc_device
    nf = C.c_size_t(0)
    assert f(st.h, mf.h, C.c_void_p(sig.data_ptr()), n, nch, n, C.c_void_p(buf.data_ptr()), pad,
             C.c_void_p(torch.cuda.current_stream().cuda_stream), C.byref(nf)) == 0
    torch.cuda.synchronize()
    assert nf.value == fr
    rows = buf.view(nch, pad)
    assert torch.equal(rows[:, :fr * width].reshape(nch, fr, width), ref)
    assert bool((rows[:, fr * width:] == -7.0).all())


def test_stft_mel_mismatched_plan(vdev):
    import torch
    st = vdev.Stft(1024, 256)
    mf = vdev.Mfcc(512, 40, 13, 16000.0, 20.0, 8000.0)
    sig = torch.rand(1, 48000, device="cuda")
    with pytest.raises(vdev.VvError):
        mf.from_signal(st, sig)
