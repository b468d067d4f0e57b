"""Config-5 building blocks on the GPU through the C ABI (vv_dsp_amd.h):
device selection, one rank's channel shard, and the half-spectrum packing that
halves the gather (SURVEY 8e row note 1).  The collective itself is covered by
tests/test_dist_gloo.py (layout) and bench.py's gather leg (RCCL)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_device_select(vdev):
    L = vdev.lib()
    d = C.c_int(-1)
    assert L.vv_dsp_amd_get_device(C.byref(d)) == 0 and 0 <= d.value < vdev.device_count()
    assert L.vv_dsp_amd_set_device(d.value) == 0
    assert L.vv_dsp_amd_set_device(vdev.device_count()) == 3      # OUT_OF_RANGE
    assert L.vv_dsp_amd_set_device(-1) == 3
    assert L.vv_dsp_amd_get_device(None) == 1


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_channel_shard_equals_whole_job(vdev, kind):
    """Rank r of world 3 computes channels shard_range(7, 3, r) through
    vv_dsp_stft_channel_shard_device; stacked, the shards equal the whole 7-channel
    call bit for bit (pairs never span channels)."""
    import torch
    L = vdev.lib()
    nch, n, nfft, hop = 7, 30011, 1024, 256
    g = torch.Generator(device="cuda").manual_seed(5)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(nfft, hop)
    if kind == 0:
        whole = st.spectrogram(sig)
    elif kind == 1:
        whole = st.spectrogram(sig, complex_out=True)
    else:
        whole = st.power(sig)
    parts = []
    dev = torch.cuda.current_device()
    for r in range(3):
        first, count = vdev.shard_range(nch, 3, r)
        out = torch.empty((count,) + tuple(whole.shape[1:]), dtype=whole.dtype, device="cuda")
        fr = C.c_size_t()
        row = whole[0].numel()
        assert L.vv_dsp_stft_channel_shard_device(st.h, dev, C.c_void_p(sig[first].data_ptr()), n, count, n, kind,
                                                  C.c_void_p(out.data_ptr()), row, vdev._stream(), C.byref(fr)) == 0
        assert fr.value == whole.shape[1]
        parts.append(out)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(parts), whole)
    d = C.c_int(-1)
    assert L.vv_dsp_amd_get_device(C.byref(d)) == 0 and d.value == dev     # restored


@pytest.mark.parametrize("nfft,hop", [(1024, 256), (400, 160), (480, 120), (2000, 500), (256, 64), (8192, 2048)])
def test_half_pack_round_trip_bitexact(vdev, nfft, hop):
    """Magnitude rows of the fused STFT kernels are mirror-symmetric bit for bit,
    so unpack(pack(rows)) == rows: the half-bin gather loses nothing."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(nfft)
    sig = torch.rand(3, 20 * nfft + 7, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(nfft, hop)
    mag = st.spectrogram(sig)
    half = vdev.pack_half(mag, nfft)
    assert half.shape == mag.shape[:-1] + (nfft // 2 + 1,)
    assert torch.equal(half, mag[..., :nfft // 2 + 1])
    back = vdev.unpack_half(half, nfft)
    torch.cuda.synchronize()
    assert torch.equal(back, mag)


def test_half_pack_arguments(vdev):
    import torch
    L = vdev.lib()
    x = torch.zeros(4, 16, device="cuda")
    s = vdev._stream()
    assert L.vv_dsp_spectrogram_pack_half_device(None, 4, 16, C.c_void_p(x.data_ptr()), s) == 1
    assert L.vv_dsp_spectrogram_pack_half_device(C.c_void_p(x.data_ptr()), 4, 0, C.c_void_p(x.data_ptr()), s) == 2
    assert L.vv_dsp_spectrogram_unpack_half_device(C.c_void_p(x.data_ptr()), 4, 16, C.c_void_p(x.data_ptr()), s) == 3
    odd = torch.rand(5, 9, device="cuda")      # odd fft_size: bins 0..4, mirror k -> 9 - k
    h = vdev.pack_half(odd, 9)
    back = vdev.unpack_half(h, 9)
    ref = odd[:, [0, 1, 2, 3, 4, 4, 3, 2, 1]]
    torch.cuda.synchronize()
    assert torch.equal(back, ref)
