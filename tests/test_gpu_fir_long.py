"""Long FIR filters on the GPU (beyond the fused overlap-save kernels' 6145 taps).

vv_dsp_fir_apply (fir.c:160-196): the direct form keeps the reference's
summation order across LDS tap tiles of 4096 -> bit-identical to the oracle at
any length, including the streaming history.  vv_dsp_fir_apply_fft
(fir.c:75-135): overlap-save over the four-step FFTs (N = pow2 >= 4 (L-1)) ->
within f32 FFT-convolution tolerance of the f64 convolution."""
import ctypes as C

import numpy as np
import pytest
from scipy.signal import fftconvolve

from vvapi import OK, FirState

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("taps,n", [(4097, 9000), (10000, 20000), (32768, 40000)])
def test_fir_direct_long_bitexact(amd, orc, taps, n):
    rng = np.random.default_rng(taps)
    h = orc.fir_design_lowpass(taps, 0.1, 2)
    x = rng.uniform(-1, 1, n).astype(np.float32)
    assert np.array_equal(amd.fir_apply(h, x), orc.fir_apply(h, x))


def test_fir_direct_long_streaming_state(amd, orc):
    """history across calls with a tap count that spans two LDS tiles"""
    rng = np.random.default_rng(9)
    taps = 5000
    h = orc.fir_design_lowpass(taps, 0.2, 1)
    x = rng.standard_normal(12000).astype(np.float32)
    st = FirState()
    assert amd.lib.vv_dsp_fir_state_init(C.byref(st), taps) == OK
    try:
        chunks = [x[:3], x[3:4100], x[4100:4101], x[4101:9999], x[9999:]]
        y = np.concatenate([amd.fir_apply(h, c, state=st) for c in chunks])
    finally:
        amd.lib.vv_dsp_fir_state_free(C.byref(st))
    assert np.array_equal(y, orc.fir_apply(h, x))


@pytest.mark.parametrize("taps", [6146, 10000, 32768, 100000])
def test_fir_fft_long(amd, taps):
    rng = np.random.default_rng(taps + 1)
    h = (rng.standard_normal(taps) / np.sqrt(taps)).astype(np.float32)
    for n in (1, 5000, 3 * taps + 17):
        x = rng.standard_normal(n).astype(np.float32)
        y = amd.fir_apply(h, x, fft=True)
        ref = fftconvolve(x.astype(np.float64), h.astype(np.float64))[:n]
        np.testing.assert_allclose(y, ref, rtol=1e-4, atol=2e-5)


def test_fir_fft_long_multichannel_device(vdev):
    import torch
    rng = np.random.default_rng(3)
    taps = 20000
    h = (rng.standard_normal(taps) / np.sqrt(taps)).astype(np.float32)
    x = rng.standard_normal((3, 70001)).astype(np.float32)
    plan = vdev.FirPlan(torch.from_numpy(h))
    y = plan(torch.from_numpy(x).cuda()).cpu().numpy()
    for c in range(3):
        ref = fftconvolve(x[c].astype(np.float64), h.astype(np.float64))[:x.shape[1]]
        np.testing.assert_allclose(y[c], ref, rtol=1e-4, atol=2e-5)


@pytest.mark.parametrize("taps", [300, 10000])
def test_fir_fft_mode_honours_prefix(amd, taps):
    """vvhip_fir_apply_host(mode 0) with a caller history (vv_dsp_hip.h: taps-1
    samples before x[0], oldest first): the long-filter overlap-save path has no
    history input, so a prefix must route to a path that reads it."""
    L = amd.lib
    rng = np.random.default_rng(taps + 5)
    h = (rng.standard_normal(taps) / np.sqrt(taps)).astype(np.float32)
    pre = rng.standard_normal(taps - 1).astype(np.float32)
    x = rng.standard_normal(3 * taps + 11).astype(np.float32)
    f = C.c_void_p()
    fp = C.POINTER(C.c_float)
    L.vvhip_fir_create.argtypes = [fp, C.c_size_t, C.POINTER(C.c_void_p)]
    L.vvhip_fir_apply_host.argtypes = [C.c_void_p, fp, fp, C.c_size_t, fp, C.c_int]
    L.vvhip_fir_destroy.argtypes = [C.c_void_p]
    assert L.vvhip_fir_create(h.ctypes.data_as(fp), taps, C.byref(f)) == OK
    try:
        y = np.zeros_like(x)
        assert L.vvhip_fir_apply_host(f, x.ctypes.data_as(fp), y.ctypes.data_as(fp), len(x),
                                      pre.ctypes.data_as(fp), 0) == OK
    finally:
        L.vvhip_fir_destroy(f)
    full = np.concatenate([pre, x]).astype(np.float64)
    ref = fftconvolve(full, h.astype(np.float64))[taps - 1: taps - 1 + len(x)]
    np.testing.assert_allclose(y, ref, rtol=1e-4, atol=2e-5)
