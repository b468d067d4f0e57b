"""Zero-phase FIR filtering on the GPU (vv_dsp_filtfilt_fir, reference
src/filter/common.c:23-80) through the C ABI: bit-identical to the reference
compiled from its own sources (the oracle checks the same), including signals
shorter than the reflection pad, a single tap and long filters; the device
batched entry point row by row; the reference's own test (filter_tests.c:62-80)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("taps,n", [(9, 64), (1, 10), (2, 1), (5, 3), (33, 20), (257, 4000), (64, 1000),
                                    (1000, 300), (4097, 9000), (257, 100003), (257, 100000), (15, 65536)])
def test_filtfilt_bitexact(amd, ref, taps, n):
    rng = np.random.default_rng(taps * 7 + n)
    h = (rng.standard_normal(taps) * 0.2).astype(np.float32)
    x = rng.uniform(-1, 1, n).astype(np.float32)
    st, y = amd.filtfilt(h, x)
    assert st == 0
    st_r, yr = ref.filtfilt(h, x)
    assert st_r == 0
    assert np.array_equal(y, yr), (taps, n, np.max(np.abs(y - yr)))


def test_filtfilt_reference_test(amd):
    """filter_tests.c:62-80: 9-tap Hamming lowpass (fc 0.25) on a square wave of
    64 samples; the centre mean stays below 0.2."""
    h = amd.fir_design_lowpass(9, 0.25, 1)
    x = np.where(np.arange(64) % 8 < 4, 1.0, -1.0).astype(np.float32)
    st, y = amd.filtfilt(h, x)
    assert st == 0 and abs(float(np.mean(y[9:55]))) < 0.2


def test_filtfilt_empty_is_noop(amd):
    h = np.ones(5, np.float32)
    st, y = amd.filtfilt(h, np.zeros(0, np.float32))
    assert st == 0 and y.size == 0


@pytest.mark.parametrize("nch,n,taps", [(3, 5000, 257), (2, 7, 33), (3, 20000, 257), (2, 40000, 16)])
def test_filtfilt_device_batched(vdev, ref, nch, n, taps):
    import torch
    rng = np.random.default_rng(nch + n)
    h = (rng.standard_normal(taps) * 0.1).astype(np.float32)
    x = rng.uniform(-1, 1, (nch, n)).astype(np.float32)
    plan = vdev.FirPlan(torch.from_numpy(h))
    y = plan.filtfilt(torch.from_numpy(x).cuda()).cpu().numpy()
    for c in range(nch):
        assert np.array_equal(y[c], ref.filtfilt(h, x[c])[1]), c
