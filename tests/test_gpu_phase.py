"""GPU parity of the instantaneous phase / frequency (reference
src/spectral/hilbert.c:77-113, test tests/hilbert_tests.c:16-48) through the
C ABI, against the compiled reference and the oracle restatement.

Phase: f64 increments like the reference, summed by a parallel prefix scan, so
only the association of the f64 sum differs (~1e-16 relative): the f32 outputs
must be within one f32 ulp of the reference's and almost all bit-identical.
Frequency: elementwise f64 arithmetic identical to the reference: bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sine_analytic(lib, n, fs, f0, phase=0.0):
    t = np.arange(n) / fs
    return lib.hilbert(np.sin(2 * np.pi * f0 * t + phase).astype(np.float32))


def _within_one_ulp(a, b):
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    assert np.all(d <= np.spacing(np.maximum(np.abs(a), np.abs(b))).astype(np.float64)), float(d.max())
    assert np.mean(a == b) >= 0.999, float(np.mean(a == b))


def test_hilbert_tests_known_answer(amd):
    """hilbert_tests.c:16-48: bin-centred sine, N 256, fs 1000: Re(z) = x within
    1e-3, mean instantaneous frequency within 0.5 Hz of f0."""
    n, fs = 256, 1000.0
    f0 = 31 * fs / n
    x = np.sin(2 * np.pi * f0 * np.arange(n) / fs).astype(np.float32)
    z = amd.hilbert(x)
    assert np.max(np.abs(z.real - x)) <= 1e-3
    fr = amd.inst_freq(amd.inst_phase(z), fs)
    assert fr[0] == 0.0
    assert abs(fr[1:].astype(np.float64).mean() - f0) < 0.5


@pytest.mark.parametrize("n", [1, 2, 3, 255, 4096, 4097, 20000, 300001])
def test_inst_phase_vs_reference(amd, ref, orc, n):
    rng = np.random.default_rng(n)
    z = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
    pa, pr = amd.inst_phase(z), ref.inst_phase(z)
    assert np.array_equal(pr, orc.inst_phase(z))
    _within_one_ulp(pa, pr)
    for fs in (1000.0, 48000.0):
        assert np.array_equal(amd.inst_freq(pr, fs), ref.inst_freq(pr, fs)), fs


def test_inst_phase_sine_and_zeros(amd, ref):
    z = _sine_analytic(ref, 16384, 48000.0, 440.0, 0.3)
    _within_one_ulp(amd.inst_phase(z), ref.inst_phase(z))
    z = np.zeros(5000, np.complex64)   # atan2(0, 0) = 0 everywhere but around the spikes
    z[[10, 4095, 4096, 4999]] = [1 + 1j, -1 - 1e-3j, -1 + 1e-3j, 1j]
    assert np.array_equal(amd.inst_phase(z), ref.inst_phase(z))


def test_inst_phase_freq_batched_device(vdev, amd):
    import torch
    rng = np.random.default_rng(5)
    b, n = 7, 9000
    z = (rng.standard_normal((b, n)) + 1j * rng.standard_normal((b, n))).astype(np.complex64)
    p = vdev.instantaneous_phase(torch.from_numpy(z).cuda())
    f = vdev.instantaneous_frequency(p, 16000.0).cpu().numpy()
    p = p.cpu().numpy()
    for r in range(b):
        assert np.array_equal(p[r], amd.inst_phase(z[r])), r
        assert np.array_equal(f[r], amd.inst_freq(p[r], 16000.0)), r


def test_inst_phase_arguments(amd):
    import ctypes as C
    L = amd.lib
    out = np.zeros(4, np.float32)
    fp = out.ctypes.data_as(C.POINTER(C.c_float))
    assert L.vv_dsp_instantaneous_phase(None, 4, fp) == 1
    assert L.vv_dsp_instantaneous_phase(fp, 0, fp) == 2
    assert L.vv_dsp_instantaneous_frequency(None, 4, 1.0, fp) == 1
    assert L.vv_dsp_instantaneous_frequency(fp, 0, 1.0, fp) == 2


def test_inst_freq_in_place_device(vdev):
    """d_phase == d_freq: the shim reads from a copy (f[i] needs p[i-1])."""
    import ctypes as C
    import torch
    rng = np.random.default_rng(8)
    p = torch.from_numpy(np.cumsum(rng.uniform(-1, 1, (5, 70001)), axis=1).astype(np.float32)).cuda()
    want = vdev.instantaneous_frequency(p, 8000.0)
    L = vdev.lib()
    ip = p.clone()
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert L.vv_dsp_instantaneous_frequency_device(C.c_void_p(ip.data_ptr()), 70001, 5, 8000.0,
                                                   C.c_void_p(ip.data_ptr()), s) == 0
    torch.cuda.synchronize()
    assert torch.equal(ip, want)
