"""GPU parity of the spectral data-format helpers (src/spectral/utils.c:5-73)
through the reference's C API and the batched device API: the shifts and the
phase wrap are exact (a permutation; the reference's float loops verbatim), so
they must be bit-identical to the compiled reference; the unwrap sums the
reference's own float increments in f64 (the reference sums them in float), so
it is checked against that f64 sum and, at the reference loop's rounding, against
the reference."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 5, 8, 9, 1000, 1024, 4097, 48000, 1 << 20]


@pytest.mark.parametrize("n", SIZES)
def test_shift_and_wrap_bitexact(amd, ref, n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n).astype(np.float32)
    z = (x + 1j * rng.standard_normal(n)).astype(np.complex64)
    for f in ("fftshift", "ifftshift"):
        assert np.array_equal(getattr(amd, f)(x), getattr(ref, f)(x)), (f, n)
        assert np.array_equal(getattr(amd, f)(z), getattr(ref, f)(z)), (f, n)
    ph = (rng.standard_normal(n) * 30).astype(np.float32)
    ph[: min(n, 4)] = [np.float32(np.pi), -np.float32(np.pi), 7 * np.float32(np.pi), 0.0][: min(n, 4)]
    assert np.array_equal(amd.phase_wrap(ph), ref.phase_wrap(ph)), n


def _increments(w):
    """the reference's float increments (utils.c:67-71), in float32 arithmetic"""
    pi, two_pi = np.float32(np.pi), np.float32(2 * np.pi)
    d = np.empty_like(w)
    d[0] = w[0]
    dd = (w[1:] - w[:-1]).astype(np.float32)
    dd = np.where(dd > pi, (dd - two_pi).astype(np.float32), np.where(dd < -pi, (dd + two_pi).astype(np.float32), dd))
    d[1:] = dd
    return d


@pytest.mark.parametrize("n", SIZES)
def test_phase_unwrap(amd, ref, n):
    rng = np.random.default_rng(n + 1)
    true = np.cumsum(rng.uniform(-2.5, 2.5, n))
    w = ref.phase_wrap(true.astype(np.float32))
    u = amd.phase_unwrap(w)
    exact = np.cumsum(_increments(w).astype(np.float64))
    scale = max(1.0, float(np.abs(exact).max()))
    # f64 sum of the same increments, rounded once to float
    assert np.max(np.abs(u - exact)) <= 2 * np.spacing(np.float32(scale)), n
    r = ref.phase_unwrap(w)   # float accumulation: ~sqrt(n) ulp of drift
    assert np.max(np.abs(u - r)) <= max(64, 4 * np.sqrt(n)) * np.spacing(np.float32(scale)), n


def test_utils_batched_device(vdev, amd):
    import torch
    g = torch.Generator(device="cuda").manual_seed(3)
    import ctypes as C
    L = vdev.lib()
    L.vv_dsp_fftshift_device.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_int, C.c_int,
                                         C.c_void_p]
    L.vv_dsp_phase_unwrap_device.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p]
    L.vv_dsp_phase_wrap_device.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for n in (7, 1024, 5000):
        x = torch.randn(9, n, device="cuda", generator=g)
        z = torch.complex(x, torch.randn(9, n, device="cuda", generator=g))
        for t, cpx in ((x, 0), (z, 1)):
            for inv in (0, 1):
                y = torch.empty_like(t)
                assert L.vv_dsp_fftshift_device(t.data_ptr(), y.data_ptr(), n, 9, cpx, inv, s) == 0
                ip = t.clone()   # in place
                assert L.vv_dsp_fftshift_device(ip.data_ptr(), ip.data_ptr(), n, 9, cpx, inv, s) == 0
                torch.cuda.synchronize()
                assert torch.equal(ip, y)
                f = amd.ifftshift if inv else amd.fftshift
                np.testing.assert_array_equal(y[4].cpu().numpy(), f(t[4].cpu().numpy()))
        w = torch.empty_like(x)
        assert L.vv_dsp_phase_wrap_device((x * 20).contiguous().data_ptr(), w.data_ptr(), 9 * n, s) == 0
        u = torch.empty_like(x)
        assert L.vv_dsp_phase_unwrap_device(w.data_ptr(), u.data_ptr(), n, 9, s) == 0
        torch.cuda.synchronize()
        np.testing.assert_array_equal(w[2].cpu().numpy(), amd.phase_wrap((x[2] * 20).cpu().numpy()))
        np.testing.assert_array_equal(u[6].cpu().numpy(), amd.phase_unwrap(w[6].cpu().numpy()))
