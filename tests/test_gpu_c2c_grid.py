"""Batched C2C launch shapes (fft_kernels.hip run_c2c): for 256..4096 points the
default is a non-persistent grid, one transform per wave slot, on the loop-free
kernel (k_c2c<N, FWD, true>); knob C2C_ONE = 0 runs the looping kernel on the
same grid, C2C_TPW = 0 the persistent grid with its one-transform prefetch, and
C2C_TPW = t > 0 t transforms per slot.  The transform arithmetic is the same in
every shape, so outputs must be bit-identical (fft_kiss.c:27-74 semantics,
pinned to f64 by test_gpu_parity.py).  Batches not a multiple of the 4 slots per
workgroup, forward and backward (1/n), out-of-place and in-place."""
import ctypes as C

import numpy as np
import pytest
import torch
import vvdsp_amd as vv

pytestmark = pytest.mark.gpu


def _x(n, batch, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.complex(torch.rand(batch, n, device="cuda", generator=g) - 0.5,
                         torch.rand(batch, n, device="cuda", generator=g) - 0.5)


@pytest.mark.parametrize("n", [16, 32, 64, 128, 256, 1024, 2048, 4096])
@pytest.mark.parametrize("fwd", [True, False])
def test_c2c_grid_shapes_bit_identical(n, fwd):
    """(16..128 points: the default stages each wave's 1024-point block through
    LDS; knob C2C_SMALL = 0 the persistent strided kernel.)  Batch 1031: the last
    wave's block is partial."""
    batch = 1031
    x = _x(n, batch, n + fwd)
    p = vv.FftPlan(n, vv.C2C, vv.FWD if fwd else vv.BWD, batch=batch)
    ref = p(x).clone()
    for kn in ({"C2C_ONE": 0}, {"C2C_TPW": 0}, {"C2C_TPW": 3}, {"C2C_TPW": 1, "C2C_ONE": 0}, {"C2C_SMALL": 0}):
        with vv.knobs(**kn):
            got = p(x).clone()
        assert torch.equal(got.view(torch.int64), ref.view(torch.int64)), kn
    # and the default against f64
    want = np.fft.fft(x.cpu().numpy().astype(np.complex128), axis=1)
    if not fwd:
        want = np.fft.ifft(x.cpu().numpy().astype(np.complex128), axis=1)
    err = np.abs(ref.cpu().numpy() - want).max() / np.abs(want).max()
    assert err < 1e-5, err


def test_c2c_one_transform_in_place():
    n, batch = 1024, 777
    x = _x(n, batch, 5)
    p = vv.FftPlan(n, vv.C2C, vv.FWD, batch=batch)
    ref = p(x).clone()
    y = x.clone()
    p(y, out=y)
    assert torch.equal(y.view(torch.int64), ref.view(torch.int64))


@pytest.mark.parametrize("n", [32, 64, 128, 256, 1024, 4096])
@pytest.mark.parametrize("kind", ["r2c", "c2r"])
def test_real_grid_shapes_bit_identical(n, kind):
    """R2C / C2R (fft_kiss.c:120-174 semantics): C2R of n <= 1024 launches one
    transform per slot on a non-persistent grid by default; knob REAL_TPW = 0 / 1
    forces the persistent / one-per-slot grid -- the same values bit for bit."""
    batch, h = 1029, n // 2 + 1
    g = torch.Generator(device="cuda").manual_seed(n)
    if kind == "r2c":
        x = torch.rand(batch, n, device="cuda", generator=g) - 0.5
        p = vv.FftPlan(n, vv.R2C, vv.FWD, batch=batch)
    else:
        x = torch.complex(torch.rand(batch, h, device="cuda", generator=g) - 0.5,
                          torch.rand(batch, h, device="cuda", generator=g) - 0.5)
        p = vv.FftPlan(n, vv.C2R, vv.BWD, batch=batch)
    ref = p(x).clone()
    # (R2C / C2R of 32..128: staged by default; knobs R2C_SMALL / REAL_SMALL = 0 the strided kernels)
    for kn in ({"REAL_TPW": 0}, {"REAL_TPW": 1}, {"REAL_SMALL": 0}, {"R2C_SMALL": 0}):
        with vv.knobs(**kn):
            got = p(x).clone()
        assert torch.equal(got.view(torch.int32) if got.dtype == torch.float32 else got.view(torch.int64),
                           ref.view(torch.int32) if ref.dtype == torch.float32 else ref.view(torch.int64)), kn
    xn = x.cpu().numpy().astype(np.complex128 if kind == "c2r" else np.float64)
    want = np.fft.rfft(xn, axis=1) if kind == "r2c" else np.fft.irfft(xn, n=n, axis=1)
    err = np.abs(ref.cpu().numpy() - want).max() / np.abs(want).max()
    assert err < 1e-5, err


@pytest.mark.parametrize("n", [400, 441, 960])
@pytest.mark.parametrize("kind", ["c2c", "r2c"])
def test_mixed_register_grid_bit_identical(n, kind):
    """Speech-length C2C and R2C rows on the two-pass register kernel
    (mixed_fft.hip k_stft_sq MODE 0 / 5): a non-persistent grid by default, knob
    MIX_TPW = 0 the persistent one -- the same values bit for bit, and the
    default against f64 (fft_kiss.c:76-92 / 120-147 semantics)."""
    batch = 1037
    g = torch.Generator(device="cuda").manual_seed(n)
    if kind == "c2c":
        x = torch.complex(torch.rand(batch, n, device="cuda", generator=g) - 0.5,
                          torch.rand(batch, n, device="cuda", generator=g) - 0.5)
        p = vv.FftPlan(n, vv.C2C, vv.FWD, batch=batch)
    else:
        x = torch.rand(batch, n, device="cuda", generator=g) - 0.5
        p = vv.FftPlan(n, vv.R2C, vv.FWD, batch=batch)
    ref = p(x).clone()
    with vv.knobs(MIX_TPW=0):
        got = p(x).clone()
    assert torch.equal(got.view(torch.int64), ref.view(torch.int64))
    xn = x.cpu().numpy().astype(np.complex128 if kind == "c2c" else np.float64)
    want = np.fft.fft(xn, axis=1) if kind == "c2c" else np.fft.rfft(xn, axis=1)
    err = np.abs(ref.cpu().numpy() - want).max() / np.abs(want).max()
    assert err < 2e-5, err


@pytest.mark.parametrize("n", [16, 64, 128])
def test_c2c_small_rows_unaligned_buffer(n):
    """A batch starting 8 B past a 16 B boundary takes the strided kernel (the
    staged one needs 16 B aligned buffers): the same values."""
    batch = 333
    flat = _x(1, batch * n + 2, n).view(-1)
    x = flat[1:1 + batch * n].view(batch, n)      # 8 B aligned, not 16
    p = vv.FftPlan(n, vv.C2C, vv.FWD, batch=batch)
    got = p(x).clone()
    ref = p(x.clone()).clone()                     # a fresh (aligned) copy
    assert torch.equal(got.view(torch.int64), ref.view(torch.int64))


def _off(shape, dtype, seed, floats=2):
    """a random (batch, m) tensor whose data starts `floats` floats (8 B) past a
    16 B boundary: a view into a larger allocation"""
    g = torch.Generator(device="cuda").manual_seed(seed)
    per = 2 if dtype == torch.complex64 else 1
    numel = shape[0] * shape[1]
    flat = torch.rand(numel * per + 8, device="cuda", generator=g) - 0.5
    v = flat[floats:floats + numel * per]
    return v.view(torch.complex64).view(shape) if per == 2 else v.view(shape)


@pytest.mark.parametrize("n", [32, 64, 128])
@pytest.mark.parametrize("kind", ["r2c", "c2r", "hilbert", "dct"])
def test_small_real_rows_unaligned_buffers(n, kind):
    """the staged 16..128-point kernels gate on 16 B alignment -- R2C
    on its input, C2R on its output, Hilbert and DCT-II on both buffers.  Views
    8 B past a 16 B boundary (input and output) take the other kernels: the same
    values (bit for bit for R2C / C2R / Hilbert; DCT-II's staged kernel contracts
    differently, so it is held to f64 and to the aligned result at 1e-6)."""
    batch, h = 333, n // 2 + 1
    assert _off((batch, n), torch.float32, 1).data_ptr() % 16 == 8
    L = vv.lib()
    s = torch.cuda.current_stream().cuda_stream
    if kind in ("r2c", "c2r"):
        p = vv.FftPlan(n, vv.R2C if kind == "r2c" else vv.C2R, vv.FWD if kind == "r2c" else vv.BWD, batch=batch)
        x = _off((batch, n), torch.float32, n) if kind == "r2c" else _off((batch, h), torch.complex64, n)
        y = _off((batch, h), torch.complex64, 0) if kind == "r2c" else _off((batch, n), torch.float32, 0)
        p(x, out=y)
        ref = p(x.clone())
    elif kind == "hilbert":
        x = _off((batch, n), torch.float32, n)
        y = _off((batch, n), torch.complex64, 0)
        assert L.vv_dsp_hilbert_analytic_device(C.c_void_p(x.data_ptr()), n, batch, C.c_void_p(y.data_ptr()),
                                                C.c_void_p(s)) == 0
        ref = vv.hilbert(x.clone())
    else:
        x = _off((batch, n), torch.float32, n)
        y = _off((batch, n), torch.float32, 0)
        pl = C.c_void_p()
        assert L.vv_dsp_dct_make_plan(n, 2, 1, C.byref(pl)) == 0
        assert L.vv_dsp_dct_execute_device(pl, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), batch,
                                           C.c_void_p(s)) == 0
        L.vv_dsp_dct_destroy(pl)
        ref = vv.dct(x.clone())
    torch.cuda.synchronize()
    if kind == "dct":
        import scipy.fft
        want = scipy.fft.dct(x.double().cpu().numpy(), type=2, axis=1) / 2
        got = y.cpu().numpy()
        assert np.abs(got - want).max() <= 5e-5 + 5e-5 * np.abs(want).max()
        assert np.allclose(got, ref.cpu().numpy(), rtol=1e-6, atol=1e-6)
    else:
        a, b = y.contiguous(), ref
        if a.dtype == torch.complex64:
            a, b = a.view(torch.float32), b.view(torch.float32)
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
