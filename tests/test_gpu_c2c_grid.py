"""Batched C2C launch shapes (fft_kernels.hip run_c2c): for 256..4096 points the
default is a non-persistent grid, one transform per wave slot, on the loop-free
kernel (k_c2c<N, FWD, true>); knob C2C_ONE = 0 runs the looping kernel on the
same grid, C2C_TPW = 0 the persistent grid with its one-transform prefetch, and
C2C_TPW = t > 0 t transforms per slot.  The transform arithmetic is the same in
every shape, so outputs must be bit-identical (fft_kiss.c:27-74 semantics,
pinned to f64 by test_gpu_parity.py).  Batches not a multiple of the 4 slots per
workgroup, forward and backward (1/n), out-of-place and in-place."""
import numpy as np
import pytest
import torch
import vvdsp_amd as vv

pytestmark = pytest.mark.gpu


def _x(n, batch, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.complex(torch.rand(batch, n, device="cuda", generator=g) - 0.5,
                         torch.rand(batch, n, device="cuda", generator=g) - 0.5)


@pytest.mark.parametrize("n", [256, 1024, 2048, 4096])
@pytest.mark.parametrize("fwd", [True, False])
def test_c2c_grid_shapes_bit_identical(n, fwd):
    batch = 1031
    x = _x(n, batch, n + fwd)
    p = vv.FftPlan(n, vv.C2C, vv.FWD if fwd else vv.BWD, batch=batch)
    ref = p(x).clone()
    for kn in ({"C2C_ONE": 0}, {"C2C_TPW": 0}, {"C2C_TPW": 3}, {"C2C_TPW": 1, "C2C_ONE": 0}):
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
