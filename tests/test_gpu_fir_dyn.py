"""FIR overlap-save through the dynamic band walk (k_fir_bulk_reg EXP bit 8,
the default bulk launch: persistent grid, per-(device, stream) counters reset by
each launch's last waves) against the static XCD walk (VVHIP_FIR_DYN=0): the
same kernel arithmetic, so outputs are bit-identical -- config 4's shape, odd
channel counts and lengths with edge pairs, repeated launches and two streams.
The static walk itself is pinned to the f64 convolution in test_gpu_parity.py /
test_gpu_fullsize.py (fir.c:75-135 overlap-save)."""
import os

import pytest

pytestmark = pytest.mark.gpu


def _static(plan, x):
    os.environ["VVHIP_FIR_DYN"] = "0"
    try:
        return plan(x).clone()
    finally:
        os.environ["VVHIP_FIR_DYN"] = ""


@pytest.mark.parametrize("nch,n", [(8, 1 << 24), (3, 5_000_001), (1, 777_777), (5, 1537)])
def test_fir_dynamic_walk_equals_static(vdev, orc, nch, n):
    import torch
    h = orc.fir_design_lowpass(257, 0.25, 2)
    plan = vdev.FirPlan(torch.from_numpy(h))
    g = torch.Generator(device="cuda").manual_seed(nch * 7 + n % 97)
    x = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    ref = _static(plan, x)
    for _ in range(3):   # the counters come back to zero after every launch
        got = plan(x)
        torch.cuda.synchronize()
        assert torch.equal(got, ref)


def test_fir_dynamic_walk_two_streams(vdev, orc):
    import torch
    h = orc.fir_design_lowpass(257, 0.25, 2)
    plan = vdev.FirPlan(torch.from_numpy(h))
    x = torch.rand(4, 3_000_000, device="cuda") * 2 - 1
    ref = _static(plan, x)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    o1, o2 = torch.empty_like(x), torch.empty_like(x)
    torch.cuda.synchronize()
    for _ in range(2):
        with torch.cuda.stream(s1):
            plan(x, out=o1)
        with torch.cuda.stream(s2):
            plan(x, out=o2)
    torch.cuda.synchronize()
    assert torch.equal(o1, ref)
    assert torch.equal(o2, ref)
