"""FIR overlap-save through the dynamic band walk (k_fir_bulk_reg EXP bit 8,
the default bulk launch for jobs of >= 8 pairs per wave slot: persistent grid,
per-(device, stream) counters reset by each launch's last waves) against the
static XCD walk (knob FIR_DYN=0): the same kernel arithmetic, so outputs are
bit-identical -- config 4's shape, odd channel counts and lengths with edge
pairs, repeated launches, two streams and a HIP-graph capture.  The path
counters (vvhip_debug_get STAT_FIR_DYN / STAT_FIR_STATIC) show which walk ran.
The static walk itself is pinned to the f64 convolution in test_gpu_parity.py /
test_gpu_fullsize.py (fir.c:75-135 overlap-save)."""
import pytest
import vvdsp_amd as vv

pytestmark = pytest.mark.gpu


def _static(plan, x):
    with vv.knobs(FIR_DYN=0):
        return plan(x).clone()


def _walks(fn):
    """(dynamic launches, static launches) made by fn()"""
    d0, s0 = vv.debug_get("STAT_FIR_DYN"), vv.debug_get("STAT_FIR_STATIC")
    fn()
    return vv.debug_get("STAT_FIR_DYN") - d0, vv.debug_get("STAT_FIR_STATIC") - s0


# (nch, n, dynamic walk expected): >= 8 pairs per wave slot of the 256-CU x 16-wave grid
@pytest.mark.parametrize("nch,n,dyn", [(8, 1 << 24, True), (6, 9_000_001, True), (3, 5_000_001, False),
                                       (1, 777_777, False), (5, 1537, False)])
def test_fir_dynamic_walk_equals_static(vdev, orc, nch, n, dyn):
    import torch
    h = orc.fir_design_lowpass(257, 0.25, 2)
    plan = vdev.FirPlan(torch.from_numpy(h))
    g = torch.Generator(device="cuda").manual_seed(nch * 7 + n % 97)
    x = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    ref = _static(plan, x)
    for _ in range(3):   # the counters come back to zero after every launch
        got = []
        walks = _walks(lambda: got.append(plan(x)))
        torch.cuda.synchronize()
        assert walks == ((1, 0) if dyn else (0, 1)), walks
        assert torch.equal(got[0], ref)


def test_fir_dynamic_walk_two_streams(vdev, orc):
    import torch
    h = orc.fir_design_lowpass(257, 0.25, 2)
    plan = vdev.FirPlan(torch.from_numpy(h))
    x = torch.rand(5, 12_000_000, device="cuda") * 2 - 1
    ref = _static(plan, x)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    o1, o2 = torch.empty_like(x), torch.empty_like(x)
    torch.cuda.synchronize()
    d0 = vv.debug_get("STAT_FIR_DYN")
    for _ in range(2):
        with torch.cuda.stream(s1):
            plan(x, out=o1)
        with torch.cuda.stream(s2):
            plan(x, out=o2)
    torch.cuda.synchronize()
    assert vv.debug_get("STAT_FIR_DYN") - d0 == 4
    assert torch.equal(o1, ref)
    assert torch.equal(o2, ref)
