"""FIR overlap-save (fir.c:75-135 semantics).  The default kernel for taps <=
257 is k_fir_r32 (1024-point blocks split 32 x 32, one LDS transpose per FFT):
against the direct form and the 16 x 16 x 4 kernels it replaced (knob FIR_R32
= 0), at config 4's shape and at ragged shapes (pairs of a wave straddling
channels, an odd pair count, edge pairs, histories).
The 16 x 16 x 4 kernel's dynamic band walk (k_fir_bulk_reg EXP bit 8,
its bulk launch for jobs of >= 8 pairs per wave slot: persistent grid,
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
    with vv.knobs(FIR_DYN=0, FIR_R32=0):
        return plan(x).clone()


def _walks(fn):
    """(dynamic launches, static launches) made by fn()"""
    d0, s0 = vv.debug_get("STAT_FIR_DYN"), vv.debug_get("STAT_FIR_STATIC")
    fn()
    return vv.debug_get("STAT_FIR_DYN") - d0, vv.debug_get("STAT_FIR_STATIC") - s0


# (nch, n, dynamic walk expected): >= 8 pairs per wave slot of the 256-CU x 16-wave
# grid; n a multiple of 4 (16 B aligned channels: the bulk kernel; other strides
# run every pair through the bounds-checked k_fir_pair)
@pytest.mark.parametrize("nch,n,dyn", [(8, 1 << 24, True), (6, 9_000_004, True), (3, 5_000_004, False),
                                       (1, 777_780, False), (5, 1540, None)])
def test_fir_dynamic_walk_equals_static(vdev, orc, nch, n, dyn):
    import torch
    h = orc.fir_design_lowpass(257, 0.25, 2)
    plan = vdev.FirPlan(torch.from_numpy(h))
    g = torch.Generator(device="cuda").manual_seed(nch * 7 + n % 97)
    x = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    ref = _static(plan, x)
    for _ in range(3):   # the counters come back to zero after every launch
        got = []
        with vv.knobs(FIR_R32=0):
            walks = _walks(lambda: got.append(plan(x)))
        torch.cuda.synchronize()
        # dyn None: every pair is an edge pair (k_fir_pair alone, neither bulk walk)
        assert walks == ((0, 0) if dyn is None else (1, 0) if dyn else (0, 1)), walks
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
    with vv.knobs(FIR_R32=0):
        for _ in range(2):
            with torch.cuda.stream(s1):
                plan(x, out=o1)
            with torch.cuda.stream(s2):
                plan(x, out=o2)
    torch.cuda.synchronize()
    assert vv.debug_get("STAT_FIR_DYN") - d0 == 4
    assert torch.equal(o1, ref)
    assert torch.equal(o2, ref)


# (nch, n): config 4; odd pair totals (a wave's second half idle); pairs of one
# wave in two channels; short channels that are all edge pairs; n < one block
@pytest.mark.parametrize("nch,n", [(8, 1 << 24), (3, 5_000_001), (5, 1537), (7, 100_003), (2, 3000), (1, 700),
                                   (4, 768 * 2 * 5 + 1)])
def test_fir_r32_vs_direct_and_previous(vdev, orc, nch, n):
    """k_fir_r32 against the bit-exact direct form (|err| <= 1e-5, the config-4
    bound of test_gpu_fullsize.py) and against the 16 x 16 x 4 kernel (both are
    f32 overlap-save: within 2e-6 of each other); the path counter shows r32 ran."""
    import torch
    h = orc.fir_design_lowpass(257, 0.25, 2)
    plan = vdev.FirPlan(torch.from_numpy(h))
    g = torch.Generator(device="cuda").manual_seed(nch * 31 + n % 1013)
    x = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    r0 = vv.debug_get("STAT_FIR_R32")
    y = plan(x)
    torch.cuda.synchronize()
    assert vv.debug_get("STAT_FIR_R32") - r0 == 1
    yd = plan(x, direct=True)
    with vv.knobs(FIR_R32=0):
        yo = plan(x)
    torch.cuda.synchronize()
    assert (y - yd).abs().max().item() < 1e-5
    assert (y - yo).abs().max().item() < 2e-6
    y2 = plan(x)   # deterministic
    assert torch.equal(y, y2)


def test_fir_r32_strided_and_prefix(vdev, amd, orc):
    """Channels at a padded stride through the device entry, and the streaming
    history (vv_dsp_fir_apply_fft on host buffers is the zero-state call; the
    prefix path is fir_apply with state through OLS when the library picks it):
    rows equal the contiguous call bit for bit."""
    import torch
    h = orc.fir_design_lowpass(257, 0.25, 2)
    plan = vdev.FirPlan(torch.from_numpy(h))
    nch, n, pad = 3, 2_000_017, 29
    big = torch.rand(nch, n + pad, device="cuda") * 2 - 1
    x = big[:, :n]
    y = torch.full((nch, n + pad), -9.0, device="cuda")
    import ctypes as C
    L = vdev.lib()
    assert L.vv_dsp_fir_apply_fft_device(plan.h, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), n, nch,
                                         n + pad, n + pad, C.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    ref = plan(x.contiguous())
    torch.cuda.synchronize()
    assert torch.equal(y[:, :n], ref)
    assert bool((y[:, n:] == -9.0).all())

