"""Framing helpers (reference src/core/framing.c:58-146):
vv_dsp_get_num_frames, vv_dsp_fetch_frame, vv_dsp_overlap_add, and their
batched device forms.

CPU: the oracle restatement bit-exact against the reference's compiled
framing.c on random cases (zero padding, reflection incl. frames longer than
the signal, windows), and the reference's own known answers
(tests/framing_tests.c:17-200) restated.  GPU: the product's host API and the
batched device kernels bit-exact against the oracle (both are copies, one
rounded window multiply, and frame-ordered sums)."""
import numpy as np
import pytest

CASES = [(10, 4, 2), (6, 4, 2), (1000, 256, 128), (1000, 257, 100), (5, 16, 3), (1, 4, 1), (3000, 1024, 256)]


def _check_known_answers(lib):
    """framing_tests.c:17-200 (values restated)."""
    assert lib.get_num_frames(1024, 256, 128, 0) == 7
    assert lib.get_num_frames(1024, 256, 128, 1) == 8
    assert lib.get_num_frames(100, 256, 128, 0) == 0
    assert lib.get_num_frames(100, 256, 128, 1) == 1
    assert lib.get_num_frames(1024, 256, 0, 0) == 0
    sig = np.arange(10, dtype=np.float32)
    for idx, want in ((0, [0, 1, 2, 3]), (1, [2, 3, 4, 5]), (4, [8, 9, 0, 0])):
        st, fr = lib.fetch_frame(sig, 4, 2, idx, 0)
        assert st == 0 and np.array_equal(fr, np.float32(want))
    sig = np.arange(1, 7, dtype=np.float32)
    for idx, want in ((0, [2, 1, 1, 2]), (1, [1, 2, 3, 4])):
        st, fr = lib.fetch_frame(sig, 4, 2, idx, 1)
        assert st == 0 and np.array_equal(fr, np.float32(want))
    st, fr = lib.fetch_frame(np.float32([1, 2, 3, 4]), 4, 4, 0, 0, window=np.float32([0.5, 1, 1, 0.5]))
    assert st == 0 and np.array_equal(fr, np.float32([0.5, 2, 3, 2]))
    out = np.zeros(8, np.float32)
    assert lib.overlap_add(np.float32([1, 2, 3, 4]), out, 2, 0) == 0
    assert lib.overlap_add(np.float32([0.5, 1, 1.5, 2]), out, 2, 1) == 0
    assert np.array_equal(out, np.float32([1, 2, 3.5, 5, 1.5, 2, 0, 0]))
    sig = np.arange(1, 9, dtype=np.float32)
    out = np.zeros(8, np.float32)
    for i in range(lib.get_num_frames(8, 4, 2, 0)):
        st, fr = lib.fetch_frame(sig, 4, 2, i, 0)
        assert st == 0 and lib.overlap_add(fr, out, 2, i) == 0
    assert np.array_equal(out, np.float32([1, 2, 6, 8, 10, 12, 7, 8]))
    # error codes (framing_tests.c test_error_conditions)
    assert lib.fetch_frame(np.float32([1, 2, 3, 4]), 4, 0, 0, 0)[0] == 2
    assert lib.overlap_add(np.float32([1, 2]), np.zeros(0, np.float32), 1, 0) == 2


def _random_pairs(lib_a, lib_b, seed):
    rng = np.random.default_rng(seed)
    for n, L, hop in CASES:
        x = rng.standard_normal(n).astype(np.float32)
        w = rng.random(L).astype(np.float32)
        for center in (0, 1):
            nf = lib_a.get_num_frames(n, L, hop, center)
            assert nf == lib_b.get_num_frames(n, L, hop, center)
            for idx in sorted({0, 1, max(nf - 1, 0), nf, nf + 3}):
                for win in (None, w):
                    sa, fa = lib_a.fetch_frame(x, L, hop, idx, center, win)
                    sb, fb = lib_b.fetch_frame(x, L, hop, idx, center, win)
                    assert sa == sb == 0 and np.array_equal(fa, fb), (n, L, hop, center, idx)
        out_a = rng.standard_normal(n).astype(np.float32)
        out_b = out_a.copy()
        for idx in range(lib_a.get_num_frames(n, L, hop, 0) + 2):
            fr = rng.standard_normal(L).astype(np.float32)
            assert lib_a.overlap_add(fr, out_a, hop, idx) == lib_b.overlap_add(fr, out_b, hop, idx) == 0
        assert np.array_equal(out_a, out_b), (n, L, hop)


def test_oracle_framing_known_answers(orc):
    _check_known_answers(orc)


def test_oracle_framing_bitexact_vs_reference(orc, ref):
    _check_known_answers(ref)
    _random_pairs(orc, ref, 1)


@pytest.mark.gpu
def test_framing_host_api_gpu(amd, orc):
    _check_known_answers(amd)
    _random_pairs(amd, orc, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("n,L,hop,center", [(48000, 1024, 256, 0), (48000, 1024, 256, 1), (3000, 1000, 333, 1),
                                            (700, 1024, 128, 1), (100000, 400, 160, 0)])
def test_framing_device_batched(vdev, orc, n, L, hop, center):
    """vv_dsp_fetch_frames_device / vv_dsp_overlap_add_device over whole frame
    ranges, bit-exact against the per-frame oracle loop."""
    import ctypes as C
    import torch
    lib = vdev.lib()
    lib.vv_dsp_fetch_frames_device.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t,
                                               C.c_size_t, C.c_size_t, C.c_int, C.c_void_p, C.c_void_p]
    lib.vv_dsp_overlap_add_device.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t,
                                              C.c_size_t, C.c_size_t, C.c_void_p]
    rng = np.random.default_rng(n + L + center)
    x = rng.standard_normal(n).astype(np.float32)
    w = rng.random(L).astype(np.float32)
    nf = orc.get_num_frames(n, L, hop, center) + 2   # and two frames past the end
    f0 = 3 if nf > 6 else 0
    cnt = nf - f0
    xd, wd = torch.from_numpy(x).cuda(), torch.from_numpy(w).cuda()
    frd = torch.empty(cnt, L, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    assert lib.vv_dsp_fetch_frames_device(xd.data_ptr(), n, frd.data_ptr(), L, hop, f0, cnt, center, wd.data_ptr(),
                                          s) == 0
    ref = np.stack([orc.fetch_frame(x, L, hop, f0 + i, center, w)[1] for i in range(cnt)])
    assert np.array_equal(frd.cpu().numpy(), ref)
    # overlap-add the same frames back (frame order sums), into a random base signal
    base = rng.standard_normal(n).astype(np.float32)
    od = torch.from_numpy(base.copy()).cuda()
    assert lib.vv_dsp_overlap_add_device(frd.data_ptr(), cnt, od.data_ptr(), n, L, hop, f0, s) == 0
    o_ref = base.copy()
    for i in range(cnt):
        assert orc.overlap_add(ref[i], o_ref, hop, f0 + i) == 0
    assert np.array_equal(od.cpu().numpy(), o_ref)
