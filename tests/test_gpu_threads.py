"""Host-buffer calls sharing one handle from several threads (SURVEY 8b row 3:
the HIP backend must be reentrant per plan or say so).  The reference's
vv_dsp_fft_execute takes a const plan (fft.h:227) and its Kiss C2C is
reentrant; here a plan's host-path stream, staging buffers and lanes are
guarded per handle, so concurrent calls take turns and every result equals the
single-threaded one.  ctypes drops the GIL for the foreign call, so the
threads really overlap inside the library."""
import ctypes as C
import threading

import numpy as np
import pytest

from vvapi import C2C, R2C, FWD, OK, StftParams

pytestmark = pytest.mark.gpu


def _run_threads(fns, iters=6):
    errs = []

    def body(fn):
        try:
            for _ in range(iters):
                fn()
        except Exception as e:   # noqa: BLE001 -- reported below
            errs.append(e)
    ts = [threading.Thread(target=body, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs


@pytest.mark.parametrize("kind,n,batch,chunk_mb", [(C2C, 1024, 1, ""), (R2C, 4096, 3, ""),
                                                   (C2C, 1024, 600, "1")])
def test_shared_fft_plan_two_threads(amd_lib_path, knob, kind, n, batch, chunk_mb):
    if chunk_mb:
        knob("HOST_CHUNK_MB", chunk_mb)   # the pipelined two-lane host path
    L = C.CDLL(amd_lib_path)
    L.vv_dsp_fft_make_plan_many.argtypes = [C.c_size_t, C.c_int, C.c_int, C.c_size_t, C.POINTER(C.c_void_p)]
    L.vv_dsp_fft_execute.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.vv_dsp_fft_destroy.argtypes = [C.c_void_p]
    rng = np.random.default_rng(n + batch)
    p = C.c_void_p()
    assert L.vv_dsp_fft_make_plan_many(n, kind, FWD, batch, C.byref(p)) == OK
    try:
        ins, want = [], []
        for _ in range(3):
            if kind == C2C:
                x = (rng.random((batch, n)) - 0.5 + 1j * (rng.random((batch, n)) - 0.5)).astype(np.complex64)
                y = np.empty_like(x)
            else:
                x = (rng.random((batch, n)) - 0.5).astype(np.float32)
                y = np.empty((batch, n // 2 + 1), np.complex64)
            assert L.vv_dsp_fft_execute(p, x.ctypes.data, y.ctypes.data) == OK
            ins.append(x)
            want.append(y)

        def worker(i):
            def fn():
                out = np.empty_like(want[i])
                assert L.vv_dsp_fft_execute(p, ins[i].ctypes.data, out.ctypes.data) == OK
                assert np.array_equal(out, want[i]), i
            return fn
        _run_threads([worker(i) for i in range(3)])
    finally:
        L.vv_dsp_fft_destroy(p)


def test_shared_stft_handle_two_threads(amd):
    rng = np.random.default_rng(2)
    sigs = [rng.uniform(-1, 1, m).astype(np.float32) for m in (48000, 30001, 1000)]
    st, h = amd.stft_create(1024, 256)
    assert st == OK
    try:
        want = [amd.spectrogram_h(h, s, 1024, 256) for s in sigs]

        def worker(i):
            def fn():
                assert np.array_equal(amd.spectrogram_h(h, sigs[i], 1024, 256), want[i]), i
            return fn
        _run_threads([worker(i) for i in range(3)])
    finally:
        amd.lib.vv_dsp_stft_destroy(h)
