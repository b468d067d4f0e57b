"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every
function the public headers declare, validates arguments exactly like the
reference front-end (src/spectral/fft.c:63-71, stft.c:31-34, dct.c:70-83,
fir.c:51-53,80-81) and -- with no GPU -- fails loudly instead of computing on
the CPU."""
import ctypes as C
import glob
import os
import re

import pytest

from conftest import ROOT
from vvapi import (VvDsp, StftParams, FirState, OK, ERR_NULL, ERR_SIZE, ERR_RANGE, ERR_INTERNAL, ERR_UNSUPPORTED,
                   C2C, R2C, FWD, BWD, KISS, HIP)

DECL = re.compile(r"\b((?:vv_dsp|vvhip)_\w+)\s*\(")


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")) + glob.glob(
            os.path.join(ROOT, "include", "vv_dsp", "**", "*.h"), recursive=True):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        for stmt in text.split(";"):
            stmt = stmt.strip()
            if stmt.startswith("typedef") or "(*" in stmt or "#define" in stmt:
                continue
            m = DECL.search(stmt)
            if m and "(" in stmt:
                names.add(m.group(1))
    return sorted(names)


def test_header_symbols_exported(amd_lib_path):
    lib = C.CDLL(amd_lib_path)
    names = declared_functions()
    assert len(names) > 50, names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"declared but not exported: {missing}"


def test_hip_vtable_exported(amd_lib_path):
    lib = C.CDLL(amd_lib_path)
    assert hasattr(lib, "vv_dsp_fft_hip_vtable")


@pytest.fixture(scope="module")
def cpu_lib(amd_lib_path):
    return VvDsp(amd_lib_path)


def _no_gpu(cpu_lib):
    return cpu_lib.lib.vvhip_available() <= 0


def test_argument_validation_matches_reference(cpu_lib, ref):
    for lib in (cpu_lib, ref):
        L = lib.lib
        p = C.c_void_p()
        assert L.vv_dsp_fft_make_plan(16, C2C, FWD, None) == ERR_NULL
        assert L.vv_dsp_fft_make_plan(0, C2C, FWD, C.byref(p)) == ERR_SIZE
        assert L.vv_dsp_fft_make_plan(16, 7, FWD, C.byref(p)) == ERR_RANGE
        assert L.vv_dsp_fft_make_plan(16, C2C, 0, C.byref(p)) == ERR_RANGE
        assert L.vv_dsp_fft_execute(None, None, None) == ERR_NULL
        assert L.vv_dsp_fft_destroy(None) == OK
        assert L.vv_dsp_fft_set_backend(5) == ERR_RANGE
        assert L.vv_dsp_fft_set_fftw_flag(0) == ERR_UNSUPPORTED
        h = C.c_void_p()
        assert L.vv_dsp_stft_create(None, C.byref(h)) == ERR_NULL
        for bad in (StftParams(0, 1, 1), StftParams(16, 0, 1), StftParams(16, 17, 1)):
            assert L.vv_dsp_stft_create(C.byref(bad), C.byref(h)) == ERR_SIZE
        assert L.vv_dsp_stft_destroy(None) == ERR_NULL
        L.vv_dsp_dct_make_plan.argtypes = [C.c_size_t, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
        assert L.vv_dsp_dct_make_plan(0, 2, 1, C.byref(p)) == ERR_SIZE
        assert L.vv_dsp_dct_make_plan(8, 5, 1, C.byref(p)) == ERR_RANGE
        assert L.vv_dsp_dct_make_plan(8, 2, 0, C.byref(p)) == ERR_RANGE
        import numpy as np
        hbuf = np.zeros(8, np.float32)
        hp = hbuf.ctypes.data_as(C.POINTER(C.c_float))
        assert L.vv_dsp_fir_design_lowpass(None, 8, 0.25, 2) == ERR_NULL
        assert L.vv_dsp_fir_design_lowpass(hp, 0, 0.25, 2) == ERR_SIZE
        assert L.vv_dsp_fir_design_lowpass(hp, 8, 1.5, 2) == ERR_RANGE
        st = FirState()
        assert L.vv_dsp_fir_state_init(C.byref(st), 0) == ERR_SIZE
        assert L.vv_dsp_fir_apply_fft(C.byref(st), hp, hp, hp, 8) == ERR_SIZE   # num_taps == 0
        assert L.vv_dsp_hilbert_analytic(hp, 0, hp) == ERR_SIZE
        assert L.vv_dsp_instantaneous_phase(None, 4, hp) == ERR_NULL
        assert L.vv_dsp_instantaneous_phase(hp, 0, hp) == ERR_SIZE
        assert L.vv_dsp_instantaneous_frequency(hp, 4, 1000.0, None) == ERR_NULL
        assert L.vv_dsp_instantaneous_frequency(hp, 0, 1000.0, hp) == ERR_SIZE
        # czt.c:22-63, cepstrum.c:7-11 / 43-48, minphase.c:7-10 (n = 0: the FFT plan fails -> INTERNAL)
        lib.czt_params(0.0, 1.0, 4, 1000.0)   # binds argtypes
        f = C.c_float()
        fpp = C.cast(C.byref(f), C.POINTER(C.c_float))
        assert L.vv_dsp_czt_params_for_freq_range(0.0, 1.0, 4, 1000.0, None, fpp, fpp, fpp) == ERR_NULL
        assert L.vv_dsp_czt_params_for_freq_range(0.0, 1.0, 0, 1000.0, fpp, fpp, fpp, fpp) == ERR_SIZE
        assert L.vv_dsp_czt_params_for_freq_range(0.0, 1.0, 4, 0.0, fpp, fpp, fpp, fpp) == ERR_SIZE
        for fn in (L.vv_dsp_czt_exec_cpx, L.vv_dsp_czt_exec_real):
            assert fn(None, 4, 4, 1.0, 0.0, 1.0, 0.0, hp) == ERR_NULL
            assert fn(hp, 4, 4, 1.0, 0.0, 1.0, 0.0, None) == ERR_NULL
            assert fn(hp, 0, 4, 1.0, 0.0, 1.0, 0.0, hp) == ERR_SIZE
            assert fn(hp, 4, 0, 1.0, 0.0, 1.0, 0.0, hp) == ERR_SIZE
        for fn in (L.vv_dsp_cepstrum_real, L.vv_dsp_icepstrum_minphase, L.vv_dsp_minphase_from_cepstrum):
            assert fn(None, 4, hp) == ERR_NULL
            assert fn(hp, 4, None) == ERR_NULL
            assert fn(hp, 0, hp) == ERR_INTERNAL
        # utils.c:5-73: shifts and unwrap reject n = 0, wrap accepts it
        z0 = np.zeros(0, np.float32)
        for f in ("fftshift", "ifftshift", "phase_unwrap"):
            assert lib._util(f, z0)[0] == ERR_SIZE
        assert lib._util("phase_wrap", z0)[0] == OK
        for f in (L.vv_dsp_fftshift_real, L.vv_dsp_ifftshift_cpx, L.vv_dsp_phase_wrap, L.vv_dsp_phase_unwrap):
            assert f(None, hp, 4) == ERR_NULL


def test_fir_design_bitexact_host_setup(cpu_lib, orc):
    """Coefficient design is one-time host setup with the reference's arithmetic."""
    for taps in (1, 2, 7, 33, 257, 1000):
        for wk in (0, 1, 2, 3):
            import numpy as np
            assert np.array_equal(cpu_lib.fir_design_lowpass(taps, 0.3, wk), orc.fir_design_lowpass(taps, 0.3, wk),
                                  equal_nan=True)


def test_czt_params_bitexact_host_setup(cpu_lib, ref):
    """vv_dsp_czt_params_for_freq_range is scalar host setup with the reference's
    float arithmetic (czt.c:22-42): bit-identical."""
    for args in ((800.0, 1200.0, 64, 48000.0), (0.0, 24000.0, 1024, 48000.0), (-100.0, 100.0, 3, 1000.0),
                 (5.0, 5.0, 7, 44100.0)):
        assert cpu_lib.czt_params(*args) == ref.czt_params(*args)


def test_mel_filterbank_bitexact_host_setup(cpu_lib, orc, ref):
    """The mel filterbank and conversions are host setup with the reference's
    arithmetic (mel.c:14-193): bit-identical to the reference and the oracle."""
    import numpy as np
    for hz in (0.0, 440.0, 8000.0, -1.0):
        assert cpu_lib.hz_to_mel(hz) == ref.hz_to_mel(hz)
        assert cpu_lib.mel_to_hz(hz) == ref.mel_to_hz(hz)
    for args in ((512, 26, 16000.0, 0.0, 8000.0), (1024, 40, 48000.0, 20.0, 20000.0), (2048, 128, 44100.0, 0.0,
                                                                                        22050.0)):
        st, fb = cpu_lib.mel_filterbank(*args)
        st_r, fb_r = ref.mel_filterbank(*args)
        assert st == st_r == 0 and np.array_equal(fb, fb_r) and np.array_equal(fb, orc.mel_filterbank(*args)[1])
    # argument errors are the reference's codes (mel.c:78-98): size, range, variant
    for bad in ((512, 300, 16000.0, 0.0, 8000.0), (512, 26, 16000.0, 0.0, 9000.0), (0, 26, 16000.0, 0.0, 8000.0)):
        assert cpu_lib.mel_filterbank(*bad)[0] == ref.mel_filterbank(*bad)[0]
    assert cpu_lib.mel_filterbank(512, 26, 16000.0, 0.0, 8000.0, variant=1)[0] == \
        ref.mel_filterbank(512, 26, 16000.0, 0.0, 8000.0, variant=1)[0] == ERR_RANGE


def test_no_gpu_mel_fails_loudly(cpu_lib):
    """The per-frame mel/MFCC work has no CPU path: without a device it reports UNSUPPORTED."""
    import numpy as np
    if not _no_gpu(cpu_lib):
        pytest.skip("a GPU is visible")
    st, fb = cpu_lib.mel_filterbank(512, 26, 16000.0, 0.0, 8000.0)
    assert st == OK
    power = np.ones((2, 257), np.float32)
    for call in (lambda: cpu_lib.log_mel(power, fb, 1e-10), lambda: cpu_lib.mfcc(np.ones((2, 26), np.float32), 13, 0.0),
                 lambda: cpu_lib.mfcc_pipeline(power, 512, 26, 13, 16000.0, 0.0, 8000.0, 22.0, 1e-10)):
        with pytest.raises(RuntimeError, match="status 6"):
            call()


def test_no_gpu_fails_loudly(cpu_lib):
    if not _no_gpu(cpu_lib):
        pytest.skip("a GPU is visible")
    L = cpu_lib.lib
    p = C.c_void_p()
    # no CPU backend is compiled in: KISS slot empty, HIP unavailable -> UNSUPPORTED
    assert L.vv_dsp_fft_is_backend_available(KISS) == 0
    assert L.vv_dsp_fft_is_backend_available(HIP) == 0
    assert L.vv_dsp_fft_make_plan(1024, C2C, FWD, C.byref(p)) == ERR_UNSUPPORTED
    assert L.vv_dsp_fft_set_backend(KISS) == ERR_UNSUPPORTED
    h = C.c_void_p()
    assert L.vv_dsp_stft_create(C.byref(StftParams(1024, 256, 1)), C.byref(h)) == ERR_UNSUPPORTED
    import numpy as np
    x = np.zeros(64, np.float32)
    z = np.zeros(128, np.float32)
    fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
    assert L.vv_dsp_hilbert_analytic(fp(x), 64, fp(z)) == ERR_UNSUPPORTED
    assert L.vv_dsp_dct_forward(64, 2, fp(x), fp(z)) == ERR_UNSUPPORTED
    assert L.vv_dsp_instantaneous_phase(fp(z), 64, fp(x)) == ERR_UNSUPPORTED
    assert L.vv_dsp_instantaneous_frequency(fp(x), 64, 1000.0, fp(z)) == ERR_UNSUPPORTED
    st = FirState()
    assert L.vv_dsp_fir_state_init(C.byref(st), 4) == OK
    assert L.vv_dsp_fir_apply(C.byref(st), fp(x), fp(x), fp(z), 64) == ERR_UNSUPPORTED
    assert L.vv_dsp_fir_apply_fft(C.byref(st), fp(x), fp(x), fp(z), 64) == ERR_UNSUPPORTED
    L.vv_dsp_fir_state_free(C.byref(st))
    cpu_lib.czt_params(0.0, 1.0, 4, 1000.0)   # binds argtypes
    assert L.vv_dsp_czt_exec_cpx(fp(z), 32, 32, 1.0, 0.0, 1.0, 0.0, fp(z)) == ERR_UNSUPPORTED
    assert L.vv_dsp_czt_exec_real(fp(x), 32, 32, 1.0, 0.0, 1.0, 0.0, fp(z)) == ERR_UNSUPPORTED
    assert L.vv_dsp_cepstrum_real(fp(x), 64, fp(x)) == ERR_UNSUPPORTED
    assert L.vv_dsp_icepstrum_minphase(fp(x), 64, fp(x)) == ERR_UNSUPPORTED
    assert L.vv_dsp_minphase_from_cepstrum(fp(x), 64, fp(z)) == ERR_UNSUPPORTED
    for f in ("fftshift", "ifftshift", "phase_wrap", "phase_unwrap"):
        assert cpu_lib._util(f, x)[0] == ERR_UNSUPPORTED
    assert L.vv_dsp_spectral_dummy() == 42
    assert b"no HIP device" in L.vvhip_last_error()


def test_oracle_not_linked_into_product(amd_lib_path):
    """The product must not contain or load the oracle/reference code."""
    import subprocess
    out = subprocess.run(["nm", "-D", amd_lib_path], capture_output=True, text=True).stdout
    assert "orc_" not in out and "kiss_execute" not in out and "fft_iterative_radix2" not in out
    funcs = [ln.split()[-1] for ln in out.splitlines() if " T " in ln]
    # exported functions are the C ABI only (kernel registration stubs are data symbols)
    assert all(s.startswith(("vv_dsp_", "vvhip_")) or s in ("_init", "_fini") for s in funcs), funcs
    ldd = subprocess.run(["ldd", amd_lib_path], capture_output=True, text=True).stdout
    assert "oracle" not in ldd and "vvref" not in ldd


def test_windows_bitexact_host_setup(cpu_lib, ref):
    """vv_dsp_window_{boxcar,hann,hamming} (window.c:16-49): one-time host
    tables with the reference's float arithmetic, bit-identical to the compiled
    reference, with its argument checks (window_tests.c:104-115: N = 0 ->
    INVALID_SIZE, NULL -> NULL_POINTER)."""
    import numpy as np
    for kind in (0, 1, 2):
        for n in (1, 2, 8, 17, 400, 1024, 4096):
            st, w = cpu_lib.window(kind, n)
            st_r, w_r = ref.window(kind, n)
            assert st == st_r == OK
            assert np.array_equal(w, w_r), (kind, n)
        assert cpu_lib.window(kind, 0)[0] == ref.window(kind, 0)[0] == ERR_SIZE
        assert cpu_lib.window(kind, 4, null_out=True)[0] == ERR_NULL
    st, w = cpu_lib.window(1, 8)   # gtest/test_window.cpp:154-178, 1e-6
    exp = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(8) / 7)
    assert np.max(np.abs(w - exp)) <= 1e-6


def test_filtfilt_argument_checks(cpu_lib, ref):
    """common.c:28-29: NULL -> NULL_POINTER, num_taps = 0 -> INVALID_SIZE
    (no GPU needed: checked before any device work)."""
    import numpy as np
    L = cpu_lib.lib
    h = np.ones(3, np.float32)
    x = np.ones(8, np.float32)
    y = np.zeros(8, np.float32)
    for lib in (L, ref.lib):
        assert lib.vv_dsp_filtfilt_fir(None, C.c_size_t(3), x.ctypes.data_as(C.c_void_p), y.ctypes.data_as(C.c_void_p),
                                       C.c_size_t(8)) == ERR_NULL
        assert lib.vv_dsp_filtfilt_fir(h.ctypes.data_as(C.c_void_p), C.c_size_t(0), x.ctypes.data_as(C.c_void_p),
                                       y.ctypes.data_as(C.c_void_p), C.c_size_t(8)) == ERR_SIZE


def test_knob_registry_without_gpu():
    """The A/B knobs and path counters (csrc/hip/debug.hip) through the C-ABI,
    no GPU needed: every documented knob can be set, read back and cleared
    (-1 = unset, the launcher's default path); counters read as integers and
    clear to 0; unknown names and negative values are refused; the VVHIP_
    prefix is accepted."""
    import vvdsp_amd as vv
    knobs = ["STFT_CPS", "STFT_RUN", "STFT_DBS", "POW_OLD", "STFT_RING", "STFT_DYN", "FS_VAR", "FS_CHUNK_MB",
             "FS_OLD", "BLUE_UNFUSED", "C2C_MAX", "STFT_SQ", "MIX_VAR", "MIX_CHUNK_MB", "MIX_R2C_FULL", "FIR_OLD",
             "FIR_DYN", "FIR_DIRECT_LDS", "FIR_BLOCK", "HOST_CHUNK_MB", "NO_MIXED", "REAL_PROMOTE", "ISTFT_OLD",
             "MEL_FUSED", "CZT_UNFUSED", "CEPS_UNFUSED", "FIR_R32", "DIST_SLAB_KB", "POW_R32", "MAG_R32"]
    try:
        for i, k in enumerate(knobs):
            vv.debug_set(k, i + 1)
            assert vv.debug_get(k) == i + 1
            assert vv.debug_get("VVHIP_" + k) == i + 1
            vv.debug_clear(k)
            assert vv.debug_get(k) == -1
        for st in ("STAT_STFT_DYN", "STAT_FIR_DYN", "STAT_FIR_STATIC", "STAT_MEL_FUSED", "STAT_MEL_SPLIT",
                   "STAT_FIR_R32", "STAT_POW_R32", "STAT_MAG_R32"):
            vv.debug_clear(st)
            assert vv.debug_get(st) == 0
        for bad in ("NOT_A_KNOB", "STFT_HALF", "FIR_REG", "MEL_OLD", "C2C_R32"):   # removed in round 4
            with pytest.raises(vv.VvError):
                vv.debug_get(bad)
        assert vv.lib().vvhip_debug_set(b"STFT_DYN", -3) != 0
    finally:
        vv.debug_clear(None)
