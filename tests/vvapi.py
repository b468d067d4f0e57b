"""ctypes binding of the vv-dsp public C API (the reference's names and ABI).

The same binding drives two libraries that export the identical C99 surface:
  * oracle/_ref/libvvref.so  -- the reference's own sources (parity checker), and
  * vv-dsp_amd/lib/libvvdsp_amd.so -- our MI355X drop-in (HIP backend).
so the parity tests read like the reference's own C tests
(tests/fft_backend_tests.c, tests/spectral_tests.c in the reference tree).

ABI follows include/vv_dsp/vv_dsp_types.h:70-128 (float real, {re,im} complex,
int status enum) and include/vv_dsp/spectral/{fft,stft,dct,hilbert}.h,
include/vv_dsp/filter/fir.h of the reference.
"""
import ctypes as C
import numpy as np

OK = 0
ERR_NULL, ERR_SIZE, ERR_RANGE, ERR_INTERNAL, ERR_NAN, ERR_UNSUPPORTED = 1, 2, 3, 4, 5, 6
C2C, R2C, C2R = 0, 1, 2
FWD, BWD = 1, -1
KISS, FFTW, FFTS, HIP = 0, 1, 2, 3
WIN_BOXCAR, WIN_HANN, WIN_HAMMING = 0, 1, 2
FIRWIN_RECT, FIRWIN_HAMMING, FIRWIN_HANNING, FIRWIN_BLACKMAN = 0, 1, 2, 3
DCT_II, DCT_III, DCT_IV = 2, 3, 4

_f32p = C.POINTER(C.c_float)
_vp = C.c_void_p


class StftParams(C.Structure):
    _fields_ = [("fft_size", C.c_size_t), ("hop_size", C.c_size_t), ("window", C.c_int)]


class FirState(C.Structure):
    _fields_ = [("history", _f32p), ("history_size", C.c_size_t),
                ("history_idx", C.c_size_t), ("num_taps", C.c_size_t)]


def _fp(a):
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_f32p)


def _cplx_view(a):
    """complex64 ndarray -> float32 view (interleaved re,im)."""
    a = np.ascontiguousarray(a, dtype=np.complex64)
    return a.view(np.float32)


# ---- CZT and cepstrum (src/spectral/czt.c, src/envelope/{cepstrum,minphase}.c) ----
# The same methods on both wrappers: VvDsp binds the public vv_dsp_* names
# (reference or MI355X library), Oracle the orc_* restatement.
def _czt_names(lib, prefix):
    if prefix == "vv_dsp_":
        return (lib.vv_dsp_czt_params_for_freq_range, lib.vv_dsp_czt_exec_cpx, lib.vv_dsp_czt_exec_real,
                lib.vv_dsp_cepstrum_real, lib.vv_dsp_icepstrum_minphase, lib.vv_dsp_minphase_from_cepstrum)
    return (lib.orc_czt_params, lib.orc_czt_cpx, lib.orc_czt_real, lib.orc_cepstrum_real,
            lib.orc_icepstrum_minphase, lib.orc_minphase_from_cepstrum)


class _CztMixin:
    _prefix = "vv_dsp_"

    def _czt_setup(self):
        if getattr(self, "_czt_ok", False):
            return self._czt_fns
        fns = _czt_names(self.lib, self._prefix)
        par, cpx, real, ceps, iceps, minph = fns
        if self._prefix == "vv_dsp_":
            par.argtypes = [C.c_float, C.c_float, C.c_size_t, C.c_float] + [_f32p] * 4
        else:
            par.argtypes = [C.c_float, C.c_float, C.c_size_t, C.c_float, _f32p, _f32p]
        for f in (cpx, real):
            f.argtypes = [_f32p, C.c_size_t, C.c_size_t] + [C.c_float] * 4 + [_f32p]
        for f in (ceps, iceps, minph):
            f.argtypes = [_f32p, C.c_size_t, _f32p]
        self._czt_fns, self._czt_ok = fns, True
        return fns

    def czt_params(self, f_start, f_end, m, fs):
        """-> (status, W, A) as complex (vv_dsp_czt_params_for_freq_range, czt.c:22-42)"""
        par = self._czt_setup()[0]
        if self._prefix == "vv_dsp_":
            v = [C.c_float() for _ in range(4)]
            st = par(f_start, f_end, m, fs, *[C.cast(C.byref(x), _f32p) for x in v])
            return st, complex(v[0].value, v[1].value), complex(v[2].value, v[3].value)
        w, a = np.zeros(2, np.float32), np.zeros(2, np.float32)
        st = par(f_start, f_end, m, fs, _fp(w), _fp(a))
        return st, complex(w[0], w[1]), complex(a[0], a[1])

    def czt_status(self, x, m, w, a):
        """-> (status, X complex64[m]); x complex -> czt_exec_cpx, real -> czt_exec_real"""
        _, cpx, real = self._czt_setup()[:3]
        X = np.zeros(2 * max(m, 1), np.float32)
        if np.iscomplexobj(x):
            xf = _cplx_view(x)
            st = cpx(_fp(xf), len(x), m, w.real, w.imag, a.real, a.imag, _fp(X))
        else:
            xf = np.ascontiguousarray(x, np.float32)
            st = real(_fp(xf), len(x), m, w.real, w.imag, a.real, a.imag, _fp(X))
        return st, X.view(np.complex64)[:m]

    def czt(self, x, m, w, a):
        st, X = self.czt_status(x, m, w, a)
        if st != OK:
            raise RuntimeError(f"czt status {st}{self._err() if hasattr(self, '_err') else ''}")
        return X

    def _ceps_call(self, i, x, out_len):
        f = self._czt_setup()[i]
        x = np.ascontiguousarray(x, np.float32)
        out = np.zeros(max(out_len, 1), np.float32)
        st = f(_fp(x), len(x), _fp(out))
        if st != OK:
            raise RuntimeError(f"cepstrum-family status {st}")
        return out[:out_len]

    def cepstrum(self, x):
        """vv_dsp_cepstrum_real (cepstrum.c:7-41)"""
        return self._ceps_call(3, x, len(x))

    def icepstrum_minphase(self, c):
        """vv_dsp_icepstrum_minphase (cepstrum.c:43-78)"""
        return self._ceps_call(4, c, len(c))

    def minphase_from_cepstrum(self, c):
        """vv_dsp_minphase_from_cepstrum (minphase.c:7-31) -> complex64[n]"""
        return self._ceps_call(5, c, 2 * len(c)).view(np.complex64)

    # ---- spectral utilities (src/spectral/utils.c:5-73) ------------------
    def _util(self, name, x, out_like=None):
        """-> (status, out) of one utils.c call; x float32 or complex64 (the shifts)"""
        L = self.lib
        cpx = np.iscomplexobj(x)
        xf = _cplx_view(x) if cpx else np.ascontiguousarray(x, np.float32)
        out = np.zeros_like(xf)
        n = len(x)
        if self._prefix == "orc_":
            if name in ("fftshift", "ifftshift"):
                f = L.orc_fftshift
                f.argtypes = [_f32p, _f32p, C.c_size_t, C.c_int, C.c_int]
                st = f(_fp(xf) if n else None, _fp(out) if n else None, n, int(cpx), int(name == "ifftshift"))
            else:
                f = getattr(L, "orc_" + name)
                f.argtypes = [_f32p, _f32p, C.c_size_t]
                st = f(_fp(xf), _fp(out), n)
        else:
            sym = {"fftshift": "vv_dsp_fftshift_", "ifftshift": "vv_dsp_ifftshift_"}.get(name)
            f = getattr(L, sym + ("cpx" if cpx else "real")) if sym else getattr(L, "vv_dsp_" + name)
            f.argtypes = [_f32p, _f32p, C.c_size_t]
            st = f(_fp(xf), _fp(out), n)
        return st, (out.view(np.complex64) if cpx else out)

    def fftshift(self, x):
        return self._util("fftshift", x)[1]

    def ifftshift(self, x):
        return self._util("ifftshift", x)[1]

    def phase_wrap(self, x):
        return self._util("phase_wrap", x)[1]

    def phase_unwrap(self, x):
        return self._util("phase_unwrap", x)[1]



class VvDsp(_CztMixin):
    """Thin wrapper around a library exporting the vv_dsp_* API."""

    def __init__(self, path):
        self.path = path
        self.lib = L = C.CDLL(path)
        L.vv_dsp_fft_make_plan.argtypes = [C.c_size_t, C.c_int, C.c_int, C.POINTER(_vp)]
        L.vv_dsp_fft_execute.argtypes = [_vp, _vp, _vp]
        L.vv_dsp_fft_destroy.argtypes = [_vp]
        L.vv_dsp_fft_set_backend.argtypes = [C.c_int]
        L.vv_dsp_fft_get_backend.restype = C.c_int
        L.vv_dsp_fft_is_backend_available.argtypes = [C.c_int]
        L.vv_dsp_stft_create.argtypes = [C.POINTER(StftParams), C.POINTER(_vp)]
        L.vv_dsp_stft_destroy.argtypes = [_vp]
        L.vv_dsp_stft_process.argtypes = [_vp, _f32p, _f32p]
        L.vv_dsp_stft_reconstruct.argtypes = [_vp, _f32p, _f32p, _f32p]
        L.vv_dsp_stft_spectrogram.argtypes = [_vp, _f32p, C.c_size_t, _f32p, C.POINTER(C.c_size_t)]
        L.vv_dsp_hilbert_analytic.argtypes = [_f32p, C.c_size_t, _f32p]
        L.vv_dsp_instantaneous_phase.argtypes = [_f32p, C.c_size_t, _f32p]
        L.vv_dsp_instantaneous_frequency.argtypes = [_f32p, C.c_size_t, C.c_double, _f32p]
        L.vv_dsp_dct_forward.argtypes = [C.c_size_t, C.c_int, _f32p, _f32p]
        L.vv_dsp_dct_inverse.argtypes = [C.c_size_t, C.c_int, _f32p, _f32p]
        L.vv_dsp_fir_design_lowpass.argtypes = [_f32p, C.c_size_t, C.c_float, C.c_int]
        L.vv_dsp_fir_state_init.argtypes = [C.POINTER(FirState), C.c_size_t]
        L.vv_dsp_fir_state_free.argtypes = [C.POINTER(FirState)]
        L.vv_dsp_fir_state_free.restype = None
        L.vv_dsp_fir_apply.argtypes = [C.POINTER(FirState), _f32p, _f32p, _f32p, C.c_size_t]
        L.vv_dsp_fir_apply_fft.argtypes = [C.POINTER(FirState), _f32p, _f32p, _f32p, C.c_size_t]
        if hasattr(L, "vv_dsp_window_hann"):
            L.vv_dsp_window_hann.argtypes = [C.c_size_t, _f32p]
        if hasattr(L, "vvhip_available"):
            L.vvhip_available.restype = C.c_int
            L.vvhip_last_error.restype = C.c_char_p

    def _err(self):
        if hasattr(self.lib, "vvhip_last_error"):
            return ": " + self.lib.vvhip_last_error().decode(errors="replace")
        return ""

    # ---- FFT ------------------------------------------------------------
    def make_plan(self, n, kind, direction):
        p = _vp()
        st = self.lib.vv_dsp_fft_make_plan(n, kind, direction, C.byref(p))
        return st, p

    def fft(self, x, kind=C2C, direction=FWD, n=None):
        """Execute one transform with the reference's buffer conventions (fft.h:169-177)."""
        if kind == C2C:
            xin = _cplx_view(x)
            n = len(x) if n is None else n
            out = np.zeros(2 * n, np.float32)
        elif kind == R2C:
            xin = np.ascontiguousarray(x, np.float32)
            n = len(x) if n is None else n
            out = np.zeros(2 * (n // 2 + 1), np.float32)
        else:
            xin = _cplx_view(x)
            assert n is not None
            out = np.zeros(n, np.float32)
        st, p = self.make_plan(n, kind, direction)
        if st != OK:
            raise RuntimeError(f"make_plan status {st}{self._err()}")
        try:
            st = self.lib.vv_dsp_fft_execute(p, xin.ctypes.data, out.ctypes.data)
            if st != OK:
                raise RuntimeError(f"execute status {st}{self._err()}")
        finally:
            self.lib.vv_dsp_fft_destroy(p)
        return out.view(np.complex64) if kind != C2R else out

    # ---- STFT -----------------------------------------------------------
    def stft_create(self, nfft, hop, window=WIN_HANN):
        prm = StftParams(nfft, hop, window)
        h = _vp()
        st = self.lib.vv_dsp_stft_create(C.byref(prm), C.byref(h))
        return st, h

    def spectrogram(self, x, nfft, hop, window=WIN_HANN):
        st, h = self.stft_create(nfft, hop, window)
        if st != OK:
            raise RuntimeError(f"stft_create status {st}")
        try:
            return self.spectrogram_h(h, x, nfft, hop)
        finally:
            self.lib.vv_dsp_stft_destroy(h)

    def spectrogram_h(self, h, x, nfft, hop):
        """vv_dsp_stft_spectrogram on an existing handle"""
        x = np.ascontiguousarray(x, np.float32)
        n = len(x)
        frames = 1 if n < nfft else 1 + (n - nfft + hop) // hop
        out = np.zeros(frames * nfft, np.float32)
        nf = C.c_size_t(0)
        st = self.lib.vv_dsp_stft_spectrogram(h, _fp(x), n, _fp(out), C.byref(nf))
        if st != OK:
            raise RuntimeError(f"spectrogram status {st}")
        assert nf.value == frames
        return out.reshape(frames, nfft)

    def stft_process(self, h, frame, nfft):
        spec = np.zeros(2 * nfft, np.float32)
        st = self.lib.vv_dsp_stft_process(h, _fp(np.ascontiguousarray(frame, np.float32)), _fp(spec))
        if st != OK:
            raise RuntimeError(f"stft_process status {st}")
        return spec.view(np.complex64)

    # ---- Hilbert / DCT / FIR -------------------------------------------
    def hilbert(self, x):
        x = np.ascontiguousarray(x, np.float32)
        z = np.zeros(2 * len(x), np.float32)
        st = self.lib.vv_dsp_hilbert_analytic(_fp(x), len(x), _fp(z))
        if st != OK:
            raise RuntimeError(f"hilbert status {st}")
        return z.view(np.complex64)

    def inst_phase(self, z):
        """vv_dsp_instantaneous_phase (hilbert.c:77-96): complex[N] -> unwrapped phase[N]"""
        zf = _cplx_view(z)
        out = np.zeros(len(z), np.float32)
        st = self.lib.vv_dsp_instantaneous_phase(_fp(zf), len(z), _fp(out))
        if st != OK:
            raise RuntimeError(f"instantaneous_phase status {st}{self._err()}")
        return out

    def inst_freq(self, phase, fs):
        """vv_dsp_instantaneous_frequency (hilbert.c:98-113)"""
        phase = np.ascontiguousarray(phase, np.float32)
        out = np.zeros_like(phase)
        st = self.lib.vv_dsp_instantaneous_frequency(_fp(phase), len(phase), fs, _fp(out))
        if st != OK:
            raise RuntimeError(f"instantaneous_frequency status {st}{self._err()}")
        return out

    def dct(self, x, dct_type=DCT_II, inverse=False):
        st, y = self.dct_status(x, dct_type, inverse)
        if st != OK:
            raise RuntimeError(f"dct status {st}")
        return y

    def dct_status(self, x, dct_type=DCT_II, inverse=False):
        """(status, output) of vv_dsp_dct_forward / vv_dsp_dct_inverse."""
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros_like(x)
        f = self.lib.vv_dsp_dct_inverse if inverse else self.lib.vv_dsp_dct_forward
        return f(len(x), dct_type, _fp(x), _fp(y)), y

    def fir_design_lowpass(self, taps, fc, wkind=FIRWIN_HANNING):
        h = np.zeros(taps, np.float32)
        st = self.lib.vv_dsp_fir_design_lowpass(_fp(h), taps, fc, wkind)
        if st != OK:
            raise RuntimeError(f"fir_design status {st}")
        return h

    def fir_apply(self, h, x, fft=False, state=None):
        """Zero-state (fresh) FIR unless a FirState is supplied."""
        h = np.ascontiguousarray(h, np.float32)
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros_like(x)
        own = state is None
        if own:
            state = FirState()
            assert self.lib.vv_dsp_fir_state_init(C.byref(state), len(h)) == OK
        try:
            f = self.lib.vv_dsp_fir_apply_fft if fft else self.lib.vv_dsp_fir_apply
            st = f(C.byref(state), _fp(h), _fp(x), _fp(y), len(x))
            if st != OK:
                raise RuntimeError(f"fir status {st}")
        finally:
            if own:
                self.lib.vv_dsp_fir_state_free(C.byref(state))
        return y

    # ---- framing (src/core/framing.c:58-146) ---------------------------------
    def _framing_setup(self):
        L = self.lib
        if getattr(self, "_framing", False):
            return
        L.vv_dsp_get_num_frames.argtypes = [C.c_size_t, C.c_size_t, C.c_size_t, C.c_int]
        L.vv_dsp_get_num_frames.restype = C.c_size_t
        L.vv_dsp_fetch_frame.argtypes = [_f32p, C.c_size_t, _f32p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int, _f32p]
        L.vv_dsp_overlap_add.argtypes = [_f32p, _f32p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t]
        self._framing = True

    def get_num_frames(self, n, frame_len, hop, center):
        self._framing_setup()
        return self.lib.vv_dsp_get_num_frames(n, frame_len, hop, center)

    def fetch_frame(self, x, frame_len, hop, index, center, window=None):
        """-> (status, frame)"""
        self._framing_setup()
        x = np.ascontiguousarray(x, np.float32)
        fr = np.zeros(frame_len, np.float32)
        w = None if window is None else _fp(np.ascontiguousarray(window, np.float32))
        st = self.lib.vv_dsp_fetch_frame(_fp(x), len(x), _fp(fr), frame_len, hop, index, center, w)
        return st, fr

    def overlap_add(self, frame, out, hop, index):
        """out (float32, modified in place) += frame at index*hop -> status"""
        self._framing_setup()
        frame = np.ascontiguousarray(frame, np.float32)
        assert out.dtype == np.float32 and out.flags.c_contiguous
        return self.lib.vv_dsp_overlap_add(_fp(frame), _fp(out), len(out), len(frame), hop, index)

    def hann(self, n):
        w = np.zeros(n, np.float32)
        assert self.lib.vv_dsp_window_hann(n, _fp(w)) == OK
        return w

    def window(self, kind, n, null_out=False):
        """vv_dsp_window_{boxcar,hann,hamming} (kind = the STFT enum) -> (status, w)"""
        f = (self.lib.vv_dsp_window_boxcar, self.lib.vv_dsp_window_hann, self.lib.vv_dsp_window_hamming)[kind]
        w = np.zeros(max(n, 1), np.float32)
        return f(C.c_size_t(n), None if null_out else _fp(w)), w[:n]

    def filtfilt(self, h, x):
        """vv_dsp_filtfilt_fir (filter/common.c:23-80) -> (status, y)"""
        h = np.ascontiguousarray(h, np.float32)
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros(max(len(x), 1), np.float32)
        st = self.lib.vv_dsp_filtfilt_fir(_fp(h), C.c_size_t(len(h)), _fp(x), _fp(y), C.c_size_t(len(x)))
        return st, y[:len(x)]

    # ---- mel / MFCC (include/vv_dsp/features/mel.h) ---------------------
    def _mel_setup(self):
        L = self.lib
        if getattr(self, "_mel_ok", False):
            return L
        L.vv_dsp_hz_to_mel.argtypes = [C.c_float]
        L.vv_dsp_hz_to_mel.restype = C.c_float
        L.vv_dsp_mel_to_hz.argtypes = [C.c_float]
        L.vv_dsp_mel_to_hz.restype = C.c_float
        L.vv_dsp_mel_filterbank_create.argtypes = [C.c_size_t, C.c_size_t, C.c_float, C.c_float, C.c_float,
                                                   C.c_int, C.POINTER(_f32p), C.POINTER(C.c_size_t),
                                                   C.POINTER(C.c_size_t)]
        L.vv_dsp_mel_filterbank_free.argtypes = [_f32p, C.c_size_t]
        L.vv_dsp_mel_filterbank_free.restype = None
        L.vv_dsp_compute_log_mel_spectrogram.argtypes = [_f32p, C.c_size_t, C.c_size_t, _f32p, C.c_size_t,
                                                         C.c_float, _f32p]
        L.vv_dsp_mfcc.argtypes = [_f32p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int, C.c_float, _f32p]
        L.vv_dsp_mfcc_init.argtypes = [C.c_size_t, C.c_size_t, C.c_size_t, C.c_float, C.c_float, C.c_float,
                                       C.c_int, C.c_int, C.c_float, C.c_float, C.POINTER(_vp)]
        L.vv_dsp_mfcc_process.argtypes = [_vp, _f32p, C.c_size_t, _f32p]
        L.vv_dsp_mfcc_destroy.argtypes = [_vp]
        self._mel_ok = True
        return L

    def hz_to_mel(self, hz):
        return self._mel_setup().vv_dsp_hz_to_mel(hz)

    def mel_to_hz(self, mel):
        return self._mel_setup().vv_dsp_mel_to_hz(mel)

    def mel_filterbank(self, n_fft, n_mels, sr, fmin, fmax, variant=0):
        L = self._mel_setup()
        p, nf, fl = _f32p(), C.c_size_t(), C.c_size_t()
        st = L.vv_dsp_mel_filterbank_create(n_fft, n_mels, sr, fmin, fmax, variant, C.byref(p), C.byref(nf),
                                            C.byref(fl))
        if st != OK:
            return st, None
        fb = np.ctypeslib.as_array(p, shape=(nf.value * fl.value,)).copy().reshape(nf.value, fl.value)
        L.vv_dsp_mel_filterbank_free(p, nf.value)
        return OK, fb

    def log_mel(self, power, fb, eps):
        L = self._mel_setup()
        power = np.ascontiguousarray(power, np.float32)
        fb = np.ascontiguousarray(fb, np.float32)
        out = np.zeros((power.shape[0], fb.shape[0]), np.float32)
        st = L.vv_dsp_compute_log_mel_spectrogram(_fp(power), power.shape[0], power.shape[1], _fp(fb),
                                                  fb.shape[0], eps, _fp(out))
        if st != OK:
            raise RuntimeError(f"log_mel status {st}{self._err()}")
        return out

    def mfcc(self, log_mel, n_coeffs, lifter, dct_type=DCT_II):
        L = self._mel_setup()
        log_mel = np.ascontiguousarray(log_mel, np.float32)
        out = np.zeros((log_mel.shape[0], n_coeffs), np.float32)
        st = L.vv_dsp_mfcc(_fp(log_mel), log_mel.shape[0], log_mel.shape[1], n_coeffs, dct_type, lifter,
                           _fp(out))
        if st != OK:
            raise RuntimeError(f"mfcc status {st}{self._err()}")
        return out

    def mfcc_pipeline(self, power, n_fft, n_mels, n_coeffs, sr, fmin, fmax, lifter, eps):
        """vv_dsp_mfcc_init / _process / _destroy"""
        L = self._mel_setup()
        power = np.ascontiguousarray(power, np.float32)
        plan = _vp()
        st = L.vv_dsp_mfcc_init(n_fft, n_mels, n_coeffs, sr, fmin, fmax, 0, DCT_II, lifter, eps, C.byref(plan))
        if st != OK:
            raise RuntimeError(f"mfcc_init status {st}{self._err()}")
        try:
            out = np.zeros((power.shape[0], n_coeffs), np.float32)
            st = L.vv_dsp_mfcc_process(plan, _fp(power), power.shape[0], _fp(out))
            if st != OK:
                raise RuntimeError(f"mfcc_process status {st}{self._err()}")
        finally:
            L.vv_dsp_mfcc_destroy(plan)
        return out


class Oracle(_CztMixin):
    """Binding of oracle/liboracle.so (our C restatement; test infrastructure)."""
    _prefix = "orc_"

    def __init__(self, path):
        self.lib = L = C.CDLL(path)
        L.orc_fft_c2c.argtypes = [_f32p, _f32p, C.c_size_t, C.c_int]
        L.orc_fft_r2c.argtypes = [_f32p, _f32p, C.c_size_t]
        L.orc_fft_c2r.argtypes = [_f32p, _f32p, C.c_size_t]
        L.orc_window.argtypes = [C.c_int, C.c_size_t, _f32p]
        L.orc_stft_spectrogram.argtypes = [_f32p, C.c_size_t, C.c_size_t, _f32p, C.c_size_t,
                                           _f32p, C.POINTER(C.c_size_t)]
        L.orc_stft_num_frames.argtypes = [C.c_size_t] * 3
        L.orc_stft_num_frames.restype = C.c_size_t
        L.orc_stft_process.argtypes = [_f32p, C.c_size_t, _f32p, _f32p]
        L.orc_stft_reconstruct.argtypes = [_f32p, C.c_size_t, _f32p, _f32p, _f32p]
        L.orc_hilbert_analytic.argtypes = [_f32p, C.c_size_t, _f32p]
        L.orc_inst_phase.argtypes = [_f32p, C.c_size_t, _f32p]
        L.orc_inst_freq.argtypes = [_f32p, C.c_size_t, C.c_double, _f32p]
        L.orc_dct.argtypes = [_f32p, _f32p, C.c_size_t, C.c_int, C.c_int]
        L.orc_fir_design_lowpass.argtypes = [_f32p, C.c_size_t, C.c_float, C.c_int]
        L.orc_fir_apply.argtypes = [_f32p, C.c_size_t, _f32p, C.POINTER(C.c_size_t), _f32p,
                                    _f32p, C.c_size_t]
        L.orc_fir_apply_fft.argtypes = [_f32p, C.c_size_t, _f32p, _f32p, C.c_size_t]

    def fft(self, x, kind=C2C, direction=FWD, n=None):
        if kind == C2C:
            xin = _cplx_view(x)
            n = len(x)
            out = np.zeros(2 * n, np.float32)
            assert self.lib.orc_fft_c2c(_fp(xin), _fp(out), n, direction) == 0
            return out.view(np.complex64)
        if kind == R2C:
            xin = np.ascontiguousarray(x, np.float32)
            n = len(x)
            out = np.zeros(2 * (n // 2 + 1), np.float32)
            assert self.lib.orc_fft_r2c(_fp(xin), _fp(out), n) == 0
            return out.view(np.complex64)
        xin = _cplx_view(x)
        out = np.zeros(n, np.float32)
        assert self.lib.orc_fft_c2r(_fp(xin), _fp(out), n) == 0
        return out

    def window(self, kind, n):
        w = np.zeros(n, np.float32)
        assert self.lib.orc_window(kind, n, _fp(w)) == 0
        return w

    def spectrogram(self, x, nfft, hop, window=WIN_HANN):
        w = self.window(window, nfft)
        x = np.ascontiguousarray(x, np.float32)
        frames = self.lib.orc_stft_num_frames(len(x), nfft, hop)
        out = np.zeros(frames * nfft, np.float32)
        nf = C.c_size_t(0)
        assert self.lib.orc_stft_spectrogram(_fp(w), nfft, hop, _fp(x), len(x), _fp(out),
                                             C.byref(nf)) == 0
        return out.reshape(frames, nfft)

    def hilbert(self, x):
        x = np.ascontiguousarray(x, np.float32)
        z = np.zeros(2 * len(x), np.float32)
        assert self.lib.orc_hilbert_analytic(_fp(x), len(x), _fp(z)) == 0
        return z.view(np.complex64)

    def inst_phase(self, z):
        zf = _cplx_view(z)
        out = np.zeros(len(z), np.float32)
        assert self.lib.orc_inst_phase(_fp(zf), len(z), _fp(out)) == 0
        return out

    def inst_freq(self, phase, fs):
        phase = np.ascontiguousarray(phase, np.float32)
        out = np.zeros_like(phase)
        assert self.lib.orc_inst_freq(_fp(phase), len(phase), fs, _fp(out)) == 0
        return out

    def dct(self, x, dct_type=DCT_II, inverse=False):
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros_like(x)
        assert self.lib.orc_dct(_fp(x), _fp(y), len(x), dct_type, -1 if inverse else 1) == 0
        return y

    def fir_design_lowpass(self, taps, fc, wkind=FIRWIN_HANNING):
        h = np.zeros(taps, np.float32)
        assert self.lib.orc_fir_design_lowpass(_fp(h), taps, fc, wkind) == 0
        return h

    # ---- mel / MFCC (oracle restatement of src/features/mel.c) ----------
    def hz_to_mel(self, hz):
        self.lib.orc_hz_to_mel.argtypes = [C.c_float]
        self.lib.orc_hz_to_mel.restype = C.c_float
        return self.lib.orc_hz_to_mel(hz)

    def mel_to_hz(self, mel):
        self.lib.orc_mel_to_hz.argtypes = [C.c_float]
        self.lib.orc_mel_to_hz.restype = C.c_float
        return self.lib.orc_mel_to_hz(mel)

    def mel_filterbank(self, n_fft, n_mels, sr, fmin, fmax):
        self.lib.orc_mel_filterbank.argtypes = [C.c_size_t, C.c_size_t, C.c_float, C.c_float, C.c_float, _f32p]
        fb = np.zeros((n_mels, n_fft // 2 + 1), np.float32)
        st = self.lib.orc_mel_filterbank(n_fft, n_mels, sr, fmin, fmax, _fp(fb))
        return st, (fb if st == 0 else None)

    def log_mel(self, power, fb, eps):
        self.lib.orc_log_mel.argtypes = [_f32p, C.c_size_t, C.c_size_t, _f32p, C.c_size_t, C.c_float, _f32p]
        power = np.ascontiguousarray(power, np.float32)
        fb = np.ascontiguousarray(fb, np.float32)
        out = np.zeros((power.shape[0], fb.shape[0]), np.float32)
        assert self.lib.orc_log_mel(_fp(power), power.shape[0], power.shape[1], _fp(fb), fb.shape[0], eps,
                                    _fp(out)) == 0
        return out

    def mfcc(self, log_mel, n_coeffs, lifter):
        self.lib.orc_mfcc.argtypes = [_f32p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_float, _f32p]
        log_mel = np.ascontiguousarray(log_mel, np.float32)
        out = np.zeros((log_mel.shape[0], n_coeffs), np.float32)
        assert self.lib.orc_mfcc(_fp(log_mel), log_mel.shape[0], log_mel.shape[1], n_coeffs, lifter, _fp(out)) == 0
        return out

    def get_num_frames(self, n, frame_len, hop, center):
        L = self.lib
        L.orc_get_num_frames.argtypes = [C.c_size_t, C.c_size_t, C.c_size_t, C.c_int]
        L.orc_get_num_frames.restype = C.c_size_t
        return L.orc_get_num_frames(n, frame_len, hop, center)

    def fetch_frame(self, x, frame_len, hop, index, center, window=None):
        L = self.lib
        L.orc_fetch_frame.argtypes = [_f32p, C.c_size_t, _f32p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int, _f32p]
        x = np.ascontiguousarray(x, np.float32)
        fr = np.zeros(frame_len, np.float32)
        w = None if window is None else _fp(np.ascontiguousarray(window, np.float32))
        st = L.orc_fetch_frame(_fp(x), len(x), _fp(fr), frame_len, hop, index, center, w)
        return st, fr

    def overlap_add(self, frame, out, hop, index):
        L = self.lib
        L.orc_overlap_add.argtypes = [_f32p, _f32p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t]
        frame = np.ascontiguousarray(frame, np.float32)
        return L.orc_overlap_add(_fp(frame), _fp(out), len(out), len(frame), hop, index)

    def filtfilt(self, h, x):
        L = self.lib
        L.orc_filtfilt_fir.argtypes = [_f32p, C.c_size_t, _f32p, _f32p, C.c_size_t]
        h = np.ascontiguousarray(h, np.float32)
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros(max(len(x), 1), np.float32)
        assert L.orc_filtfilt_fir(_fp(h), len(h), _fp(x), _fp(y), len(x)) == 0
        return y[:len(x)]

    def fir_apply(self, h, x, fft=False):
        h = np.ascontiguousarray(h, np.float32)
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros_like(x)
        if fft:
            assert self.lib.orc_fir_apply_fft(_fp(h), len(h), _fp(x), _fp(y), len(x)) == 0
        else:
            hist = np.zeros(max(len(h) - 1, 1), np.float32)
            idx = C.c_size_t(0)
            assert self.lib.orc_fir_apply(_fp(h), len(h), _fp(hist), C.byref(idx), _fp(x),
                                          _fp(y), len(x)) == 0
        return y

