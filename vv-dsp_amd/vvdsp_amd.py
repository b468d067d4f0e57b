"""ctypes binding of libvvdsp_amd.so's batched / device-pointer API (vv_dsp_amd.h).

Device memory and streams come from PyTorch (plumbing only): tensors are
passed as raw HBM pointers, streams as hipStream_t handles.  All compute runs
in the library's hand-written gfx950 kernels; there is no Python or CPU
fallback -- loading fails loudly when the library or a device is missing.

`import torch` happens before the library is loaded so that one HIP runtime
(torch's libamdhip64.so.7) serves both.
"""
import ctypes as C
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VVDSP_AMD_LIB") or os.path.join(HERE, "lib", "libvvdsp_amd.so")   # override: A/B builds

OK = 0
C2C, R2C, C2R = 0, 1, 2
FWD, BWD = 1, -1
WIN_BOXCAR, WIN_HANN, WIN_HAMMING = 0, 1, 2

_vp = C.c_void_p
_sz = C.c_size_t
_lib = None


class StftParams(C.Structure):
    _fields_ = [("fft_size", C.c_size_t), ("hop_size", C.c_size_t), ("window", C.c_int)]


class VvError(RuntimeError):
    pass


def lib():
    """Load (once) and return the CDLL; raise if the native library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise VvError(f"native library missing: {LIB_PATH} (run `make -C vv-dsp_amd`)")
    L = C.CDLL(LIB_PATH)
    L.vvhip_available.restype = C.c_int
    L.vvhip_last_error.restype = C.c_char_p
    L.vvhip_version.restype = C.c_char_p
    L.vvhip_debug_set.argtypes = [C.c_char_p, C.c_longlong]
    L.vvhip_debug_clear.argtypes = [C.c_char_p]
    L.vvhip_debug_get.argtypes = [C.c_char_p]
    L.vvhip_debug_get.restype = C.c_longlong
    L.vv_dsp_fft_make_plan_many.argtypes = [_sz, C.c_int, C.c_int, _sz, C.POINTER(_vp)]
    L.vv_dsp_fft_execute_device.argtypes = [_vp, _vp, _vp, _vp]
    L.vv_dsp_fft_destroy.argtypes = [_vp]
    L.vv_dsp_stft_create.argtypes = [C.POINTER(StftParams), C.POINTER(_vp)]
    L.vv_dsp_stft_destroy.argtypes = [_vp]
    L.vv_dsp_stft_spectrogram_device.argtypes = [_vp, _vp, _sz, _sz, _sz, _vp, _sz, _vp, C.POINTER(_sz)]
    L.vv_dsp_stft_spectrum_device.argtypes = [_vp, _vp, _sz, _sz, _sz, _vp, _sz, _vp, C.POINTER(_sz)]
    L.vv_dsp_stft_power_device.argtypes = [_vp, _vp, _sz, _sz, _sz, _vp, _sz, _vp, C.POINTER(_sz)]
    L.vv_dsp_stft_power_pitched_device.argtypes = [_vp, _vp, _sz, _sz, _sz, _vp, _sz, _sz, _vp, C.POINTER(_sz)]
    L.vv_dsp_mfcc_process_pitched_device.argtypes = [_vp, _vp, _sz, _sz, _vp, _vp]
    L.vv_dsp_log_mel_pitched_device.argtypes = [_vp, _vp, _sz, _sz, _vp, _vp]
    L.vv_dsp_stft_log_mel_device.argtypes = [_vp, _vp, _vp, _sz, _sz, _sz, _vp, _sz, _vp, C.POINTER(_sz)]
    L.vv_dsp_stft_mfcc_device.argtypes = [_vp, _vp, _vp, _sz, _sz, _sz, _vp, _sz, _vp, C.POINTER(_sz)]
    L.vv_dsp_stft_frames_range_device.argtypes = [_vp, _vp, _sz, _sz, _sz, _sz, _sz, _vp, _sz, C.c_int, _vp]
    L.vv_dsp_stft_process_device.argtypes = [_vp, _vp, _sz, _vp, _vp]
    L.vv_dsp_stft_reconstruct_device.argtypes = [_vp, _vp, _sz, _vp, _vp, _vp]
    L.vv_dsp_instantaneous_phase_device.argtypes = [_vp, _sz, _sz, _vp, _vp]
    L.vv_dsp_instantaneous_frequency_device.argtypes = [_vp, _sz, _sz, C.c_double, _vp, _vp]
    L.vv_dsp_fir_plan_create.argtypes = [_vp, _sz, C.POINTER(_vp)]
    L.vv_dsp_fir_plan_destroy.argtypes = [_vp]
    L.vv_dsp_fir_apply_fft_device.argtypes = [_vp, _vp, _vp, _sz, _sz, _sz, _sz, _vp]
    L.vv_dsp_fir_apply_direct_device.argtypes = [_vp, _vp, _vp, _sz, _sz, _sz, _sz, _vp]
    L.vv_dsp_filtfilt_fir_device.argtypes = [_vp, _vp, _vp, _sz, _sz, _sz, _sz, _vp]
    L.vv_dsp_hilbert_analytic_device.argtypes = [_vp, _sz, _sz, _vp, _vp]
    L.vv_dsp_dct_make_plan.argtypes = [_sz, C.c_int, C.c_int, C.POINTER(_vp)]
    L.vv_dsp_dct_execute_device.argtypes = [_vp, _vp, _vp, _sz, _vp]
    L.vv_dsp_dct_destroy.argtypes = [_vp]
    L.vv_dsp_mfcc_init.argtypes = [_sz, _sz, _sz, C.c_float, C.c_float, C.c_float, C.c_int, C.c_int, C.c_float,
                                   C.c_float, C.POINTER(_vp)]
    L.vv_dsp_mfcc_destroy.argtypes = [_vp]
    L.vv_dsp_mfcc_process_device.argtypes = [_vp, _vp, _sz, _vp, _vp]
    L.vv_dsp_log_mel_device.argtypes = [_vp, _vp, _sz, _vp, _vp]
    L.vv_dsp_czt_plan_create.argtypes = [_sz, _sz, C.c_float, C.c_float, C.c_float, C.c_float, C.POINTER(_vp)]
    L.vv_dsp_czt_plan_destroy.argtypes = [_vp]
    L.vv_dsp_czt_execute_device.argtypes = [_vp, _vp, C.c_int, _sz, _vp, _vp]
    L.vv_dsp_dist_init_all.argtypes = [C.c_int, C.POINTER(C.c_int), C.POINTER(_vp)]
    L.vv_dsp_dist_init_loopback.argtypes = [C.c_int, C.c_int, C.POINTER(_vp)]
    L.vv_dsp_dist_from_comm.argtypes = [_vp, C.POINTER(_vp)]
    L.vv_dsp_dist_unique_id.argtypes = [C.c_char_p]
    L.vv_dsp_dist_init_rank.argtypes = [C.c_int, C.c_int, C.c_char_p, C.c_int, C.POINTER(_vp)]
    L.vv_dsp_dist_comm_count.argtypes = [_vp, C.c_int, C.POINTER(C.c_int)]
    L.vv_dsp_dist_destroy.argtypes = [_vp]
    L.vv_dsp_dist_local_ranks.argtypes = [_vp]
    L.vv_dsp_dist_rank_info.argtypes = [_vp, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.vv_dsp_dist_stft.argtypes = [_vp, _vp, _vp, _sz, _sz, _sz, C.c_int, _vp, _vp, C.POINTER(_sz)]
    L.vv_dsp_dist_gather_rows.argtypes = [_vp, _vp, _sz, _sz, _sz, C.c_int, _vp, C.c_int, _vp]
    L.vv_dsp_dist_fft.argtypes = [_vp, _sz, C.c_int, C.c_int, _sz, _vp, _vp, _vp]
    L.vv_dsp_dist_fir_apply_fft.argtypes = [_vp, _vp, _sz, _sz, _vp, _sz, _vp, _sz, _vp]
    L.vv_dsp_stft_get_sizes.argtypes = [_vp, C.POINTER(_sz), C.POINTER(_sz)]
    for f in ("cepstrum_real", "icepstrum_minphase", "minphase_from_cepstrum"):
        getattr(L, f"vv_dsp_{f}_device").argtypes = [_vp, _sz, _sz, _vp, _vp]
    L.vvhip_fir_block_size.argtypes = [_vp, _sz]
    L.vvhip_fir_block_size.restype = _sz
    L.vv_dsp_amd_set_device.argtypes = [C.c_int]
    L.vv_dsp_amd_get_device.argtypes = [C.POINTER(C.c_int)]
    L.vv_dsp_shard_range.argtypes = [_sz, _sz, _sz, C.POINTER(_sz), C.POINTER(_sz)]
    L.vv_dsp_stft_channel_shard_device.argtypes = [_vp, C.c_int, _vp, _sz, _sz, _sz, C.c_int, _vp, _sz, _vp,
                                                   C.POINTER(_sz)]
    L.vv_dsp_spectrogram_pack_half_device.argtypes = [_vp, _sz, _sz, _vp, _vp]
    L.vv_dsp_spectrogram_unpack_half_device.argtypes = [_vp, _sz, _sz, _vp, _vp]
    _lib = L
    return L


def _check(st, what):
    if st != OK:
        msg = lib().vvhip_last_error().decode(errors="replace")
        raise VvError(f"{what} failed with status {st}: {msg}")


def _ptr(t):
    assert t.is_cuda and t.is_contiguous(), "device tensors must be contiguous CUDA(HIP) tensors"
    return C.c_void_p(t.data_ptr())


def _stream(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def _expect(t, dtype, numel, what):
    """A kernel trusts the sizes it is given: check a tensor against the plan
    before its pointer goes down (too few elements would be read or written
    past the allocation)."""
    if t.dtype != dtype:
        raise VvError(f"{what}: dtype {t.dtype}, expected {dtype}")
    if t.numel() < numel:
        raise VvError(f"{what}: {t.numel()} elements, the plan needs {numel}")
    if not (t.is_cuda and t.is_contiguous()):
        raise VvError(f"{what}: must be a contiguous device tensor")


def debug_set(name, value):
    """Select a launcher alternative (csrc/hip/debug.hip knob, e.g. "STFT_DYN", 0)."""
    if lib().vvhip_debug_set(name.encode(), int(value)) != 0:
        raise VvError(f"unknown knob {name!r} or bad value {value!r}")


def debug_clear(name=None):
    """Back to the default path (None: every knob, and every path counter to 0)."""
    if lib().vvhip_debug_clear(None if name is None else name.encode()) != 0:
        raise VvError(f"unknown knob {name!r}")


def debug_get(name):
    """A knob's value (-1 = unset) or a path counter ("STAT_FIR_DYN", ...)."""
    v = lib().vvhip_debug_get(name.encode())
    if v == -2:
        raise VvError(f"unknown knob {name!r}")
    return v


class knobs:
    """with vv.knobs(STFT_DYN=0): ...  -- set knobs for a block, clear them after."""

    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        for k, v in self.kw.items():
            debug_set(k, v)
        return self

    def __exit__(self, *exc):
        for k in self.kw:
            debug_clear(k)
        return False


def device_count():
    return lib().vvhip_available()


class FftPlan:
    """Batched FFT plan (vv_dsp_fft_make_plan_many) executed on device tensors."""

    def __init__(self, n, kind=C2C, direction=FWD, batch=1):
        self.n, self.kind, self.direction, self.batch = n, kind, direction, batch
        self.h = _vp()
        _check(lib().vv_dsp_fft_make_plan_many(n, kind, direction, batch, C.byref(self.h)), "make_plan_many")

    def __call__(self, x, out=None, stream=None):
        n, b = self.n, self.batch
        if self.kind == C2C:
            shape, dt, in_dt, in_len = (b, n), torch.complex64, torch.complex64, n
        elif self.kind == R2C:
            shape, dt, in_dt, in_len = (b, n // 2 + 1), torch.complex64, torch.float32, n
        else:
            shape, dt, in_dt, in_len = (b, n), torch.float32, torch.complex64, n // 2 + 1
        _expect(x, in_dt, b * in_len, "fft input")
        if out is None:
            out = torch.empty(shape, dtype=dt, device=x.device)
        _expect(out, dt, shape[0] * shape[1], "fft output")
        _check(lib().vv_dsp_fft_execute_device(self.h, _ptr(x), _ptr(out), _stream(stream)), "fft_execute_device")
        return out

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.vv_dsp_fft_destroy(self.h)
            self.h = None


class Stft:
    """STFT handle: fused window + FFT + |X| (or complex) over many channels."""

    def __init__(self, nfft, hop, window=WIN_HANN):
        self.nfft, self.hop = nfft, hop
        self.h = _vp()
        prm = StftParams(nfft, hop, window)
        _check(lib().vv_dsp_stft_create(C.byref(prm), C.byref(self.h)), "stft_create")

    def frames(self, n):
        return 1 if n < self.nfft else 1 + (n - self.nfft + self.hop) // self.hop

    def spectrogram(self, sig, out=None, stream=None, complex_out=False):
        """sig: (nch, n) or (n,) float32 device tensor -> (nch, frames, nfft)."""
        sig2 = sig if sig.dim() == 2 else sig.unsqueeze(0)
        nch, n = sig2.shape
        fr = self.frames(n)
        dt = torch.complex64 if complex_out else torch.float32
        if sig2.dtype != torch.float32 or sig2.stride(1) != 1:
            raise VvError("stft signal: float32 rows with unit sample stride")
        if out is None:
            out = torch.empty((nch, fr, self.nfft), dtype=dt, device=sig.device)
        _expect(out, dt, nch * fr * self.nfft, "stft output")
        nf = _sz(0)
        f = lib().vv_dsp_stft_spectrum_device if complex_out else lib().vv_dsp_stft_spectrogram_device
        _check(f(self.h, _ptr(sig2), n, nch, sig2.stride(0), _ptr(out), fr * self.nfft, _stream(stream),
                 C.byref(nf)), "stft_spectrogram_device")
        assert nf.value == fr
        return out if sig.dim() == 2 else out[0]

    def power(self, sig, out=None, stream=None, pitch=None):
        """sig: (nch, n) or (n,) float32 -> power spectrogram (nch, frames, nfft//2 + 1).
        pitch: rows `pitch` >= nfft//2 + 1 floats apart (vv_dsp_stft_power_pitched_device):
        returns the (nch, frames, pitch) buffer, bins 0..nfft//2 of each row written."""
        sig2 = sig if sig.dim() == 2 else sig.unsqueeze(0)
        nch, n = sig2.shape
        fr, nh = self.frames(n), self.nfft // 2 + 1
        if sig2.dtype != torch.float32 or sig2.stride(1) != 1:
            raise VvError("stft signal: float32 rows with unit sample stride")
        w = nh if pitch is None else int(pitch)
        if out is None:
            out = torch.empty((nch, fr, w), dtype=torch.float32, device=sig.device)
        _expect(out, torch.float32, nch * fr * w, "stft power output")
        nf = _sz(0)
        if pitch is None:
            _check(lib().vv_dsp_stft_power_device(self.h, _ptr(sig2), n, nch, sig2.stride(0), _ptr(out), fr * nh,
                                                   _stream(stream), C.byref(nf)), "stft_power_device")
        else:
            _check(lib().vv_dsp_stft_power_pitched_device(self.h, _ptr(sig2), n, nch, sig2.stride(0), _ptr(out),
                                                           fr * w, w, _stream(stream), C.byref(nf)),
                   "stft_power_pitched_device")
        assert nf.value == fr
        return out if sig.dim() == 2 else out[0]

    def frames_range(self, sig, frame0, nframes, kind=0, out=None, stream=None):
        """Rows of frames [frame0, frame0 + nframes) of sig's spectrogram (one shard
        of a long signal): kind 0 magnitude, 1 complex, 2 power (nfft//2 + 1 bins)."""
        sig2 = sig if sig.dim() == 2 else sig.unsqueeze(0)
        nch, n = sig2.shape
        width = self.nfft // 2 + 1 if kind == 2 else self.nfft
        dt = torch.complex64 if kind == 1 else torch.float32
        if sig2.dtype != torch.float32 or sig2.stride(1) != 1:
            raise VvError("stft signal: float32 rows with unit sample stride")
        if out is None:
            out = torch.empty((nch, nframes, width), dtype=dt, device=sig.device)
        _expect(out, dt, nch * nframes * width, "stft frames_range output")
        if nframes == 0 and frame0 <= self.frames(n):   # empty range: nothing to write (out has no storage)
            return out if sig.dim() == 2 else out[0]
        _check(lib().vv_dsp_stft_frames_range_device(self.h, _ptr(sig2), n, nch, sig2.stride(0), frame0, nframes,
                                                      _ptr(out), nframes * width, kind, _stream(stream)),
               "stft_frames_range_device")
        return out if sig.dim() == 2 else out[0]

    def process(self, frames, stream=None):
        """frames: (count, nfft) float32 -> (count, nfft) complex64 (vv_dsp_stft_process batched)."""
        _expect(frames, torch.float32, frames.shape[0] * self.nfft, "stft_process frames")
        out = torch.empty((frames.shape[0], self.nfft), dtype=torch.complex64, device=frames.device)
        _check(lib().vv_dsp_stft_process_device(self.h, _ptr(frames), frames.shape[0], _ptr(out),
                                                _stream(stream)), "stft_process_device")
        return out

    def reconstruct(self, spec, out_add, norm_add=None, stream=None):
        """spec: (count, nfft) complex64 frames at this handle's hop; adds into
        out_add (and norm_add), each at least (count - 1) * hop + nfft long."""
        count = spec.shape[0]
        _expect(spec, torch.complex64, count * self.nfft, "stft_reconstruct spectra")
        need = (count - 1) * self.hop + self.nfft if count else 0
        _expect(out_add, torch.float32, need, "stft_reconstruct out_add")
        if norm_add is not None:
            _expect(norm_add, torch.float32, need, "stft_reconstruct norm_add")
        _check(lib().vv_dsp_stft_reconstruct_device(self.h, _ptr(spec), spec.shape[0], _ptr(out_add),
                                                    _ptr(norm_add) if norm_add is not None else None,
                                                    _stream(stream)), "stft_reconstruct_device")
        return out_add

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.vv_dsp_stft_destroy(self.h)
            self.h = None


class Mfcc:
    """vv_dsp_mfcc_init plan (src/features/mel.c:249-310) run on device power rows:
    (..., n_fft//2 + 1) float32 -> MFCC (..., n_coeffs) or log-mel (..., n_mels)."""

    def __init__(self, n_fft, n_mels, n_coeffs, sample_rate, fmin, fmax, lifter=0.0, eps=1e-10):
        self.n_fft, self.n_mels, self.n_coeffs = n_fft, n_mels, n_coeffs
        self.h = _vp()
        _check(lib().vv_dsp_mfcc_init(n_fft, n_mels, n_coeffs, sample_rate, fmin, fmax, 0, 2, lifter, eps,
                                      C.byref(self.h)), "mfcc_init")

    def _run(self, power, width, f, fp, what, stream, pitched):
        nb = self.n_fft // 2 + 1
        if pitched:   # rows power.shape[-1] >= nb floats apart, bins 0..nb-1 used
            w = power.shape[-1]
            if w < nb:
                raise VvError(f"pitched power rows: pitch {w} below {nb} bins")
            p2 = power.reshape(-1, w)
            out = torch.empty((p2.shape[0], width), dtype=torch.float32, device=power.device)
            _check(fp(self.h, _ptr(p2), p2.shape[0], w, _ptr(out), _stream(stream)), what)
            return out.reshape(*power.shape[:-1], width)
        assert power.shape[-1] == nb, f"power rows must have {nb} bins"
        p2 = power.reshape(-1, nb)
        out = torch.empty((p2.shape[0], width), dtype=torch.float32, device=power.device)
        _check(f(self.h, _ptr(p2), p2.shape[0], _ptr(out), _stream(stream)), what)
        return out.reshape(*power.shape[:-1], width)

    def __call__(self, power, stream=None, pitched=False):
        """pitched: power's last dimension is the row pitch (vv_dsp_mfcc_process_pitched_device)"""
        return self._run(power, self.n_coeffs, lib().vv_dsp_mfcc_process_device,
                         lib().vv_dsp_mfcc_process_pitched_device, "mfcc_process_device", stream, pitched)

    def log_mel(self, power, stream=None, pitched=False):
        return self._run(power, self.n_mels, lib().vv_dsp_log_mel_device, lib().vv_dsp_log_mel_pitched_device,
                         "log_mel_device", stream, pitched)

    def from_signal(self, stft, sig, log_mel=False, out=None, stream=None):
        """Signal (nch, n) or (n,) float32 -> MFCC (nch, frames, n_coeffs), or log-mel
        (nch, frames, n_mels) with log_mel=True, through `stft`'s power rows without
        writing them to HBM (vv_dsp_stft_mfcc_device / vv_dsp_stft_log_mel_device):
        equal to self(stft.power(sig)) / self.log_mel(stft.power(sig))."""
        sig2 = sig if sig.dim() == 2 else sig.unsqueeze(0)
        nch, n = sig2.shape
        if sig2.dtype != torch.float32 or sig2.stride(1) != 1:
            raise VvError("mel signal: float32 rows with unit sample stride")
        fr = stft.frames(n)
        width = self.n_mels if log_mel else self.n_coeffs
        if out is None:
            out = torch.empty((nch, fr, width), dtype=torch.float32, device=sig.device)
        _expect(out, torch.float32, nch * fr * width, "mel output")
        f = lib().vv_dsp_stft_log_mel_device if log_mel else lib().vv_dsp_stft_mfcc_device
        nf = _sz(0)
        _check(f(stft.h, self.h, _ptr(sig2), n, nch, sig2.stride(0), _ptr(out), fr * width, _stream(stream),
                 C.byref(nf)), "stft_mel_device")
        assert nf.value == fr
        return out if sig.dim() == 2 else out[0]

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.vv_dsp_mfcc_destroy(self.h)
            self.h = None


class FirPlan:
    def __init__(self, h):
        h = h.detach().to("cpu", torch.float32).contiguous()
        self.taps = h.numel()
        self.h = _vp()
        _check(lib().vv_dsp_fir_plan_create(C.c_void_p(h.data_ptr()), self.taps, C.byref(self.h)), "fir_plan_create")

    def __call__(self, x, out=None, direct=False, stream=None):
        """x: (nch, n) float32 device tensor -> y (nch, n)."""
        x2 = x if x.dim() == 2 else x.unsqueeze(0)
        nch, n = x2.shape
        if out is None:
            out = torch.empty_like(x2)
        f = lib().vv_dsp_fir_apply_direct_device if direct else lib().vv_dsp_fir_apply_fft_device
        _check(f(self.h, _ptr(x2), _ptr(out), n, nch, x2.stride(0), out.stride(0), _stream(stream)), "fir_apply")
        return out if x.dim() == 2 else out[0]

    def filtfilt(self, x, out=None, stream=None):
        """Zero-phase filtering (vv_dsp_filtfilt_fir, filter/common.c:23-80) of
        x: (nch, n) float32 device tensor -> y (nch, n), bit-identical per row."""
        x2 = x if x.dim() == 2 else x.unsqueeze(0)
        nch, n = x2.shape
        if x2.dtype != torch.float32 or x2.stride(1) != 1:
            raise VvError("filtfilt input: float32 rows with unit sample stride")
        if out is None:
            out = torch.empty_like(x2)
        _expect(out, torch.float32, nch * n, "filtfilt output")
        _check(lib().vv_dsp_filtfilt_fir_device(self.h, _ptr(x2), _ptr(out), n, nch, x2.stride(0), out.stride(0),
                                                _stream(stream)), "filtfilt_device")
        return out if x.dim() == 2 else out[0]

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.vv_dsp_fir_plan_destroy(self.h)
            self.h = None


def shard_range(total, world, rank):
    """vv_dsp_shard_range: rank's contiguous channel block (first, count)."""
    a, b = _sz(), _sz()
    _check(lib().vv_dsp_shard_range(total, world, rank, C.byref(a), C.byref(b)), "shard_range")
    return a.value, b.value


def pack_half(rows, nfft, out=None, stream=None):
    """[..., nfft] float32 device rows -> [..., nfft/2+1] (vv_dsp_spectrogram_pack_half_device)."""
    if rows.shape[-1] != nfft:
        raise VvError(f"pack_half: rows of {rows.shape[-1]} bins, expected {nfft}")
    nrows = rows.numel() // nfft
    if out is None:
        out = torch.empty(tuple(rows.shape[:-1]) + (nfft // 2 + 1,), dtype=torch.float32, device=rows.device)
    _expect(rows, torch.float32, nrows * nfft, "pack_half input")
    _expect(out, torch.float32, nrows * (nfft // 2 + 1), "pack_half output")
    _check(lib().vv_dsp_spectrogram_pack_half_device(_ptr(rows), nrows, nfft, _ptr(out), _stream(stream)),
           "spectrogram_pack_half_device")
    return out


def unpack_half(half, nfft, out=None, stream=None):
    """[..., nfft/2+1] -> [..., nfft], bin k > nfft/2 from bin nfft-k (vv_dsp_spectrogram_unpack_half_device)."""
    if half.shape[-1] != nfft // 2 + 1:
        raise VvError(f"unpack_half: rows of {half.shape[-1]} bins, expected {nfft // 2 + 1}")
    nrows = half.numel() // (nfft // 2 + 1)
    if out is None:
        out = torch.empty(tuple(half.shape[:-1]) + (nfft,), dtype=torch.float32, device=half.device)
    _expect(half, torch.float32, nrows * (nfft // 2 + 1), "unpack_half input")
    _expect(out, torch.float32, nrows * nfft, "unpack_half output")
    _check(lib().vv_dsp_spectrogram_unpack_half_device(_ptr(half), nrows, nfft, _ptr(out), _stream(stream)),
           "spectrogram_unpack_half_device")
    return out


def hilbert(x, stream=None):
    """x: (batch, N) or (N,) float32 device tensor -> complex64 analytic signal."""
    x2 = x if x.dim() == 2 else x.unsqueeze(0)
    b, n = x2.shape
    z = torch.empty((b, n), dtype=torch.complex64, device=x.device)
    _check(lib().vv_dsp_hilbert_analytic_device(_ptr(x2), n, b, _ptr(z), _stream(stream)), "hilbert_device")
    return z if x.dim() == 2 else z[0]


def instantaneous_phase(z, stream=None):
    """z: (batch, N) or (N,) complex64 analytic rows -> unwrapped phase float32 (hilbert.c:77-96)."""
    z2 = z if z.dim() == 2 else z.unsqueeze(0)
    b, n = z2.shape
    _expect(z2, torch.complex64, b * n, "instantaneous_phase input")
    p = torch.empty((b, n), dtype=torch.float32, device=z.device)
    _check(lib().vv_dsp_instantaneous_phase_device(_ptr(z2), n, b, _ptr(p), _stream(stream)),
           "instantaneous_phase_device")
    return p if z.dim() == 2 else p[0]


def instantaneous_frequency(phase, sample_rate, stream=None):
    """phase: (batch, N) or (N,) float32 -> frequency in Hz, element 0 of a row = 0 (hilbert.c:98-113)."""
    p2 = phase if phase.dim() == 2 else phase.unsqueeze(0)
    b, n = p2.shape
    _expect(p2, torch.float32, b * n, "instantaneous_frequency input")
    f = torch.empty_like(p2)
    _check(lib().vv_dsp_instantaneous_frequency_device(_ptr(p2), n, b, float(sample_rate), _ptr(f),
                                                       _stream(stream)), "instantaneous_frequency_device")
    return f if phase.dim() == 2 else f[0]


def dct(x, dct_type=2, inverse=False, stream=None):
    x2 = x if x.dim() == 2 else x.unsqueeze(0)
    b, n = x2.shape
    p = _vp()
    _check(lib().vv_dsp_dct_make_plan(n, dct_type, -1 if inverse else 1, C.byref(p)), "dct_make_plan")
    try:
        y = torch.empty_like(x2)
        _check(lib().vv_dsp_dct_execute_device(p, _ptr(x2), _ptr(y), b, _stream(stream)), "dct_execute_device")
    finally:
        lib().vv_dsp_dct_destroy(p)
    return y if x.dim() == 2 else y[0]


class CztPlan:
    """Chirp-z transform of `batch` rows (vv_dsp_czt_exec_cpx / _real semantics,
    czt.c:44-178): X[k] = sum_n x[n] A^-n W^(nk), k < m.  x: (batch, n) or (n,)
    complex64 or float32 device tensor -> complex64 (batch, m)."""

    def __init__(self, n, m, w, a=1.0 + 0j):
        self.n, self.m = n, m
        self.h = _vp()
        w, a = complex(w), complex(a)
        _check(lib().vv_dsp_czt_plan_create(n, m, w.real, w.imag, a.real, a.imag, C.byref(self.h)),
               "czt_plan_create")

    def __call__(self, x, out=None, stream=None):
        x2 = x if x.dim() == 2 else x.unsqueeze(0)
        b = x2.shape[0]
        real = not x2.is_complex()
        _expect(x2, torch.float32 if real else torch.complex64, b * self.n, "czt input")
        if x2.shape[1] != self.n:
            raise VvError(f"czt input: rows of {x2.shape[1]}, the plan's N is {self.n}")
        if out is None:
            out = torch.empty((b, self.m), dtype=torch.complex64, device=x.device)
        _expect(out, torch.complex64, b * self.m, "czt output")
        _check(lib().vv_dsp_czt_execute_device(self.h, _ptr(x2), 1 if real else 0, b, _ptr(out), _stream(stream)),
               "czt_execute_device")
        return out if x.dim() == 2 else out.view(-1)[:self.m]

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.vv_dsp_czt_plan_destroy(self.h)
            self.h = None


def _ceps_rows(fn, x, out_dtype, what, stream):
    x2 = x if x.dim() == 2 else x.unsqueeze(0)
    b, n = x2.shape
    _expect(x2, torch.float32, b * n, what + " input")
    y = torch.empty((b, n), dtype=out_dtype, device=x.device)
    _check(getattr(lib(), fn)(_ptr(x2), n, b, _ptr(y), _stream(stream)), fn)
    return y if x.dim() == 2 else y[0]


def cepstrum(x, stream=None):
    """real cepstrum of float32 rows (cepstrum.c:7-41): Re IFFT(log(|FFT x| + 1e-12))"""
    return _ceps_rows("vv_dsp_cepstrum_real_device", x, torch.float32, "cepstrum", stream)


def icepstrum_minphase(c, stream=None):
    """minimum-phase signal from cepstrum rows (cepstrum.c:43-78)"""
    return _ceps_rows("vv_dsp_icepstrum_minphase_device", c, torch.float32, "icepstrum_minphase", stream)


def minphase_from_cepstrum(c, stream=None):
    """minimum-phase spectrum (complex64, imaginary parts 0) from cepstrum rows (minphase.c:7-31)"""
    return _ceps_rows("vv_dsp_minphase_from_cepstrum_device", c, torch.complex64, "minphase_from_cepstrum", stream)


def _ptrs(xs):
    """per-local-rank pointer array (vv_dsp_dist.h): tensors, raw ints or None"""
    return (_vp * len(xs))(*[None if x is None else (x if isinstance(x, int) else x.data_ptr()) for x in xs])


def _streams(streams, n, devices=None):
    """per-slot hipStream_t array; default: each slot's device's current stream"""
    if streams is None:
        streams = [torch.cuda.current_stream(d) for d in devices] if devices is not None else \
            [torch.cuda.current_stream()] * n
    if len(streams) != n:
        raise VvError(f"{len(streams)} streams for {n} local ranks")
    return (_vp * n)(*[s if (s is None or isinstance(s, int)) else s.cuda_stream for s in streams])


class Dist:
    """Multi-GPU layout of the spectral path over RCCL (include/vv_dsp/vv_dsp_dist.h):
    Dist.all([0, 1, ...]) -- every rank in this process (ncclCommInitAll);
    Dist.from_comm(ptr)   -- one rank of a caller's ncclComm_t;
    Dist.rank(world, r, id, device) -- one rank per process (ncclCommInitRank;
                             id = Dist.unique_id() on rank 0, shared by the caller);
    Dist.loopback(world)  -- `world` ranks on one device, transfers as device copies.
    Per-rank list arguments have one element per local rank (slot); streams
    default to each slot's device's current stream."""

    def __init__(self, handle):
        self.h = handle
        self.slots = lib().vv_dsp_dist_local_ranks(self.h)
        self.devices = [self.rank_info(s)[2] for s in range(self.slots)]

    @staticmethod
    def unique_id():
        """VV_DSP_DIST_ID_BYTES (128) bytes naming a new communicator (ncclGetUniqueId)"""
        buf = C.create_string_buffer(128)
        _check(lib().vv_dsp_dist_unique_id(buf), "dist_unique_id")
        return buf.raw

    @classmethod
    def rank(cls, world, rank, uid, device):
        if len(uid) != 128:
            raise VvError("a communicator id is 128 bytes")
        h = _vp()
        _check(lib().vv_dsp_dist_init_rank(world, rank, bytes(uid), device, C.byref(h)), "dist_init_rank")
        return cls(h)

    def comm_count(self, slot=0):
        """ranks RCCL reports for slot's communicator (ncclCommCount)"""
        n = C.c_int()
        _check(lib().vv_dsp_dist_comm_count(self.h, slot, C.byref(n)), "dist_comm_count")
        return n.value

    @classmethod
    def all(cls, devices):
        h = _vp()
        arr = (C.c_int * len(devices))(*devices)
        _check(lib().vv_dsp_dist_init_all(len(devices), arr, C.byref(h)), "dist_init_all")
        return cls(h)

    @classmethod
    def loopback(cls, world, device=0):
        h = _vp()
        _check(lib().vv_dsp_dist_init_loopback(world, device, C.byref(h)), "dist_init_loopback")
        return cls(h)

    @classmethod
    def from_comm(cls, comm_ptr):
        h = _vp()
        _check(lib().vv_dsp_dist_from_comm(comm_ptr, C.byref(h)), "dist_from_comm")
        return cls(h)

    def rank_info(self, slot):
        r, w, d = C.c_int(), C.c_int(), C.c_int()
        _check(lib().vv_dsp_dist_rank_info(self.h, slot, C.byref(r), C.byref(w), C.byref(d)), "dist_rank_info")
        return r.value, w.value, d.value

    def stft(self, st, sigs, n, total_ch, ch_stride, rows, out_kind=0, streams=None):
        nf = _sz(0)
        _check(lib().vv_dsp_dist_stft(self.h, st.h, _ptrs(sigs), n, total_ch, ch_stride, out_kind, _ptrs(rows),
                                      _streams(streams, self.slots, self.devices), C.byref(nf)), "dist_stft")
        return nf.value

    def gather_rows(self, local, total_items, rows_per_item, row_floats, out, root=0, half=False, streams=None):
        """items (channels) of rows_per_item rows of row_floats floats; rank r's
        items from vv_dsp_shard_range(total_items, world, r)"""
        _check(lib().vv_dsp_dist_gather_rows(self.h, _ptrs(local), total_items, rows_per_item, row_floats,
                                             1 if half else 0,
                                             None if out is None else _ptr(out), root,
                                             _streams(streams, self.slots, self.devices)), "dist_gather_rows")

    def fft(self, n, kind, direction, total_batch, ins, outs, streams=None):
        _check(lib().vv_dsp_dist_fft(self.h, n, kind, direction, total_batch, _ptrs(ins), _ptrs(outs),
                                     _streams(streams, self.slots, self.devices)), "dist_fft")

    def fir(self, plans, n, total_ch, xs, x_stride, ys, y_stride, streams=None):
        arr = (_vp * len(plans))(*[p.h for p in plans])
        _check(lib().vv_dsp_dist_fir_apply_fft(self.h, arr, n, total_ch, _ptrs(xs), x_stride, _ptrs(ys), y_stride,
                                               _streams(streams, self.slots, self.devices)), "dist_fir_apply_fft")

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.vv_dsp_dist_destroy(self.h)
            self.h = None
