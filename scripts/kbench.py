#!/usr/bin/env python3
"""Kernel micro-benchmarks for iteration on the GPU box (not the driver bench).

Times each hot kernel with HIP events on the launch stream, interleaving
repetitions of all cases in one process (methodology rule 24), and prints
algorithmic GB/s and the fraction of the 8 TB/s HBM peak.

    python scripts/kbench.py [--reps 20] [--cases c2c1024,stft,fir,...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vv-dsp_amd"))
import vvdsp_amd as vv  # noqa: E402

PEAK = 8000.0


def case_c2c(n, batch, fwd=True):
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.complex(torch.rand(batch, n, device="cuda", generator=g) - 0.5,
                      torch.rand(batch, n, device="cuda", generator=g) - 0.5)
    y = torch.empty_like(x)
    p = vv.FftPlan(n, vv.C2C, vv.FWD if fwd else vv.BWD, batch=batch)
    return (lambda: p(x, out=y)), 2 * batch * n * 8, (x, y, p)


def case_r2c(n, batch, env=None):
    if env:
        inner = case_r2c(n, batch)
        fn = inner[0]

        def run():
            with vv.knobs(**{env[0].replace("VVHIP_", ""): int(env[1])}):
                fn()
        return (run,) + tuple(inner[1:])
    x = torch.rand(batch, n, device="cuda")
    y = torch.empty(batch, n // 2 + 1, dtype=torch.complex64, device="cuda")
    p = vv.FftPlan(n, vv.R2C, vv.FWD, batch=batch)
    return (lambda: p(x, out=y)), batch * n * 4 + batch * (n // 2 + 1) * 8, (x, y, p)


def case_c2r(n, batch):
    X = torch.complex(torch.rand(batch, n // 2 + 1, device="cuda"), torch.rand(batch, n // 2 + 1, device="cuda"))
    y = torch.empty(batch, n, device="cuda")
    p = vv.FftPlan(n, vv.C2R, vv.BWD, batch=batch)
    return (lambda: p(X, out=y)), batch * n * 4 + batch * (n // 2 + 1) * 8, (X, y, p)


def case_stft(nch, seconds, complex_out=False, env=None, shared=True):
    """the product STFT; `shared`: every such case of one shape uses the same
    buffers (same-placement A/B -- the placement of a fresh allocation alone moves
    the headline by up to 5 %, profiles/r03_kbench_placement.jsonl)"""
    if env:   # experiment switch read by the launcher at each call
        k, v = env
        inner = case_stft(nch, seconds, complex_out, shared=shared)
        fn = inner[0]

        def run():
            with vv.knobs(**{k.replace("VVHIP_", ""): int(v)}):
                fn()
        return (run,) + tuple(inner[1:])
    n = seconds * 48000
    st = vv.Stft(1024, 256)
    fr = st.frames(n)
    dt = torch.complex64 if complex_out else torch.float32
    key = ("stft", nch, n, complex_out)
    if shared and key in _SHARED:
        sig, out = _SHARED[key]
    else:
        sig = torch.rand(nch, n, device="cuda") * 2 - 1
        out = torch.empty(nch, fr, 1024, dtype=dt, device="cuda")
        if shared:
            _SHARED[key] = (sig, out)
    byts = nch * n * 4 + nch * fr * 1024 * (8 if complex_out else 4)
    return (lambda: st.spectrogram(sig, out=out, complex_out=complex_out)), byts, (sig, out, st)


def case_stft_place(in_kb, out_kb, nch=32, seconds=600):
    """the headline STFT with its input / output at a byte offset inside one
    shared pair of buffers (placement sensitivity of the same kernel)"""
    n = seconds * 48000
    st = vv.Stft(1024, 256)
    fr = st.frames(n)
    if "place" not in _SHARED:
        _SHARED["place"] = (torch.rand(nch * n + (8 << 20), device="cuda") * 2 - 1,
                            torch.empty(nch * fr * 1024 + (8 << 20), device="cuda"))
    a, b = _SHARED["place"]
    sig = a[in_kb * 256: in_kb * 256 + nch * n].view(nch, n)
    out = b[out_kb * 256: out_kb * 256 + nch * fr * 1024].view(nch, fr, 1024)
    byts = nch * n * 4 + nch * fr * 1024 * 4
    return (lambda: st.spectrogram(sig, out=out)), byts, (sig, out, st)


def case_stft_n(nch, seconds, nfft, hop, sr=16000):
    """magnitude rows at any nfft (non-power-of-two: frame gather + mixed-radix FFT + |X|)"""
    n = seconds * sr
    st = vv.Stft(nfft, hop)
    fr = st.frames(n)
    key = ("stftn", nch, n, nfft, hop)
    if key not in _SHARED:   # shared by the A/B cases of one shape (same placement)
        _SHARED[key] = (torch.rand(nch, n, device="cuda") * 2 - 1, torch.empty(nch, fr, nfft, device="cuda"))
    sig, out = _SHARED[key]
    return (lambda: st.spectrogram(sig, out=out)), nch * n * 4 + nch * fr * nfft * 4, (sig, out, st)


def case_stft_pow_n(nch, seconds, nfft, hop, sr=16000):
    """power rows [ch][frame][nfft/2+1] at any nfft (register kernel MODE 3 at the speech lengths)"""
    n = seconds * sr
    st = vv.Stft(nfft, hop)
    fr = st.frames(n)
    key = ("stftpown", nch, n, nfft, hop)
    if key not in _SHARED:
        _SHARED[key] = (torch.rand(nch, n, device="cuda") * 2 - 1, torch.empty(nch, fr, nfft // 2 + 1, device="cuda"))
    sig, out = _SHARED[key]
    return (lambda: st.power(sig, out=out)), nch * n * 4 + nch * fr * (nfft // 2 + 1) * 4, (sig, out, st)


def case_stft_mel(log_mel, nch=32, seconds=600, n_mels=40, n_coeffs=13):
    """signal -> log-mel / MFCC rows (vv_dsp_stft_log_mel_device / _mfcc_device; the
    power rows stay in LDS); bytes = signal in + rows out"""
    n = seconds * 48000
    st = vv.Stft(1024, 256)
    fr = st.frames(n)
    mf = vv.Mfcc(1024, n_mels, n_coeffs, 48000.0, 20.0, 20000.0, lifter=22.0)
    width = n_mels if log_mel else n_coeffs
    if ("melsig", nch, n) not in _SHARED:
        _SHARED[("melsig", nch, n)] = torch.rand(nch, n, device="cuda") * 2 - 1
    sig = _SHARED[("melsig", nch, n)]
    out = torch.empty(nch, fr, width, device="cuda")
    return (lambda: mf.from_signal(st, sig, log_mel=log_mel, out=out)), nch * n * 4 + nch * fr * width * 4, \
        (sig, out, st, mf)


def case_stft_power(nch, seconds):
    """power rows [ch][frame][513] (STFT mode 2, the mel kernel's input)"""
    n = seconds * 48000
    st = vv.Stft(1024, 256)
    fr = st.frames(n)
    if ("pow", nch, n) not in _SHARED:   # shared by the A/B cases (same placement)
        _SHARED[("pow", nch, n)] = (torch.rand(nch, n, device="cuda") * 2 - 1, torch.empty(nch, fr, 513, device="cuda"))
    sig, out = _SHARED[("pow", nch, n)]
    return (lambda: st.power(sig, out=out)), nch * n * 4 + nch * fr * 513 * 4, (sig, out, st)


def lowpass(taps=257, fc=0.25):
    """config 4's filter: vv_dsp_fir_design_lowpass(h, taps, fc, HANNING) by the library's
    host setup (fir.c:47-73 arithmetic).  The data matter for timing: a compute-bound kernel
    clocks differently on smooth (e.g. a bare Hann window's) spectra."""
    import ctypes
    L = vv.lib()
    L.vv_dsp_fir_design_lowpass.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_float, ctypes.c_int]
    h = np.zeros(taps, np.float32)
    assert L.vv_dsp_fir_design_lowpass(h.ctypes.data, taps, fc, 2) == 0
    return torch.from_numpy(h)


def case_fir(nch, n, taps=257):
    h = lowpass(taps)
    if ("fir", nch, n) not in _SHARED:   # shared by the A/B cases (same placement)
        _SHARED[("fir", nch, n)] = (torch.rand(nch, n, device="cuda") * 2 - 1, torch.empty(nch, n, device="cuda"))
    x, y = _SHARED[("fir", nch, n)]
    p = vv.FirPlan(h)
    return (lambda: p(x, out=y)), 2 * nch * n * 4, (x, y, p)


def case_fir_direct(nch, n, taps=257, filtfilt=False):
    """bit-exact direct form (vv_dsp_fir_apply / vv_dsp_filtfilt_fir): bytes = one read + one write"""
    h = lowpass(taps)
    x = torch.rand(nch, n, device="cuda") * 2 - 1
    y = torch.empty_like(x)
    p = vv.FirPlan(h)
    fn = (lambda: p.filtfilt(x, out=y)) if filtfilt else (lambda: p(x, out=y, direct=True))
    return fn, 2 * nch * n * 4, (x, y, p)


def case_mel(kind, frames=3599936):
    """log-mel (kind 0) / MFCC (kind 1) from power rows [frames][513] (40 mels, 13 coeffs)"""
    if "pw513" not in _SHARED:
        _SHARED["pw513"] = torch.rand(frames, 513, device="cuda") ** 2
    pw = _SHARED["pw513"]
    mf = vv.Mfcc(1024, 40, 13, 48000.0, 20.0, 20000.0, lifter=22.0)
    if kind == 0:
        return (lambda: mf.log_mel(pw)), frames * (513 + 40) * 4, (pw, mf)
    return (lambda: mf(pw)), frames * (513 + 13) * 4, (pw, mf)


def case_ola(seconds=600):
    """ISTFT overlap-add of one channel's complex frames (vv_dsp_stft_reconstruct, batched)"""
    st = vv.Stft(1024, 256)
    n = seconds * 48000
    fr = st.frames(n)
    spec = torch.complex(torch.rand(fr, 1024, device="cuda"), torch.rand(fr, 1024, device="cuda"))
    acc = torch.zeros(n + 1024, device="cuda")
    norm = torch.zeros(n + 1024, device="cuda")
    return (lambda: st.reconstruct(spec, acc, norm)), fr * 8192 + 2 * 2 * (n + 1024) * 4, (st, spec, acc, norm)


def case_hilbert(n, batch):
    x = torch.rand(batch, n, device="cuda") * 2 - 1
    vv.hilbert(x)   # plan/tables
    return (lambda: vv.hilbert(x)), batch * n * 12, (x,)


def case_dct(n, batch):
    x = torch.rand(batch, n, device="cuda") * 2 - 1
    vv.dct(x)
    return (lambda: vv.dct(x)), batch * n * 8, (x,)


def case_czt(n, m, batch):
    """batched chirp-z (czt.c:44-178) at a zoom arc; bytes = rows in + outputs"""
    import numpy as np
    x = torch.complex(torch.rand(batch, n, device="cuda") - 0.5, torch.rand(batch, n, device="cuda") - 0.5)
    p = vv.CztPlan(n, m, np.exp(-2j * np.pi * 0.05 / m), np.exp(0.3j))
    y = torch.empty(batch, m, dtype=torch.complex64, device="cuda")
    return (lambda: p(x, out=y)), batch * 8 * (n + m), (x, y, p)


def case_cepstrum(n, batch, kind=0):
    x = torch.rand(batch, n, device="cuda") * 2 - 1
    f = (vv.cepstrum, vv.icepstrum_minphase)[kind]
    return (lambda: f(x)), batch * n * 8, (x,)


def case_copy(nbytes):
    a = torch.empty(nbytes // 4, device="cuda")
    b = torch.empty_like(a)
    return (lambda: b.copy_(a)), 2 * nbytes, (a, b)


def case_wr(mode, nt, rows=3600000, blocks=2048):
    """store-pattern microbenchmark (scripts/membench.hip): rows x 4 KB"""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libmembench.so"))
    lib.membench_write.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_void_p]
    out = torch.empty(rows, 1024, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    return (lambda: lib.membench_write(out.data_ptr(), rows, mode, nt, blocks, s)), rows * 4096, (out, lib)


def case_wprobe(w, pol, band, rd, blocks=2048, items=3599936):
    """write-ceiling probe (membench.hip k_wprobe): items x 4 KB written (the
    headline's 14.7 GB of rows), + 1 KB read per item with rd; one buffer pair
    shared by every probe case (same placement)"""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libmembench.so"))
    lib.membench_wprobe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong] + [ctypes.c_int] * 5 + \
        [ctypes.c_void_p]
    if ("wprobe", items) not in _SHARED:
        _SHARED[("wprobe", items)] = (torch.rand(items * 256, device="cuda"), torch.empty(items * 1024, device="cuda"))
    a, b = _SHARED[("wprobe", items)]
    s = torch.cuda.current_stream().cuda_stream
    f = (lambda: lib.membench_wprobe(a.data_ptr(), b.data_ptr(), items, w, pol, band, rd, blocks, s))
    assert f() == 0
    return f, items * 4096 + (items * 1024 if rd else 0), (a, b, lib)


def case_stft_exp(e, nch=32, seconds=600):
    """STFT kernel with parts switched off (scripts/membench.hip k_stft_exp)"""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libmembench.so"))
    lib.membench_stft_exp.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_longlong,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    n = seconds * 48000
    sig = torch.rand(nch, n, device="cuda") * 2 - 1
    win = torch.hann_window(1024, periodic=False, device="cuda")
    fr = (n - 1024) // 256 + 1
    out = torch.empty(nch, fr, 1024, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    byts = nch * n * 4 + nch * fr * 1024 * 4
    return (lambda: lib.membench_stft_exp(sig.data_ptr(), n, nch, 256, win.data_ptr(), out.data_ptr(), e, s)), \
        byts, (sig, win, out, lib)


def case_empty(grid):
    """an empty kernel of grid x 256 threads (scripts/stftlab.hip emptylab_run): launch +
    kernel-boundary floor; bytes = config 3's, for a comparable frac column"""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libstftlab.so"))
    lib.emptylab_run.argtypes = [ctypes.c_int, ctypes.c_void_p]
    s = torch.cuda.current_stream().cuda_stream
    return (lambda: lib.emptylab_run(grid, s)), 57591808, (lib,)


def case_firlab(e, nch=8, n=1 << 24, fn="firlab_run"):
    """k_fir_bulk (config 4's bulk pairs) with parts switched off (scripts/stftlab.hip firlab_run,
    EXP bits: 1 no FFT exchanges, 2 no FFTs, 4 no stores, 8 no span loads); H = a unit impulse's spectrum"""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libstftlab.so"))
    run = getattr(lib, fn)
    run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong,
                               ctypes.c_longlong, ctypes.c_void_p]
    if ("firlab", nch, n) not in _SHARED:   # one buffer set for every FIR lab case (same placement)
        hp = torch.zeros(1024)
        hp[:257] = lowpass(257)
        _SHARED[("firlab", nch, n)] = (torch.rand(nch, n, device="cuda") * 2 - 1, torch.empty(nch, n, device="cuda"),
                                       (torch.fft.fft(hp.double()) / 1024).to(torch.complex64).cuda())
    x, y, H = _SHARED[("firlab", nch, n)]   # H: config 4's spectrum
    s = torch.cuda.current_stream().cuda_stream
    return (lambda: run(e, H.data_ptr(), x.data_ptr(), y.data_ptr(), n, nch, s)), 2 * nch * n * 4, \
        (x, y, H, lib)


def case_c2clab(e, batch=65536, fn="c2cr32lab_run"):
    """the lab's k_c2c_r32 (scripts/stftlab.hip c2cr32lab_run; EXP 2 no FFT)"""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libstftlab.so"))
    run = getattr(lib, fn)
    run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]
    if ("c2clab", batch) not in _SHARED:   # one buffer pair for every c2c lab case (same placement)
        x = torch.rand(batch, 1024, dtype=torch.complex64, device="cuda")
        _SHARED[("c2clab", batch)] = (x, torch.empty_like(x))
    x, y = _SHARED[("c2clab", batch)]
    s = torch.cuda.current_stream().cuda_stream
    return (lambda: run(e, x.data_ptr(), y.data_ptr(), batch, s)), 2 * batch * 1024 * 8, (x, y, lib)


def case_rw(w, in_bytes=3686400000, blocks=4096):
    """streaming read 1 : write w (scripts/membench.hip k_rw), 16 B/lane, nt"""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libmembench.so"))
    lib.membench_rw.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                                ctypes.c_void_p]
    n4 = in_bytes // 16
    a = torch.empty(n4 * 4, device="cuda")
    b = torch.empty(n4 * 4 * w, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    return (lambda: lib.membench_rw(a.data_ptr(), b.data_ptr(), n4, w, blocks, s)), in_bytes * (1 + w), (a, b, lib)


_SHARED = {}


def case_rwc(w, u, ntl, nts, blocks, in_bytes=3686400000):
    """contiguous mixed stream (membench.hip k_rwc): 1 KB read -> w KB written per wave item"""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libmembench.so"))
    lib.membench_rwc.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong] + [ctypes.c_int] * 5 + \
        [ctypes.c_void_p]
    items = in_bytes // 1024
    if ("rwc", w) not in _SHARED:   # one buffer pair per write ratio, shared by all rwc cases
        _SHARED[("rwc", w)] = (torch.empty(items * 256, device="cuda"), torch.empty(items * 256 * w, device="cuda"))
    a, b = _SHARED[("rwc", w)]
    s = torch.cuda.current_stream().cuda_stream
    f = (lambda: lib.membench_rwc(a.data_ptr(), b.data_ptr(), items, w, u, ntl, nts, blocks, s))
    assert f() == 0
    return f, in_bytes * (1 + w), (a, b, lib)


def case_model(depth, work, lds_bytes, walk=0, ld=0, pairs=1799968):
    """STFT memory-pipeline model (membench.hip k_model): LDS-DMA spans DEPTH pairs
    ahead, WORK x 16 packed FMAs, 8 x 1 KB nt stores per pair; LDS pad sets occupancy"""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libmembench.so"))
    lib.membench_model.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_longlong,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    if "model" not in _SHARED:
        _SHARED["model"] = (torch.empty(pairs * 512 + 4096, device="cuda"), torch.empty(pairs * 2048, device="cuda"))
    a, b = _SHARED["model"]
    s = torch.cuda.current_stream().cuda_stream
    f = (lambda: lib.membench_model(a.data_ptr(), b.data_ptr(), pairs, 256, depth, work, lds_bytes, walk, ld, s))
    assert f() == 0
    return f, pairs * 10240, (a, b, lib)


def with_env(case, key, val):
    """run a case with a launcher knob (csrc/hip/debug.hip, vvhip_debug_set) set
    around each call; `key` is the knob's VVHIP_* name"""
    def make():
        inner = case()
        fn = inner[0]
        name = key[6:] if key.startswith("VVHIP_") else key

        def run():
            vv.debug_set(name, int(val))
            fn()
            vv.debug_clear(name)
        return (run,) + tuple(inner[1:])
    return make


CASES = {
    **{f"model_d{d}w{w}l{l}k{k}": (lambda d=d, w=w, l=l, k=k: case_model(d, w, l * 1024, k))
       for d in (1, 2, 3) for w in (0, 12, 25) for l in (66, 50, 40, 32, 20) for k in (0, 1, 2, 3, 4)},
    **{f"model_ld{ld}w{w}l{l}": (lambda ld=ld, w=w, l=l: case_model(1, w, l * 1024, 1, ld))
       for ld in (1, 2) for w in (0, 12) for l in (66, 40, 20)},
    **{f"model4_ld{ld}w{w}": (lambda ld=ld, w=w: case_model(1, w, 50 * 1024, 4, ld + 10))
       for ld in (0, 1, 2) for w in (0, 12)},
    **{f"rwc{w}u{u}l{l}s{s_}b{b}": (lambda w=w, u=u, l=l, s_=s_, b=b: case_rwc(w, u, l, s_, b))
       for (w, u, l, s_) in [(4, 1, 1, 1), (4, 2, 1, 1), (4, 4, 1, 1), (4, 1, 0, 0), (4, 2, 0, 0), (4, 4, 0, 0),
                             (4, 2, 0, 1), (4, 2, 1, 0), (1, 2, 1, 1), (1, 2, 0, 0), (4, 8, 1, 1)]
       for b in (1024, 2048, 4096, 8192, 16384, 32768, 65536)},
    **{f"ex{e}": (lambda e=e: case_stft_exp(e)) for e in range(8)},
    "rw1": lambda: case_rw(1), "rw4": lambda: case_rw(4),
    **{f"rw{w}b{b}": (lambda w=w, b=b: case_rw(w, blocks=b)) for w in (1, 4) for b in (256, 512, 1024, 2048, 16384)},
    **{f"wp{w}p{p}b{b}r{r}": (lambda w=w, p=p, b=b, r=r: case_wprobe(w, p, b, r))
       for w in (1, 4) for p in (0, 1, 2, 3) for b in (0, 1, 2) for r in (0, 1)},
    **{f"wp{w}p{p}b{b}r{r}g{g}": (lambda w=w, p=p, b=b, r=r, g=g: case_wprobe(w, p, b, r, blocks=g))
       for w in (1, 4) for p in (0, 1) for b in (0, 1, 2) for r in (0, 1) for g in (1024, 4096, 16384)},
    "wr4": lambda: case_wr(0, 0), "wr4nt": lambda: case_wr(0, 1),
    "wrpat": lambda: case_wr(1, 0), "wrpatnt": lambda: case_wr(1, 1),
    "wr8nt": lambda: case_wr(2, 1), "wr16": lambda: case_wr(3, 0), "wr16nt": lambda: case_wr(3, 1),
    "copy1G": lambda: case_copy(1 << 29),
    # the config-2 byte count (512 MiB read + 512 MiB written) as a pure 1:1 stream
    **{f"rwc1G_u{u}b{b}": (lambda u=u, b=b: case_rwc(1, u, 1, 1, b, in_bytes=1 << 29))
       for u in (1, 2, 4) for b in (1024, 2048, 4096, 8192, 16384)},
    "c2c1024": lambda: case_c2c(1024, 65536),
    # large power-of-two (four-step) and Bluestein lengths; VVHIP_FS_* select the variant
    "c2c2p20": lambda: case_c2c(1 << 20, 64),
    "c2c2p20old": with_env(lambda: case_c2c(1 << 20, 64), "VVHIP_FS_OLD", "1"),
    **{f"c2c2p20v{v}": with_env(lambda: case_c2c(1 << 20, 64), "VVHIP_FS_VAR", str(v)) for v in (1, 2, 3)},
    **{f"c2c2p17v{v}": with_env(lambda: case_c2c(1 << 17, 512), "VVHIP_FS_VAR", str(v)) for v in (1, 2, 3)},
    **{f"c2c2p20ch{c}": with_env(lambda: case_c2c(1 << 20, 64), "VVHIP_FS_CHUNK_MB", str(c)) for c in (0, 16, 32, 128)},
    "c2c2p17": lambda: case_c2c(1 << 17, 512),
    "c2c2p17old": with_env(lambda: case_c2c(1 << 17, 512), "VVHIP_FS_OLD", "1"),
    "c2c2p13": lambda: case_c2c(1 << 13, 8192),
    "c2c2p13fs": with_env(lambda: case_c2c(1 << 13, 8192), "VVHIP_C2C_MAX", "4096"),
    "c2c2p13b": lambda: case_c2c(1 << 13, 8192, fwd=False),
    "r2c2p14": lambda: case_r2c(1 << 14, 4096),
    "r2c2p14fs": with_env(lambda: case_r2c(1 << 14, 4096), "VVHIP_C2C_MAX", "4096"),
    "c2r2p14": lambda: case_c2r(1 << 14, 4096),
    "r2c2p16": lambda: case_r2c(1 << 16, 1024),
    "r2c2p16old": with_env(lambda: case_r2c(1 << 16, 1024), "VVHIP_REAL_PROMOTE", "1"),
    "c2r2p16": lambda: case_c2r(1 << 16, 1024),
    "c2r2p16old": with_env(lambda: case_c2r(1 << 16, 1024), "VVHIP_REAL_PROMOTE", "1"),
    "c2c2p22": lambda: case_c2c(1 << 22, 16),
    "blue48000": lambda: case_c2c(48000, 1024),
    "blue48000nomix": with_env(lambda: case_c2c(48000, 1024), "VVHIP_NO_MIXED", "1"),
    "mix44100": lambda: case_c2c(44100, 1024),
    "mix192000": lambda: case_c2c(192000, 256),
    "mix96000": lambda: case_c2c(96000, 512),
    "blue48000unf": with_env(lambda: case_c2c(48000, 1024), "VVHIP_BLUE_UNFUSED", "1"),
    "blue48000old": with_env(lambda: case_c2c(48000, 1024), "VVHIP_FS_OLD", "1"),
    "c2c1024b": lambda: case_c2c(1024, 65536, fwd=False),
    **{f"c2cr32lab{e}": (lambda e=e: case_c2clab(e, fn="c2cr32lab_run")) for e in (0, 2)},
    # mixed-radix (7-smooth non-power-of-two) lengths; *nomix: the f64 DFT kernel / Bluestein
    **{f"mix{n}": (lambda n=n: case_c2c(n, (1 << 26) // n)) for n in (400, 480, 1000, 2000, 3000, 4000)},
    **{f"mix{n}nomix": with_env(lambda n=n: case_c2c(n, (1 << 22) // n), "VVHIP_NO_MIXED", "1") for n in (400, 3000)},
    "stft400": lambda: case_stft_n(32, 600, 400, 160),
    "stftp128": lambda: case_stft_n(8, 600, 128, 32, sr=48000),
    "stftp256": lambda: case_stft_n(8, 600, 256, 64, sr=48000),
    "stftp512": lambda: case_stft_n(8, 600, 512, 128, sr=48000),
    "stftp2048": lambda: case_stft_n(8, 600, 2048, 512, sr=48000),
    "stftp4096": lambda: case_stft_n(8, 600, 4096, 1024, sr=48000),
    "stftp8192": lambda: case_stft_n(8, 600, 8192, 2048, sr=48000),
    **{f"sqpow{nf}": (lambda nf=nf: case_stft_pow_n(32, 600, nf, nf // 4, sr=48000)) for nf in (400, 480, 960)},
    "sqpow400k16": lambda: case_stft_pow_n(32, 600, 400, 160, sr=16000),
    # speech lengths at 48 kHz (hop = nfft / 4), and VVHIP_MIX_VAR=1 (the conjugate-symmetric row emit)
    **{f"sq{nf}": (lambda nf=nf: case_stft_n(32, 600, nf, nf // 4, sr=48000))
       for nf in (320, 400, 441, 480, 600, 640, 720, 800, 900, 960)},
    **{f"sq{nf}v{v}": with_env(lambda nf=nf: case_stft_n(32, 600, nf, nf // 4, sr=48000), "VVHIP_MIX_VAR", str(v))
       for nf in (320, 400, 441, 480, 600, 640, 720, 800, 900, 960) for v in (1, 3, 4, 5, 6)},
    **{f"r2cmix{n}": (lambda n=n: case_r2c(n, (1 << 27) // n)) for n in (400, 960, 1000)},
    **{f"r2cmix{n}gen": with_env(lambda n=n: case_r2c(n, (1 << 27) // n), "VVHIP_STFT_SQ", "0") for n in (400, 960)},
    **{f"r2cmix{n}full": with_env(lambda n=n: case_r2c(n, (1 << 27) // n), "VVHIP_MIX_R2C_FULL", "1") for n in (400, 1000)},
    "stft480": lambda: case_stft_n(32, 600, 480, 120, sr=48000),
    **{f"mix{n}gen": with_env(lambda n=n: case_c2c(n, (1 << 26) // n), "VVHIP_STFT_SQ", "0")
       for n in (320, 400, 441, 480, 600, 640, 720, 800, 900, 960)},
    **{f"mix{n}": (lambda n=n: case_c2c(n, (1 << 26) // n)) for n in (320, 441, 600, 640, 720, 800, 900)},
    "mix960": lambda: case_c2c(960, (1 << 26) // 960),
    "stft960": lambda: case_stft_n(32, 600, 960, 240, sr=48000),
    # *gen: the generic mixed-radix kernel instead of the two-pass register one
    **{f"stft{nf}gen": with_env(lambda nf=nf, h=h, sr=sr: case_stft_n(32, 600, nf, h, sr=sr), "VVHIP_STFT_SQ", "0")
       for nf, h, sr in ((400, 160, 16000), (480, 120, 48000), (960, 240, 48000))},
    "c2c4096": lambda: case_c2c(4096, 16384),
    "c2c256": lambda: case_c2c(256, 262144),
    "r2c1024": lambda: case_r2c(1024, 131072),
    "c2r1024": lambda: case_c2r(1024, 131072),
    "stft": lambda: case_stft(32, 600),
    "stft_b": lambda: case_stft(32, 600, shared=False), "stft_c": lambda: case_stft(32, 600, shared=False),
    "stft256ch": lambda: case_stft(256, 600),
    **{f"place_i{i}_o{o}": (lambda i=i, o=o: case_stft_place(i, o))
       for i in (0, 4, 64, 1024, 2052) for o in (0, 4, 8, 64, 1024, 2052, 4100)},
    **{f"firlab{e}": (lambda e=e: case_firlab(e)) for e in (0, 1, 2, 3, 4, 5, 6, 8, 10, 12, 14)},
    **{f"empty{g}": (lambda g=g: case_empty(g)) for g in (703, 2048)},
    **{f"stftcps{c}": with_env(lambda: case_stft(32, 600), "VVHIP_STFT_CPS", str(c)) for c in (1, 2, 4, 8)},
    "stftspan": with_env(lambda: case_stft(32, 600), "VVHIP_STFT_RING", "0"),
    "stftchunk": with_env(lambda: case_stft(32, 600), "VVHIP_STFT_DYN", "0"),
    "melsig": lambda: case_stft_mel(True), "mfccsig": lambda: case_stft_mel(False),
    "melsig2": with_env(lambda: case_stft_mel(True), "VVHIP_MEL_FUSED", "0"),
    "mfccsig2": with_env(lambda: case_stft_mel(False), "VVHIP_MEL_FUSED", "0"),
    "stftpowdyn": with_env(lambda: case_stft_power(32, 600), "VVHIP_STFT_DYN", "1"),
    "stftcdyn": with_env(lambda: case_stft(8, 600, complex_out=True), "VVHIP_STFT_DYN", "1"),
    # probe: dynamic runs of r pairs on a ring (VAR 5)
    **{f"stftdr{r}": with_env(with_env(lambda: case_stft(32, 600), "VVHIP_STFT_DYN", "2"), "VVHIP_STFT_RUN", str(r))
       for r in (1, 2, 3, 4, 8, 16)},
    **{f"stftdb{d}": with_env(lambda: case_stft(32, 600), "VVHIP_STFT_DBS", str(d)) for d in (2, 3, 4, 5, 6, 7, 8)},
    **{f"stftdb{d}r1": with_env(with_env(lambda: case_stft(32, 600), "VVHIP_STFT_DBS", str(d)), "VVHIP_STFT_RUN", "1")
       for d in (5, 6, 7)},
    **{f"stftpowdr{r}": with_env(with_env(lambda: case_stft_power(32, 600), "VVHIP_STFT_DYN", "2"),
                                 "VVHIP_STFT_RUN", str(r)) for r in (2, 4)},
    **{f"stftcdr{r}": with_env(with_env(lambda: case_stft(8, 600, complex_out=True), "VVHIP_STFT_DYN", "2"),
                               "VVHIP_STFT_RUN", str(r)) for r in (2, 4)},
    "stftchunk256ch": with_env(lambda: case_stft(256, 600), "VVHIP_STFT_DYN", "0"),
    **{f"stftdbs{d}": with_env(lambda: case_stft(32, 600), "VVHIP_STFT_DBS", str(d)) for d in (3, 4, 5, 7, 8)},
    "stftpowspan": with_env(lambda: case_stft_power(32, 600), "VVHIP_STFT_RING", "0"),
    "stftcspan": with_env(lambda: case_stft(8, 600, complex_out=True), "VVHIP_STFT_RING", "0"),
    "stft60span": with_env(lambda: case_stft(1, 60), "VVHIP_STFT_RING", "0"),
    **{f"stftrun{r}": with_env(lambda: case_stft(32, 600), "VVHIP_STFT_RUN", str(r)) for r in (1, 2, 4, 8, 16)},
    **{f"stftpowrun{r}": with_env(lambda: case_stft_power(32, 600), "VVHIP_STFT_RUN", str(r)) for r in (1, 2, 4, 8, 16)},
    "stft60": lambda: case_stft(1, 60),
    "stft60cps1": with_env(lambda: case_stft(1, 60), "VVHIP_STFT_CPS", "1"),
    "stft60ring": with_env(lambda: case_stft(1, 60), "VVHIP_STFT_RING", "1"),
    "stftpow": lambda: case_stft_power(32, 600),
    "stftpowr32": with_env(lambda: case_stft_power(32, 600), "VVHIP_POW_R32", "1"),
    "stftmagr32": with_env(lambda: case_stft(32, 600), "VVHIP_MAG_R32", "1"),
    "stftpowold": with_env(lambda: case_stft_power(32, 600), "VVHIP_POW_OLD", "1"),
    "stftc": lambda: case_stft(8, 600, complex_out=True),
    "stftcold": with_env(lambda: case_stft(8, 600, complex_out=True), "VVHIP_POW_OLD", "1"),
    "fir": lambda: case_fir(8, 1 << 24),
    "firdirect": lambda: case_fir_direct(8, 1 << 24),
    "firdirectlds": with_env(lambda: case_fir_direct(8, 1 << 24), "VVHIP_FIR_DIRECT_LDS", "1"),
    "filtfilt": lambda: case_fir_direct(8, 1 << 24, filtfilt=True),
    "filtfiltlds": with_env(lambda: case_fir_direct(8, 1 << 24, filtfilt=True), "VVHIP_FIR_DIRECT_LDS", "1"),
    "firstatic": with_env(lambda: case_fir(8, 1 << 24), "VVHIP_FIR_DYN", "0"),
    "firold": with_env(lambda: case_fir(8, 1 << 24), "VVHIP_FIR_OLD", "1"),
    "firr16": with_env(lambda: case_fir(8, 1 << 24), "VVHIP_FIR_R32", "0"),
    "hilbert1024": lambda: case_hilbert(1024, 65536),
    "logmel": lambda: case_mel(0), "mfcc": lambda: case_mel(1),
    "ola": lambda: case_ola(),
    "olaold": with_env(lambda: case_ola(), "VVHIP_ISTFT_OLD", "1"),
    "dct1024": lambda: case_dct(1024, 131072),
    "czt1000": lambda: case_czt(1000, 1000, 16384),
    "czt1000unf": with_env(lambda: case_czt(1000, 1000, 16384), "VVHIP_CZT_UNFUSED", "1"),
    "czt48000": lambda: case_czt(48000, 4096, 256),
    "ceps1024": lambda: case_cepstrum(1024, 65536),
    "iceps1024": lambda: case_cepstrum(1024, 65536, 1),
    "ceps1024unf": with_env(lambda: case_cepstrum(1024, 65536), "VVHIP_CEPS_UNFUSED", "1"),
    "iceps1024unf": with_env(lambda: case_cepstrum(1024, 65536, 1), "VVHIP_CEPS_UNFUSED", "1"),
}
# A/B switches for launcher experiments: CASES["stftX"] = with_env(CASES["stft"], "VVHIP_EXP_...", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--mark", action="store_true",
                    help="launch a tiny torch fill kernel before each case's runs (splits a rocprofv3 trace per case)")
    ap.add_argument("--cases", default=",".join(k for k in CASES if not k.startswith(("wr", "wp", "ex", "rw", "model", "firlab", "c2cr32lab"))))
    a = ap.parse_args()
    names = a.cases.split(",")
    built = {k: CASES[k]() for k in names}
    res = {k: [] for k in names}
    s = torch.cuda.current_stream()
    for _ in range(a.rounds):
        for k in names:
            fn, byts, _keep = built[k]
            if a.mark:
                torch.cuda.synchronize()
                torch.full((1,), float(names.index(k)), device="cuda")
                torch.cuda.synchronize()
            t0 = time.perf_counter()   # warm-up: >= 3 launches and >= 50 ms (the clock ramp)
            while True:
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                if time.perf_counter() - t0 >= 0.05:
                    break
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
            for e0, e1 in ev:
                e0.record(s)
                fn()
                e1.record(s)
            torch.cuda.synchronize()
            res[k] += [e0.elapsed_time(e1) for e0, e1 in ev]
    for k in names:
        byts = built[k][1]
        ms = np.array(res[k])
        gbs = byts / (np.median(ms) * 1e-3) / 1e9
        print(json.dumps({"case": k, "ms_median": round(float(np.median(ms)), 4), "ms_mean": round(float(ms.mean()), 4),
                          "ms_min": round(float(ms.min()), 4), "GBs": round(gbs, 1),
                          "frac": round(gbs / PEAK, 4), "bytes": byts}))


if __name__ == "__main__":
    main()
