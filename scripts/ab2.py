#!/usr/bin/env python3
"""Same-buffer A/B of library builds in ONE process (timing tool, not a test).

Each build (`--libs a.so,b.so,...`) is dlopen'ed on its own (RTLD_LOCAL: its own
kernels, caches and knobs) and every case runs through the C device API of
each build on the SAME device buffers, interleaved A, B, A, B ... per round, so
neither the placement of a fresh allocation (up to 5 % on the headline,
profiles/r03_kbench_placement.jsonl) nor the box separates the builds.  Time =
HIP events around each launch on the launch stream; prints one JSON line per
(case, build) with the median and its ratio to the first build.

    python scripts/ab2.py --libs scripts/ab/prev.so,vv-dsp_amd/lib/libvvdsp_amd.so --cases fir,stft
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 8000.0
vp, sz = C.c_void_p, C.c_size_t


class StftParams(C.Structure):
    _fields_ = [("fft_size", C.c_size_t), ("hop_size", C.c_size_t), ("window", C.c_int)]


def load(spec):
    """`path` or `path@KNOB=V+KNOB2=V2`: knobs set in that build (vvhip_debug_set);
    to compare knob settings of one build, pass copies of the .so under other names
    (one file is loaded once per process)"""
    path, _, knobs = spec.partition("@")
    L = C.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL | os.RTLD_NOW)
    L.vvhip_debug_set.argtypes = [C.c_char_p, C.c_longlong]
    for kv in filter(None, knobs.split("+")):
        k, v = kv.split("=")
        if L.vvhip_debug_set(k.encode(), int(v)) != 0:
            raise SystemExit(f"{path}: unknown knob {k}")
    L.vvhip_last_error.restype = C.c_char_p
    L.vv_dsp_fir_design_lowpass.argtypes = [vp, sz, C.c_float, C.c_int]
    L.vv_dsp_fir_plan_create.argtypes = [vp, sz, C.POINTER(vp)]
    L.vv_dsp_fir_apply_fft_device.argtypes = [vp, vp, vp, sz, sz, sz, sz, vp]
    L.vv_dsp_stft_create.argtypes = [C.POINTER(StftParams), C.POINTER(vp)]
    for f in ("spectrogram", "power"):
        getattr(L, f"vv_dsp_stft_{f}_device").argtypes = [vp, vp, sz, sz, sz, vp, sz, vp, C.POINTER(sz)]
    if hasattr(L, "vv_dsp_stft_power_pitched_device"):
        L.vv_dsp_stft_power_pitched_device.argtypes = [vp, vp, sz, sz, sz, vp, sz, sz, vp, C.POINTER(sz)]
    for f in ("log_mel", "mfcc"):
        getattr(L, f"vv_dsp_stft_{f}_device").argtypes = [vp, vp, vp, sz, sz, sz, vp, sz, vp, C.POINTER(sz)]
    L.vv_dsp_mfcc_init.argtypes = [sz, sz, sz, C.c_float, C.c_float, C.c_float, C.c_int, C.c_int, C.c_float,
                                   C.c_float, C.POINTER(vp)]
    L.vv_dsp_fft_make_plan_many.argtypes = [sz, C.c_int, C.c_int, sz, C.POINTER(vp)]
    L.vv_dsp_fft_execute_device.argtypes = [vp, vp, vp, vp]
    return L


def ok(L, st, what):
    if st != 0:
        raise RuntimeError(f"{what}: status {st}: {L.vvhip_last_error().decode()}")


_BUF = {}


def buf(key, make):
    if key not in _BUF:
        _BUF[key] = make()
    return _BUF[key]


def frames_of(n, nfft=1024, hop=256):
    return 1 if n < nfft else 1 + (n - nfft + hop) // hop


def case_fir(L, s, nch=8, n=1 << 24):
    x, y = buf(("fir", nch, n), lambda: (torch.rand(nch, n, device="cuda") * 2 - 1, torch.empty(nch, n, device="cuda")))
    h = np.zeros(257, np.float32)
    ok(L, L.vv_dsp_fir_design_lowpass(h.ctypes.data, 257, 0.25, 2), "design")
    p = vp()
    ok(L, L.vv_dsp_fir_plan_create(h.ctypes.data, 257, C.byref(p)), "fir plan")
    return (lambda: ok(L, L.vv_dsp_fir_apply_fft_device(p, x.data_ptr(), y.data_ptr(), n, nch, n, n, s), "fir")), \
        2 * nch * n * 4, (lambda: y.clone())


def _stft(L):
    h = vp()
    ok(L, L.vv_dsp_stft_create(C.byref(StftParams(1024, 256, 1)), C.byref(h)), "stft create")
    return h


def case_stft_nfft(L, s, nfft, hop, nch=32, seconds=600, sr=48000):
    """magnitude rows at any nfft (speech lengths: the mixed-radix register kernels)"""
    n = seconds * sr
    fr = frames_of(n, nfft, hop)
    sig, out = buf(("stftn", nfft, hop, nch, n), lambda: (torch.rand(nch, n, device="cuda") * 2 - 1,
                                                          torch.empty(nch, fr, nfft, device="cuda")))
    h = vp()
    ok(L, L.vv_dsp_stft_create(C.byref(StftParams(nfft, hop, 1)), C.byref(h)), "stft create")
    nf = sz()
    f = L.vv_dsp_stft_spectrogram_device
    return (lambda: ok(L, f(h, sig.data_ptr(), n, nch, n, out.data_ptr(), fr * nfft, s, C.byref(nf)), "stft")), \
        nch * n * 4 + nch * fr * nfft * 4, (lambda: out.clone())


def case_stft_cpx(L, s, nfft, hop, nch=8, seconds=120, sr=48000):
    """complex rows [ch][frame][nfft] (vv_dsp_stft_spectrum_device)"""
    n = seconds * sr
    fr = frames_of(n, nfft, hop)
    sig, out = buf(("stftc", nfft, hop, nch, n), lambda: (torch.rand(nch, n, device="cuda") * 2 - 1,
                                                          torch.empty(nch, fr, nfft, dtype=torch.complex64,
                                                                      device="cuda")))
    h = vp()
    ok(L, L.vv_dsp_stft_create(C.byref(StftParams(nfft, hop, 1)), C.byref(h)), "stft create")
    nf = sz()
    f = L.vv_dsp_stft_spectrum_device
    f.argtypes = [vp, vp, sz, sz, sz, vp, sz, vp, C.POINTER(sz)]
    return (lambda: ok(L, f(h, sig.data_ptr(), n, nch, n, out.data_ptr(), fr * nfft, s, C.byref(nf)), "stftc")), \
        nch * n * 4 + nch * fr * nfft * 8, (lambda: out.clone())


def case_stft_rows(L, s, kind, nch, seconds):
    """kind mag / pow (packed 513-float rows) / pow544 (rows 544 floats apart;
    bytes counted as the 513 floats written)"""
    n = seconds * 48000
    fr = frames_of(n)
    w = {"mag": 1024, "pow": 513, "pow544": 544}[kind]
    sig, out = buf(("stft", kind, nch, n), lambda: (torch.rand(nch, n, device="cuda") * 2 - 1,
                                                    torch.empty(nch, fr, w, device="cuda")))
    h = _stft(L)
    nf = sz()
    if kind == "pow544":
        f = L.vv_dsp_stft_power_pitched_device
        run = lambda: ok(L, f(h, sig.data_ptr(), n, nch, n, out.data_ptr(), fr * w, w, s, C.byref(nf)), "stft")  # noqa
        return run, nch * n * 4 + nch * fr * 513 * 4, (lambda: out[:, :, :513].clone())
    f = L.vv_dsp_stft_spectrogram_device if kind == "mag" else L.vv_dsp_stft_power_device
    return (lambda: ok(L, f(h, sig.data_ptr(), n, nch, n, out.data_ptr(), fr * w, s, C.byref(nf)), "stft")), \
        nch * n * 4 + nch * fr * w * 4, (lambda: out.clone())


def case_mel(L, s, mfcc, nch=32, seconds=600):
    n = seconds * 48000
    fr = frames_of(n)
    w = 13 if mfcc else 40
    sig, out = buf(("mel", mfcc, nch, n), lambda: (torch.rand(nch, n, device="cuda") * 2 - 1,
                                                   torch.empty(nch, fr, w, device="cuda")))
    h = _stft(L)
    m = vp()
    ok(L, L.vv_dsp_mfcc_init(1024, 40, 13, 48000.0, 20.0, 20000.0, 0, 2, 22.0, 1e-10, C.byref(m)), "mfcc init")
    f = L.vv_dsp_stft_mfcc_device if mfcc else L.vv_dsp_stft_log_mel_device
    nf = sz()
    return (lambda: ok(L, f(h, m, sig.data_ptr(), n, nch, n, out.data_ptr(), fr * w, s, C.byref(nf)), "mel")), \
        nch * n * 4 + nch * fr * w * 4, (lambda: out.clone())


def case_c2c(L, s, n=1024, batch=65536):
    x, y = buf(("c2c", n, batch), lambda: (torch.complex(torch.rand(batch, n, device="cuda") - 0.5,
                                                         torch.rand(batch, n, device="cuda") - 0.5),
                                           torch.empty(batch, n, dtype=torch.complex64, device="cuda")))
    p = vp()
    ok(L, L.vv_dsp_fft_make_plan_many(n, 0, 1, batch, C.byref(p)), "fft plan")
    return (lambda: ok(L, L.vv_dsp_fft_execute_device(p, x.data_ptr(), y.data_ptr(), s), "fft")), \
        2 * batch * n * 8, (lambda: y.clone())


def case_real(L, s, n, batch, kind):
    """batched R2C (kind 1: real[n] -> cpx[n/2+1]) or C2R (kind 2, 1/n scaled)"""
    h = n // 2 + 1
    if kind == 1:
        x, y = buf(("r2c", n, batch), lambda: (torch.rand(batch, n, device="cuda") - 0.5,
                                               torch.empty(batch, h, dtype=torch.complex64, device="cuda")))
    else:
        x, y = buf(("c2r", n, batch), lambda: (torch.complex(torch.rand(batch, h, device="cuda") - 0.5,
                                                             torch.rand(batch, h, device="cuda") - 0.5),
                                               torch.empty(batch, n, device="cuda")))
    p = vp()
    ok(L, L.vv_dsp_fft_make_plan_many(n, kind, 1 if kind == 1 else -1, batch, C.byref(p)), "fft plan")
    return (lambda: ok(L, L.vv_dsp_fft_execute_device(p, x.data_ptr(), y.data_ptr(), s), "fft")), \
        batch * (n * 4 + h * 8), (lambda: y.clone())


def case_hilbert(L, s, n=1024, batch=65536):
    """batched Hilbert analytic rows real[batch][n] -> cpx[batch][n] (12 B per point)"""
    x, z = buf(("hil", n, batch), lambda: (torch.rand(batch, n, device="cuda") - 0.5,
                                           torch.empty(batch, n, dtype=torch.complex64, device="cuda")))
    L.vv_dsp_hilbert_analytic_device.argtypes = [vp, sz, sz, vp, vp]
    return (lambda: ok(L, L.vv_dsp_hilbert_analytic_device(x.data_ptr(), n, batch, z.data_ptr(), s), "hilbert")), \
        batch * n * 12, (lambda: z.clone())


def case_dct(L, s, n=1024, batch=131072):
    """batched DCT-II forward rows (8 B per point)"""
    x, y = buf(("dct", n, batch), lambda: (torch.rand(batch, n, device="cuda") - 0.5,
                                           torch.empty(batch, n, device="cuda")))
    L.vv_dsp_dct_make_plan.argtypes = [sz, C.c_int, C.c_int, C.POINTER(vp)]
    L.vv_dsp_dct_execute_device.argtypes = [vp, vp, vp, sz, vp]
    p = vp()
    ok(L, L.vv_dsp_dct_make_plan(n, 2, 1, C.byref(p)), "dct plan")
    return (lambda: ok(L, L.vv_dsp_dct_execute_device(p, x.data_ptr(), y.data_ptr(), batch, s), "dct")), \
        batch * n * 8, (lambda: y.clone())


def burst(case, k):
    """k launches back to back per timed call (the per-launch time is ms / k)"""
    fn, byts, get = case

    def run():
        for _ in range(k):
            fn()
    return run, byts * k, get


CASES = {
    "fir": case_fir,
    "stft": lambda L, s: case_stft_rows(L, s, "mag", 32, 600),
    "stft60": lambda L, s: case_stft_rows(L, s, "mag", 1, 60),
    "stft256ch": lambda L, s: case_stft_rows(L, s, "mag", 256, 600),
    "stft60x10": lambda L, s: burst(case_stft_rows(L, s, "mag", 1, 60), 10),
    "stftpow": lambda L, s: case_stft_rows(L, s, "pow", 32, 600),
    "stftpow544": lambda L, s: case_stft_rows(L, s, "pow544", 32, 600),
    "logmel": lambda L, s: case_mel(L, s, False),
    "logmel8": lambda L, s: case_mel(L, s, False, nch=8),
    "mfcc": lambda L, s: case_mel(L, s, True),
    "c2c1024": case_c2c,
    **{f"c2c{n}": (lambda L, s, n=n: case_c2c(L, s, n, (1 << 26) // n)) for n in (16, 32, 64, 128, 256, 512, 2048, 4096, 8192)},
    **{f"r2c{n}": (lambda L, s, n=n: case_real(L, s, n, (1 << 27) // n, 1)) for n in (16, 32, 64, 128, 256, 400, 480, 960, 1024, 2048, 4096, 8192, 16384)},
    **{f"c2r{n}": (lambda L, s, n=n: case_real(L, s, n, (1 << 27) // n, 2)) for n in (16, 32, 64, 128, 256, 1024, 2048, 4096, 8192, 16384)},
    **{f"hilbert{n}": (lambda L, s, n=n: case_hilbert(L, s, n, (1 << 26) // n)) for n in (16, 32, 64, 128, 256, 1024, 2048, 4096, 8192)},
    **{f"dct{n}": (lambda L, s, n=n: case_dct(L, s, n, (1 << 27) // n)) for n in (16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 8192)},
    **{f"c2c{n}": (lambda L, s, n=n: case_c2c(L, s, n, (1 << 26) // n)) for n in (320, 400, 441, 480, 600, 640, 720, 800, 900, 960, 1000, 2000, 3000, 4000)},
    **{f"stft{n}": (lambda L, s, n=n: case_stft_nfft(L, s, n, n // 4)) for n in (64, 128, 256, 400, 480, 512, 960, 1024, 2048, 4096)},
    **{f"stftc{n}": (lambda L, s, n=n: case_stft_cpx(L, s, n, n // 4)) for n in (256, 512, 1024, 2048, 4096)},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--cases", required=True)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--check", action="store_true", help="also compare each build's output with the first's")
    a = ap.parse_args()
    libs = [load(p) for p in a.libs.split(",")]
    tags = [os.path.basename(p) for p in a.libs.split(",")]
    if len(set(p.partition("@")[0] for p in a.libs.split(","))) != len(tags):
        raise SystemExit("each build must be a distinct file (copy the .so to compare knob settings)")
    torch.cuda.init()
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    for case in a.cases.split(","):
        built = [CASES[case](L, sp) for L in libs]
        res = [[] for _ in libs]
        same = []
        if a.check:
            outs = []
            for fn, _, get in built:
                fn()
                torch.cuda.synchronize()
                outs.append(get())
            same = [bool(torch.equal(outs[0], o)) for o in outs]
            del outs
        for _ in range(a.rounds):
            for i, (fn, _, _) in enumerate(built):
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < 0.05:
                    for _ in range(3):
                        fn()
                    torch.cuda.synchronize()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
                for e0, e1 in ev:
                    e0.record(s)
                    fn()
                    e1.record(s)
                torch.cuda.synchronize()
                res[i] += [e0.elapsed_time(e1) for e0, e1 in ev]
        base = float(np.median(res[0]))
        for i, tag in enumerate(tags):
            med = float(np.median(res[i]))
            byts = built[i][1]
            line = {"case": case, "lib": tag, "ms_median": round(med, 4), "ms_min": round(float(np.min(res[i])), 4),
                    "frac": round(byts / (med * 1e-3) / 1e9 / PEAK, 4), "vs_first": round(med / base, 4)}
            if same:
                line["bit_identical_to_first"] = same[i]
            print(json.dumps(line), flush=True)
        del built
        _BUF.clear()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
