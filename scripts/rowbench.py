#!/usr/bin/env python3
"""Per-row measurement of SURVEY.md section 8 on one MI355X, with the
reference's own CPU path timed beside each row.

For every row of the hot-path scope (FFT C2C / R2C / C2R, large power-of-two
and Bluestein lengths, STFT magnitude / power / complex spectrum, ISTFT
overlap-add, DCT-II, Hilbert, FIR overlap-save and direct form, log-mel /
MFCC) this times the device-resident batched call with HIP events on the
launch stream (median of `--reps` after warm-up), reports algorithmic bytes,
GB/s and the fraction of the 8 TB/s HBM peak, and runs the same operation
through the reference sources compiled in the build container
(oracle/_ref/libvvref.so, one host thread, a bounded sample of ~0.3-2 s) to
report the reference's per-unit time.

    python scripts/rowbench.py [--reps 10] [--json profiles/r01_rows.json]
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
sys.path.insert(0, os.path.join(ROOT, "tests"))
import vvdsp_amd as vv  # noqa: E402
from vvapi import VvDsp, C2C, R2C, C2R, FWD, BWD  # noqa: E402

PEAK = 8000.0
REF_PATH = os.path.join(ROOT, "oracle", "_ref", "libvvref.so")


def gpu_time(fn, reps):
    for _ in range(3):
        fn()
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def cpu_time(fn, budget=1.0, max_calls=1000):
    """seconds per call of fn() on one host thread, over a bounded sample"""
    fn()
    t0 = time.perf_counter()
    calls = 0
    while calls < max_calls:
        fn()
        calls += 1
        if time.perf_counter() - t0 > budget:
            break
    return (time.perf_counter() - t0) / calls, calls


def row(name, ref_fn, units, ms, byts, unit_name, cpu=None, note=""):
    r = {"row": name, "workload": units[0], "gpu_ms": round(ms, 4), "bytes": byts,
         "GBs": round(byts / (ms * 1e-3) / 1e9, 1), "frac_of_8TBs": round(byts / (ms * 1e-3) / 1e9 / PEAK, 4),
         "gpu_units_per_s": round(units[1] / (ms * 1e-3), 1), "unit": unit_name, "section8": ref_fn}
    if cpu is not None:
        sec, calls, per = cpu
        r["ref_cpu_units_per_s_1thread"] = round(per / sec, 1)
        r["ref_cpu_sample"] = f"{calls} calls x {per} {unit_name}, {sec * 1e3:.3f} ms per call"
        r["gpu_over_ref_1thread"] = round(r["gpu_units_per_s"] / r["ref_cpu_units_per_s_1thread"], 1)
    if note:
        r["note"] = note
    print(json.dumps(r), flush=True)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    ref = VvDsp(REF_PATH) if os.path.exists(REF_PATH) else None
    rng = np.random.default_rng(0)
    out = []

    def cpu(fn, per, budget=1.0):
        if ref is None:
            return None
        sec, calls = cpu_time(fn, budget)
        return sec, calls, per

    # ---- a6: C2C 1024 (config 2) -------------------------------------------------
    B = 65536
    x = torch.complex(torch.rand(B, 1024, device="cuda") - 0.5, torch.rand(B, 1024, device="cuda") - 0.5)
    y = torch.empty_like(x)
    p = vv.FftPlan(1024, vv.C2C, vv.FWD, batch=B)
    ms = gpu_time(lambda: p(x, out=y), a.reps)
    xh = (rng.random(1024) + 1j * rng.random(1024)).astype(np.complex64)
    out.append(row("fft_c2c_1024", "a6 vv_dsp_fft_execute C2C", (f"{B} x 1024 c2c fwd", B), ms, 16 * 1024 * B,
                   "transforms", cpu(lambda: ref.fft(xh, C2C, FWD), 1)))
    del x, y, p

    # ---- a7/a8: R2C / C2R 1024 ---------------------------------------------------------
    B = 131072
    xr = torch.rand(B, 1024, device="cuda")
    X = torch.empty(B, 513, dtype=torch.complex64, device="cuda")
    p = vv.FftPlan(1024, vv.R2C, vv.FWD, batch=B)
    ms = gpu_time(lambda: p(xr, out=X), a.reps)
    xrh = rng.random(1024).astype(np.float32)
    out.append(row("fft_r2c_1024", "a7 vv_dsp_fft_execute R2C", (f"{B} x 1024 r2c", B), ms,
                   B * (4 * 1024 + 8 * 513), "transforms", cpu(lambda: ref.fft(xrh, R2C), 1)))
    pi = vv.FftPlan(1024, vv.C2R, vv.BWD, batch=B)
    ms = gpu_time(lambda: pi(X, out=xr), a.reps)
    Xh = np.fft.rfft(xrh).astype(np.complex64)
    out.append(row("fft_c2r_1024", "a8 vv_dsp_fft_execute C2R", (f"{B} x 1024 c2r", B), ms,
                   B * (4 * 1024 + 8 * 513), "transforms", cpu(lambda: ref.fft(Xh, C2R, BWD, n=1024), 1),
                   note="the reference's C2R is its O(n^2) DFT (fft_kiss.c:120-174)"))
    del xr, X, p, pi

    # ---- a6: large power of two (four-step) and Bluestein -----------------------------
    for n, B, label in ((1 << 20, 64, "fft_c2c_2^20"), (48000, 1024, "fft_c2c_48000_mixed_fourstep"),
                        (48001, 1024, "fft_c2c_48001_bluestein")):
        x = torch.complex(torch.rand(B, n, device="cuda") - 0.5, torch.rand(B, n, device="cuda") - 0.5)
        y = torch.empty_like(x)
        p = vv.FftPlan(n, vv.C2C, vv.FWD, batch=B)
        ms = gpu_time(lambda: p(x, out=y), a.reps)
        if n in (48000, 48001):
            # the reference's O(n^2) DFT needs minutes at n = 48000: time it at n = 4800 and scale by n^2
            xh = (rng.random(4800) + 1j * rng.random(4800)).astype(np.complex64)
            c = cpu(lambda: ref.fft(xh, C2C, FWD), 1, budget=2.0)
            c = None if c is None else (c[0] * 100.0, c[1], 1)
        else:
            xh = (rng.random(n) + 1j * rng.random(n)).astype(np.complex64)
            c = cpu(lambda: ref.fft(xh, C2C, FWD), 1, budget=2.0)
        out.append(row(label, "a6 vv_dsp_fft_execute C2C, n = " + str(n), (f"{B} x {n} c2c fwd", B), ms,
                       16 * n * B, "transforms", c,
                       note="algorithmic bytes = one read + one write; the kernel chain moves "
                            + ("5x that (3 transposes, 2 FFT passes)" if n == 1 << 20 else
                               "2x that (two mixed-radix passes, 200 x 240)" if n == 48000 else
                               "~5x that over the padded length (Bluestein)")
                            + "; the reference runs " + ("Kiss radix-2" if n == 1 << 20 else
                                                         "its O(n^2) DFT (timed at n = 4800, x100)")))
        del x, y, p

    # ---- a6/a7: 7-smooth non-power-of-two lengths (mixed radix) -------------------------
    for n in (400, 480, 1000, 3000):
        B = (1 << 26) // n
        x = torch.complex(torch.rand(B, n, device="cuda") - 0.5, torch.rand(B, n, device="cuda") - 0.5)
        y = torch.empty_like(x)
        p = vv.FftPlan(n, vv.C2C, vv.FWD, batch=B)
        ms = gpu_time(lambda: p(x, out=y), a.reps)
        xh = (rng.random(n) + 1j * rng.random(n)).astype(np.complex64)
        out.append(row(f"fft_c2c_{n}_mixed", f"a6 vv_dsp_fft_execute C2C, n = {n} (mixed radix)",
                       (f"{B} x {n} c2c fwd", B), ms, 16 * n * B, "transforms",
                       cpu(lambda: ref.fft(xh, C2C, FWD), 1, budget=1.0),
                       note="the reference runs its O(n^2) DFT (fft_kiss.c:76-92) for every non-power-of-two n"))
        del x, y, p
    torch.cuda.empty_cache()
    st4 = vv.Stft(400, 160)
    n = 600 * 16000
    sig = torch.rand(32, n, device="cuda") * 2 - 1
    fr = st4.frames(n)
    o = torch.empty(32, fr, 400, device="cuda")
    ms = gpu_time(lambda: st4.spectrogram(sig, out=o), a.reps)
    sh = rng.uniform(-1, 1, 60 * 16000).astype(np.float32)
    out.append(row("stft_mag_400_hop160_32ch", "a11 vv_dsp_stft_spectrogram, nfft 400 / hop 160 (mixed radix)",
                   ("32 ch x 600 s at 16 kHz", 32 * fr), ms, 32 * n * 4 + 32 * fr * 1600, "frames",
                   cpu(lambda: ref.spectrogram(sh, 400, 160), st4.frames(60 * 16000), budget=2.0)))
    del sig, o, st4
    torch.cuda.empty_cache()

    # ---- a9-a13: STFT magnitude / power / complex, ISTFT ------------------------------
    st = vv.Stft(1024, 256)
    for nch, sec, label in ((32, 600, "stft_mag_config5_shard"), (1, 60, "stft_mag_config3_60s")):
        n = sec * 48000
        sig = torch.rand(nch, n, device="cuda") * 2 - 1
        fr = st.frames(n)
        o = torch.empty(nch, fr, 1024, device="cuda")
        ms = gpu_time(lambda: st.spectrogram(sig, out=o), a.reps)
        sh = rng.uniform(-1, 1, 60 * 48000).astype(np.float32)
        out.append(row(label, "a11 vv_dsp_stft_spectrogram", (f"{nch} ch x {sec} s", nch * fr), ms,
                       nch * n * 4 + nch * fr * 4096, "frames",
                       cpu(lambda: ref.spectrogram(sh, 1024, 256), st.frames(60 * 48000), budget=2.0)))
        if nch == 32:
            pw = torch.empty(nch, fr, 513, device="cuda")
            ms = gpu_time(lambda: st.power(sig, out=pw), a.reps)
            out.append(row("stft_power_config5_shard", "f1 n/2+1 power spectrogram (mel input)",
                           (f"{nch} ch x {sec} s", nch * fr), ms, nch * n * 4 + nch * fr * 513 * 4, "frames"))
            # ---- f3: MFCC / log-mel from the power rows --------------------------------
            mf = vv.Mfcc(1024, 40, 13, 48000.0, 20.0, 20000.0, lifter=22.0)
            pw2 = pw.reshape(-1, 513)
            ms = gpu_time(lambda: mf(pw2), a.reps)
            ph = (rng.random((1000, 513)) ** 2).astype(np.float32)
            out.append(row("mfcc_from_power", "f3 vv_dsp_mfcc_process (40 mels, 13 coeffs, lifter 22)",
                           (f"{pw2.shape[0]} frames x 513 bins", pw2.shape[0]), ms,
                           pw2.shape[0] * (513 + 13) * 4, "frames",
                           cpu(lambda: ref.mfcc_pipeline(ph, 1024, 40, 13, 48000.0, 20.0, 20000.0, 22.0, 1e-10),
                               1000)))
            ms = gpu_time(lambda: mf.log_mel(pw2), a.reps)
            out.append(row("log_mel_from_power", "f3 vv_dsp_compute_log_mel_spectrogram (40 mels)",
                           (f"{pw2.shape[0]} frames x 513 bins", pw2.shape[0]), ms,
                           pw2.shape[0] * (513 + 40) * 4, "frames"))
            del pw, pw2, mf
        del sig, o
        torch.cuda.empty_cache()
    n = 600 * 48000
    sig = torch.rand(8, n, device="cuda") * 2 - 1
    fr = st.frames(n)
    oc = torch.empty(8, fr, 1024, dtype=torch.complex64, device="cuda")
    ms = gpu_time(lambda: st.spectrogram(sig, out=oc, complex_out=True), a.reps)
    out.append(row("stft_complex_8ch", "a10 vv_dsp_stft_process (batched, full complex spectrum)",
                   ("8 ch x 600 s", 8 * fr), ms, 8 * n * 4 + 8 * fr * 8192, "frames"))
    # ISTFT overlap-add of one channel's frames (a12 vv_dsp_stft_reconstruct, batched)
    spec = oc[0].contiguous()
    acc = torch.zeros(n + 1024, device="cuda")
    norm = torch.zeros(n + 1024, device="cuda")
    ms = gpu_time(lambda: st.reconstruct(spec, acc, norm), a.reps)
    out.append(row("istft_ola_600s", "a12 vv_dsp_stft_reconstruct (batched overlap-add)",
                   ("1 ch x 600 s", fr), ms, fr * 8192 + 2 * 2 * (n + 1024) * 4, "frames",
                   note="bytes: spectrum read once + output and window-norm accumulators read+written"))
    del sig, oc, spec, acc, norm
    torch.cuda.empty_cache()

    # ---- a15 / a16: DCT-II and Hilbert ------------------------------------------------
    B = 131072
    xd = torch.rand(B, 1024, device="cuda") * 2 - 1
    ms = gpu_time(lambda: vv.dct(xd), a.reps)
    xh = rng.standard_normal(1024).astype(np.float32)
    out.append(row("dct2_1024", "a15 vv_dsp_dct_forward DCT-II", (f"{B} x 1024", B), ms, 8 * 1024 * B,
                   "transforms", cpu(lambda: ref.dct(xh, 2, False), 1),
                   note="the reference's DCT is the O(n^2) sum (dct.c:21-30)"))
    del xd
    B = 65536
    xh_d = torch.rand(B, 1024, device="cuda") * 2 - 1
    ms = gpu_time(lambda: vv.hilbert(xh_d), a.reps)
    out.append(row("hilbert_1024", "a16 vv_dsp_hilbert_analytic", (f"{B} x 1024", B), ms, 12 * 1024 * B,
                   "transforms", cpu(lambda: ref.hilbert(xh), 1)))
    del xh_d
    torch.cuda.empty_cache()

    # ---- a17-a19: FIR (config 4) -------------------------------------------------------
    nch, n = 8, 1 << 24
    h = ref.fir_design_lowpass(257, 0.25, 2) if ref is not None else np.hanning(257).astype(np.float32)
    xf = torch.rand(nch, n, device="cuda") * 2 - 1
    yf = torch.empty_like(xf)
    fp = vv.FirPlan(torch.from_numpy(h))
    ms = gpu_time(lambda: fp(xf, out=yf), a.reps)
    xs = rng.standard_normal(65536).astype(np.float32)
    out.append(row("fir_ols_257_config4", "a18 vv_dsp_fir_apply_fft (overlap-save)", ("8 ch x 2^24", nch * n), ms,
                   8 * nch * n, "samples", cpu(lambda: ref.fir_apply(h, xs), 65536),
                   note="CPU column: the reference's direct vv_dsp_fir_apply on 65536 samples (its apply_fft "
                        "is one O(n^2)-C2R block)"))
    ms = gpu_time(lambda: fp(xf, out=yf, direct=True), max(2, a.reps // 4))
    out.append(row("fir_direct_257_config4", "a19 vv_dsp_fir_apply (direct form, bit-exact)",
                   ("8 ch x 2^24", nch * n), ms, 8 * nch * n, "samples", cpu(lambda: ref.fir_apply(h, xs), 65536),
                   note="VALU-bound: 257 multiply-adds per sample in the reference's order, no FMA (k_fir_reg)"))
    ms = gpu_time(lambda: fp.filtfilt(xf, out=yf), max(2, a.reps // 4))
    xs2 = xs[:16384]
    out.append(row("filtfilt_257_config4", "FIR caller vv_dsp_filtfilt_fir (common.c:23-80, bit-exact)",
                   ("8 ch x 2^24", nch * n), ms, 8 * nch * n, "samples",
                   cpu(lambda: ref.filtfilt(h, xs2), 16384),
                   note="two direct-form passes over the reflection-padded signal"))
    del xf, yf, fp

    # ---- f4 (CZT, czt.c:44-178) and the cepstrum family (8b callers) ---------------------
    for n, m, B, label in ((1000, 1000, 16384, "czt_1000x1000_zoom"), (48000, 4096, 256, "czt_48000x4096_zoom")):
        w, aa = np.exp(-2j * np.pi * 0.05 / m), np.exp(0.3j)
        xz = torch.complex(torch.rand(B, n, device="cuda") - 0.5, torch.rand(B, n, device="cuda") - 0.5)
        cz = vv.CztPlan(n, m, w, aa)
        yz = torch.empty(B, m, dtype=torch.complex64, device="cuda")
        ms = gpu_time(lambda: cz(xz, out=yz), a.reps)
        P = 1 << (n + m - 2).bit_length()
        xzh = (rng.random(n) + 1j * rng.random(n)).astype(np.complex64)
        out.append(row(label, f"f4 vv_dsp_czt_exec_cpx, N = {n}, M = {m} (P = {P})", (f"{B} rows", B), ms,
                       B * 8 * (n + m), "transforms", cpu(lambda: ref.czt(xzh, m, complex(w), complex(aa)), 1),
                       note="algorithmic bytes = rows in + outputs; the chain moves ~4 x 16 P per row (pre-multiply, "
                            "two P-point FFTs, product, post-multiply)"))
        del xz, yz, cz
    B = 65536
    xc = torch.rand(B, 1024, device="cuda") * 2 - 1
    ms = gpu_time(lambda: vv.cepstrum(xc), a.reps)
    xch = rng.standard_normal(1024).astype(np.float32)
    out.append(row("cepstrum_1024", "8b vv_dsp_cepstrum_real (R2C, log|X|, C2R)", (f"{B} x 1024", B), ms,
                   8 * 1024 * B, "transforms", cpu(lambda: ref.cepstrum(xch), 1),
                   note="the reference runs two C2C FFTs (Kiss radix-2 at n = 1024)"))
    ms = gpu_time(lambda: vv.icepstrum_minphase(xc), a.reps)
    out.append(row("icepstrum_minphase_1024", "8b vv_dsp_icepstrum_minphase", (f"{B} x 1024", B), ms,
                   8 * 1024 * B, "transforms", cpu(lambda: ref.icepstrum_minphase(0.05 * xch), 1)))
    del xc
    torch.cuda.empty_cache()

    # ---- host-buffer (PCIe-inclusive) rate of the reference's own host-pointer API ------
    # vv_dsp_stft_spectrogram / vv_dsp_fft_execute take host pointers: the library copies
    # H2D, runs the kernel and copies D2H on the handle's stream (two-lane pipeline).
    # Wall clock on the host thread, pageable numpy buffers as the reference's callers have.
    amd = VvDsp(os.path.join(ROOT, "vv-dsp_amd", "lib", "libvvdsp_amd.so"))
    import ctypes as C
    fp = C.POINTER(C.c_float)
    st_, h = amd.stft_create(1024, 256)
    for sec in (60, 600):
        x = rng.uniform(-1, 1, sec * 48000).astype(np.float32)
        fr = 1 + (x.size - 1024 + 256) // 256
        o = np.empty(fr * 1024, np.float32)
        nf = C.c_size_t(0)
        call = (lambda: amd.lib.vv_dsp_stft_spectrogram(h, x.ctypes.data_as(fp), x.size, o.ctypes.data_as(fp),
                                                         C.byref(nf)))
        assert call() == 0
        sec_per, calls = cpu_time(call, budget=1.5, max_calls=200)
        out.append(row(f"stft_mag_host_{sec}s", "a11 vv_dsp_stft_spectrogram, host buffers (PCIe-inclusive)",
                       (f"1 ch x {sec} s, pageable host in/out", fr), sec_per * 1e3, x.size * 4 + fr * 4096, "frames",
                       note=f"wall clock per reference-API call, {calls} calls; kernel-only rate in the rows above"))
    amd.lib.vv_dsp_stft_destroy(h)
    B = 8192
    amd.lib.vv_dsp_fft_make_plan_many.argtypes = [C.c_size_t, C.c_int, C.c_int, C.c_size_t, C.POINTER(C.c_void_p)]
    pl = C.c_void_p()
    assert amd.lib.vv_dsp_fft_make_plan_many(1024, C2C, FWD, B, C.byref(pl)) == 0
    xin = (rng.random((B, 1024)) + 1j * rng.random((B, 1024))).astype(np.complex64)
    yo = np.empty_like(xin)
    call = lambda: amd.lib.vv_dsp_fft_execute(pl, xin.ctypes.data, yo.ctypes.data)
    assert call() == 0
    sec_per, calls = cpu_time(call, budget=1.5, max_calls=200)
    out.append(row("fft_c2c_1024_host", "a6 vv_dsp_fft_execute C2C, host buffers (PCIe-inclusive)",
                   (f"{B} x 1024 c2c fwd, pageable host in/out", B), sec_per * 1e3, 16 * 1024 * B, "transforms",
                   note=f"wall clock per call of a batch-{B} plan, {calls} calls"))
    amd.lib.vv_dsp_fft_destroy(pl)

    if a.json:
        with open(a.json, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(0), "date": time.strftime("%Y-%m-%d"),
                       "rows": out}, f, indent=1)


if __name__ == "__main__":
    main()
