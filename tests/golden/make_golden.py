#!/usr/bin/env python3
"""Generate the committed golden vectors in tests/golden/*.npz.

Inputs follow the reference harness conventions (python/test_fft.py:41-54,
python/test_filters.py:36-44 of the reference) and SURVEY.md section 8c row 6.
Each file holds: the f32 input(s), `kiss` = the reference's own output
(oracle/_ref/libvvref.so, i.e. the reference sources compiled by
oracle/Makefile), and `np64` = NumPy/SciPy float64 on the same f32 inputs.

Run in the build container (needs oracle/_ref, i.e. /root/reference):
    make -C oracle && python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np
import scipy.fft
import scipy.signal

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from vvapi import VvDsp, C2C, R2C, C2R, FWD, BWD, FIRWIN_HANNING  # noqa: E402

REF = os.path.join(HERE, "..", "..", "oracle", "_ref", "libvvref.so")


def save(name, manifest, desc, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrays)
    manifest[name] = {"desc": desc, "arrays": {k: [str(v.dtype), list(v.shape)]
                                               for k, v in arrays.items()}}


def main():
    ref = VvDsp(REF)
    man = {}

    # 1. python/test_fft.py exactly: default_rng(0), C2C, then R2C, then C2R.
    for n in (16, 1024):
        rng = np.random.default_rng(0)
        x = rng.random(n) + 1j * rng.random(n)
        x32 = x.astype(np.complex64)
        xr = rng.random(n).astype(np.float32)
        X = np.fft.rfft(xr.astype(np.float64))
        X32 = X.astype(np.complex64)
        save(f"fft_testpy_n{n}", man, "python/test_fft.py inputs (seed 0): c2c fwd+bwd, r2c, c2r",
             x=x32, c2c_fwd_kiss=ref.fft(x32, C2C, FWD), c2c_fwd_np64=np.fft.fft(x32.astype(np.complex128)),
             c2c_bwd_kiss=ref.fft(x32, C2C, BWD), c2c_bwd_np64=np.fft.ifft(x32.astype(np.complex128)),
             xr=xr, r2c_kiss=ref.fft(xr, R2C), r2c_np64=np.fft.rfft(xr.astype(np.float64)),
             X=X32, c2r_kiss=ref.fft(X32, C2R, BWD, n=n),
             c2r_np64=np.fft.irfft(X32.astype(np.complex128), n=n))

    # 2. batched c2c 64 x 1024, uniform [-0.5, 0.5), seed 1
    rng = np.random.default_rng(1)
    xb = (rng.uniform(-0.5, 0.5, (64, 1024)) + 1j * rng.uniform(-0.5, 0.5, (64, 1024))).astype(np.complex64)
    kiss = np.stack([ref.fft(r, C2C, FWD) for r in xb])
    save("fft_batch64_n1024", man, "batched c2c forward 64x1024 uniform[-0.5,0.5) seed 1",
         x=xb, kiss=kiss, np64=np.fft.fft(xb.astype(np.complex128), axis=1))

    # 3. STFT spectrogram: 48000 samples uniform[-1,1) seed 3, nfft 1024 hop 256 Hann
    rng = np.random.default_rng(3)
    sig = rng.uniform(-1, 1, 48000).astype(np.float32)
    mag = ref.spectrogram(sig, 1024, 256)
    win = ref.hann(1024)
    nfr = mag.shape[0]
    pad = np.concatenate([sig.astype(np.float64), np.zeros(1024, np.float64)])
    fr = np.stack([pad[f * 256:f * 256 + 1024] for f in range(nfr)])
    np_mag = np.abs(np.fft.fft(fr * win.astype(np.float64), axis=1))
    save("stft_48000_n1024_h256", man, "stft spectrogram 48000 samples uniform[-1,1) seed 3, 1024/256 Hann",
         x=sig, window=win, kiss=mag.astype(np.float32), np64=np_mag)

    # 4. Hilbert N = 1024 and odd N = 255 (standard normal, seed 5)
    rng = np.random.default_rng(5)
    for n in (1024, 255):
        x = rng.standard_normal(n).astype(np.float32)
        save(f"hilbert_n{n}", man, f"hilbert analytic N={n} standard normal seed 5",
             x=x, kiss=ref.hilbert(x), np64=scipy.signal.hilbert(x.astype(np.float64)))

    # 5. DCT-II N in {64, 1024} (+ its inverse), standard normal seed 6
    rng = np.random.default_rng(6)
    for n in (64, 1024):
        x = rng.standard_normal(n).astype(np.float32)
        y = ref.dct(x, 2, False)
        save(f"dct2_n{n}", man, f"DCT-II forward/inverse N={n} standard normal seed 6",
             x=x, kiss=y, np64=scipy.fft.dct(x.astype(np.float64), type=2) / 2.0,
             inv_kiss=ref.dct(y, 2, True),
             inv_np64=scipy.fft.idct(2.0 * y.astype(np.float64), type=2))

    # 6. FIR: 257 taps Hann fc 0.25 on 16384 samples standard normal seed 1
    rng = np.random.default_rng(1)
    h = ref.fir_design_lowpass(257, 0.25, FIRWIN_HANNING)
    x = rng.standard_normal(16384).astype(np.float32)
    save("fir_257_n16384", man, "FIR 257-tap Hann fc=0.25, 16384 samples N(0,1) seed 1; "
         "kiss = vv_dsp_fir_apply (direct, fresh state)",
         h=h, x=x, kiss=ref.fir_apply(h, x), np64=scipy.signal.lfilter(h.astype(np.float64), [1.0],
                                                                        x.astype(np.float64)))
    # 6b. the reference's fir_apply_fft itself on a small block (its C2R is O(n^2))
    xs = x[:1500].copy()
    save("firfft_257_n1500", man, "vv_dsp_fir_apply_fft (single block) 257 taps on 1500 samples",
         h=h, x=xs, kiss=ref.fir_apply(h, xs, fft=True),
         np64=scipy.signal.lfilter(h.astype(np.float64), [1.0], xs.astype(np.float64)))

    # 7. mel filterbank / log-mel / MFCC (src/features/mel.c; mfcc_tests.c parameters)
    rng = np.random.default_rng(7)
    st, fb = ref.mel_filterbank(512, 26, 16000.0, 0.0, 8000.0)
    assert st == 0
    power = (rng.random((16, 257)) ** 2).astype(np.float32)
    power[0] = 1.0 / (1.0 + np.arange(257, dtype=np.float32))   # mfcc_tests.c synthetic spectrum
    lm = ref.log_mel(power, fb, 1e-10)
    save("mel_512_26", man, "mel filterbank 512-pt/26 mels/16 kHz/0-8 kHz (HTK), log-mel eps 1e-10 of 16 power "
         "rows (row 0 = 1/(1+k), others uniform^2 seed 7), MFCC 13 coeffs lifter 22",
         fb=fb, power=power, log_mel_kiss=lm, mfcc_kiss=ref.mfcc(lm, 13, 22.0),
         log_mel_np64=np.log(power.astype(np.float64) @ fb.astype(np.float64).T + 1e-10))

    # 8. CZT (python/test_czt.py cases) and the cepstrum family (envelope_tests.c style)
    from scipy.signal import czt as sp_czt

    def eff(z):   # W / A as the transform sees them: float pair, |z| rounded to float (czt.c:81-82)
        z = complex(np.complex64(z))
        return float(np.float32(abs(z))) * np.exp(1j * np.angle(z))

    rng = np.random.default_rng(0)
    x = (rng.standard_normal(32) + 1j * rng.standard_normal(32)).astype(np.complex64)
    w = np.array([np.exp(-2j * np.pi / 32)], np.complex64)
    save("czt_testpy_n32", man, "python/test_czt.py: 32 complex N(0,1) seed 0, M = 32, DFT parameters",
         x=x, w=w, kiss=ref.czt(x, 32, complex(w[0]), 1.0 + 0j),
         np64=sp_czt(x.astype(np.complex128), m=32, w=eff(w[0]), a=1.0))
    st, W, A = ref.czt_params(800.0, 1200.0, 64, 48000.0)
    assert st == 0
    xr = np.cos(2 * np.pi * 1000.0 * np.arange(32) / 48000.0).astype(np.float32)
    save("czt_zoom_n32_m64", man, "python/test_czt.py zoom: 1 kHz tone, 32 samples @ 48 kHz, 800-1200 Hz, M = 64 "
         "(W, A from vv_dsp_czt_params_for_freq_range)",
         x=xr, w=np.array([W], np.complex64), a=np.array([A], np.complex64), kiss=ref.czt(xr, 64, W, A),
         np64=sp_czt(xr.astype(np.float64), m=64, w=eff(W), a=eff(A)))
    rng = np.random.default_rng(8)
    x = rng.standard_normal(64).astype(np.float32)
    c = (0.05 * rng.standard_normal(64)).astype(np.float32)
    X = np.fft.fft(x.astype(np.float64))
    C = np.zeros(64)
    C[0], C[1:32] = c[0], 2 * c[1:32].astype(np.float64)
    H = np.exp(np.real(np.fft.fft(C)))
    save("cepstrum_n64", man, "cepstrum of 64 N(0,1) seed 8; minimum phase of a 0.05 N(0,1) cepstrum",
         x=x, ceps_kiss=ref.cepstrum(x), ceps_np64=np.real(np.fft.ifft(np.log(np.abs(X) + 1e-12))),
         c=c, iceps_kiss=ref.icepstrum_minphase(c), iceps_np64=np.real(np.fft.ifft(H)),
         minph_kiss=ref.minphase_from_cepstrum(c), minph_np64=H)

    round2_sets(ref, man)
    round3_sets(ref, man)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print("wrote", len(man), "golden sets")


def filtfilt_f64(h, x):
    """filter/common.c:6-80 in float64 (reflection pad of taps-1, direct form
    forward, reverse, again, reverse, centre): the f64 counterpart of the
    reference's float result."""
    h = h.astype(np.float64)
    x = x.astype(np.float64)
    n, pad = len(x), len(h) - 1
    left = [x[min(i + 1, n) - 1] for i in range(pad)][::-1]
    right = [x[n - 1 - i if i + 1 <= n else 0] for i in range(pad)]
    e = np.concatenate([np.array(left, np.float64), x, np.array(right, np.float64)])
    t = np.convolve(e, h)[: len(e)][::-1]
    t2 = np.convolve(t, h)[: len(e)][::-1]
    return t2[pad: pad + n]


def round2_sets(ref, man):
    """Round-2 fixtures: zero-phase FIR (filter/common.c), 7-smooth non-power-of-two
    FFT lengths (the reference's O(n^2) DFT, fft_kiss.c:76-92) and an STFT with
    400-sample frames."""
    h9 = ref.fir_design_lowpass(9, 0.25, 1)
    xq = np.where(np.arange(64) % 8 < 4, 1.0, -1.0).astype(np.float32)
    rng = np.random.default_rng(11)
    h257 = ref.fir_design_lowpass(257, 0.25, FIRWIN_HANNING)
    xg = rng.standard_normal(4096).astype(np.float32)
    save("filtfilt", man, "vv_dsp_filtfilt_fir: 9-tap Hamming fc 0.25 on the filter_tests.c:62-80 square wave; "
                          "257-tap Hann fc 0.25 on 4096 N(0,1) seed 11",
         h9=h9, xq=xq, yq_kiss=ref.filtfilt(h9, xq)[1], yq_np64=filtfilt_f64(h9, xq),
         h257=h257, xg=xg, yg_kiss=ref.filtfilt(h257, xg)[1], yg_np64=filtfilt_f64(h257, xg))
    rng = np.random.default_rng(12)
    x400 = (rng.random(400) - 0.5 + 1j * (rng.random(400) - 0.5)).astype(np.complex64)
    xr480 = (rng.random(480) - 0.5).astype(np.float32)
    save("fft_smooth_400_480", man, "c2c n = 400 (fwd, bwd) and r2c n = 480, uniform[-0.5,0.5) seed 12: the "
                                    "reference's O(n^2) DFT and NumPy f64",
         x=x400, c2c_fwd_kiss=ref.fft(x400, C2C, FWD), c2c_fwd_np64=np.fft.fft(x400.astype(np.complex128)),
         c2c_bwd_kiss=ref.fft(x400, C2C, BWD), c2c_bwd_np64=np.fft.ifft(x400.astype(np.complex128)),
         xr=xr480, r2c_kiss=ref.fft(xr480, R2C), r2c_np64=np.fft.rfft(xr480.astype(np.float64)))
    rng = np.random.default_rng(13)
    xs = rng.uniform(-1, 1, 16000).astype(np.float32)
    mag = ref.spectrogram(xs, 400, 160)
    w = 0.5 - 0.5 * np.cos(np.float32(2 * np.pi) / np.float32(399) * np.arange(400, dtype=np.float32))
    pad = np.concatenate([xs.astype(np.float64), np.zeros(400)])
    fr = mag.shape[0]
    np_mag = np.abs(np.fft.fft(np.stack([pad[f * 160: f * 160 + 400] for f in range(fr)]) * w.astype(np.float64),
                               axis=1))
    save("stft_16000_n400_h160", man, "stft spectrogram 16000 samples uniform[-1,1) seed 13, 400/160 Hann "
                                      "(non-power-of-two frames)",
         x=xs, kiss=mag, np64=np_mag.astype(np.float64))


REGISTER_LENGTHS = (320, 400, 441, 480, 600, 640, 720, 800, 900, 960)
# real rows whose n/2-point transform is a register length (vv-dsp_amd mixed_fft.hip VVH_SQ_HALF_LENGTHS)
REGISTER_R2C_LENGTHS = (400, 480) + tuple(2 * n for n in REGISTER_LENGTHS)


def round3_sets(ref, man):
    """Round-3 fixtures: every length of the two-pass register kernel
    (k_stft_sq), pinned to the reference's own non-power-of-two path
    (fft_kiss.c:76-92 via :114-116; R2C :120-147; STFT stft.c:74-92,112-144)
    and NumPy f64.  One set per length: c2c forward and backward of one complex
    row, and an STFT of 3*n+13 samples at hop n/2 (6 frames, the last one
    zero-padded): the reference's magnitude rows (vv_dsp_stft_spectrogram) and
    complex rows (vv_dsp_stft_process per frame), with f64 complex rows
    (magnitude and power rows follow from them)."""
    for n in REGISTER_LENGTHS:
        rng = np.random.default_rng(30000 + n)
        x = (rng.random(n) - 0.5 + 1j * (rng.random(n) - 0.5)).astype(np.complex64)
        hop = n // 2
        sig = rng.uniform(-1, 1, 3 * n + 13).astype(np.float32)
        mag = ref.spectrogram(sig, n, hop)
        nfr = mag.shape[0]
        win = ref.window(1, n)[1]
        pad = np.concatenate([sig, np.zeros(n, np.float32)])
        frames = np.stack([pad[f * hop: f * hop + n] for f in range(nfr)])
        st, h = ref.stft_create(n, hop)
        assert st == 0
        try:
            cpx = np.stack([ref.stft_process(h, fr.copy(), n) for fr in frames])
        finally:
            ref.lib.vv_dsp_stft_destroy(h)
        X64 = np.fft.fft(frames.astype(np.float64) * win.astype(np.float64), axis=1)
        save(f"register_n{n}", man, f"register-kernel length {n}: c2c fwd/bwd of one uniform[-0.5,0.5) complex "
             f"row (seed {30000 + n}); STFT of {3 * n + 13} uniform[-1,1) samples, nfft {n}, hop {hop}, Hann: "
             "reference magnitude rows, reference complex rows (stft_process), f64 complex rows",
             x=x, c2c_fwd_kiss=ref.fft(x, C2C, FWD), c2c_fwd_np64=np.fft.fft(x.astype(np.complex128)),
             c2c_bwd_kiss=ref.fft(x, C2C, BWD), c2c_bwd_np64=np.fft.ifft(x.astype(np.complex128)),
             sig=sig, hop=np.array([hop], np.int64), stft_mag_kiss=mag.astype(np.float32),
             stft_cpx_kiss=cpx.astype(np.complex64), stft_cpx_np64=X64)
    rows, kiss, np64 = {}, {}, {}
    for n in REGISTER_R2C_LENGTHS:
        rng = np.random.default_rng(31000 + n)
        xr = (rng.random(n) - 0.5).astype(np.float32)
        rows[f"x{n}"] = xr
        kiss[f"kiss{n}"] = ref.fft(xr, R2C)
        np64[f"np64_{n}"] = np.fft.rfft(xr.astype(np.float64))
    save("register_r2c", man, "R2C rows at every length whose half is a register-kernel length "
         f"{REGISTER_R2C_LENGTHS}: uniform[-0.5,0.5) seed 31000+n; the reference's R2C (its O(n^2) DFT) and "
         "NumPy f64", **rows, **kiss, **np64)


if __name__ == "__main__":
    if "--round3-only" in sys.argv:   # add the round-3 sets without rewriting the others
        with open(os.path.join(HERE, "manifest.json")) as f:
            m = json.load(f)
        round3_sets(VvDsp(REF), m)
        with open(os.path.join(HERE, "manifest.json"), "w") as f:
            json.dump(m, f, indent=1, sort_keys=True)
        print("manifest now", len(m), "sets")
    elif "--round2-only" in sys.argv:   # add the round-2 sets without rewriting the others
        with open(os.path.join(HERE, "manifest.json")) as f:
            m = json.load(f)
        round2_sets(VvDsp(REF), m)
        with open(os.path.join(HERE, "manifest.json"), "w") as f:
            json.dump(m, f, indent=1, sort_keys=True)
        print("manifest now", len(m), "sets")
    else:
        main()
