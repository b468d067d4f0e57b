/*
 * vv_oracle.c -- CPU restatement of the vv-dsp reference spectral hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see vv_oracle.h).  Never linked into the product.
 * Each routine follows the floating-point operation order of the cited
 * reference function so the results are bit-identical when built with the
 * reference's flags; tests/test_oracle.py checks exactly that.
 */
#include "vv_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ORC_PI_D 3.141592653589793238462643383279502884
/* vv_dsp_math.h: VV_DSP_PI = (float)PI_D; VV_DSP_TWO_PI = (float)(2.0 * PI_D) */
static const float kPi = (float)ORC_PI_D;
static const float kTwoPi = (float)(2.0 * ORC_PI_D);

typedef struct { float re, im; } ocpx;

static int pow2(size_t n) { return n != 0 && (n & (n - 1)) == 0; }

/* In-place bit-reversal permutation (any method gives the same permutation). */
static void bitrev_permute(ocpx* a, size_t n) {
    size_t j = 0;
    for (size_t i = 0; i + 1 < n; ++i) {
        if (i < j) { ocpx t = a[i]; a[i] = a[j]; a[j] = t; }
        size_t m = n >> 1;
        while (m >= 1 && (j & m)) { j ^= m; m >>= 1; }
        j |= m;
    }
}

/* fft_kiss.c:27-74 -- radix-2 DIT; per-stage twiddle by complex recurrence. */
static void radix2_inplace(ocpx* a, size_t n, int sign) {
    bitrev_permute(a, n);
    for (size_t span = 2; span <= n; span <<= 1) {
        const float theta = (float)(-sign) * 2.0f * kPi / (float)span;
        const float step_re = cosf(theta);
        const float step_im = sinf(theta);
        const size_t half = span >> 1;
        for (size_t base = 0; base < n; base += span) {
            float w_re = 1.0f, w_im = 0.0f;
            ocpx* lo = a + base;
            ocpx* hi = a + base + half;
            for (size_t k = 0; k < half; ++k) {
                const float t_re = w_re * hi[k].re - w_im * hi[k].im;
                const float t_im = w_re * hi[k].im + w_im * hi[k].re;
                hi[k].re = lo[k].re - t_re;
                hi[k].im = lo[k].im - t_im;
                lo[k].re += t_re;
                lo[k].im += t_im;
                const float nr = w_re * step_re - w_im * step_im;
                const float ni = w_re * step_im + w_im * step_re;
                w_re = nr;
                w_im = ni;
            }
        }
    }
    if (sign < 0) {
        const float s = 1.0f / (float)n;
        for (size_t i = 0; i < n; ++i) { a[i].re *= s; a[i].im *= s; }
    }
}

/* fft_kiss.c:76-92 -- O(n^2) DFT with per-term cosf/sinf. */
static void naive_dft(const ocpx* x, ocpx* y, size_t n, int sign) {
    const float scale = (sign < 0) ? (1.0f / (float)n) : 1.0f;
    for (size_t k = 0; k < n; ++k) {
        float acc_re = 0, acc_im = 0;
        for (size_t t = 0; t < n; ++t) {
            const float ang = (float)(-sign) * 2.0f * kPi * (float)(k * t) / (float)n;
            const float c = cosf(ang), s = sinf(ang);
            acc_re += x[t].re * c - x[t].im * s;
            acc_im += x[t].re * s + x[t].im * c;
        }
        y[k].re = acc_re * scale;
        y[k].im = acc_im * scale;
    }
}

int orc_fft_c2c(const float* in, float* out, size_t n, int dir) {
    if (!in || !out || n == 0) return 1;
    const int sign = (dir >= 0) ? +1 : -1;
    if (pow2(n)) {
        if (out != in) memcpy(out, in, sizeof(ocpx) * n);
        radix2_inplace((ocpx*)out, n, sign);
    } else {
        naive_dft((const ocpx*)in, (ocpx*)out, n, sign);
    }
    return 0;
}

int orc_fft_r2c(const float* in, float* out, size_t n) {
    if (!in || !out || n == 0) return 1;
    ocpx* buf = (ocpx*)malloc(sizeof(ocpx) * n);
    ocpx* spec = (ocpx*)malloc(sizeof(ocpx) * n);
    if (!buf || !spec) { free(buf); free(spec); return 4; }
    for (size_t i = 0; i < n; ++i) { buf[i].re = in[i]; buf[i].im = 0.0f; }
    if (pow2(n)) {
        memcpy(spec, buf, sizeof(ocpx) * n);
        radix2_inplace(spec, n, +1);
    } else {
        naive_dft(buf, spec, n, +1);
    }
    const size_t nh = n / 2 + 1;
    memcpy(out, spec, sizeof(ocpx) * nh);
    if ((n & 1) == 0 && nh > 1) out[2 * (nh - 1) + 1] = 0.0f;  /* Nyquist imag forced 0 */
    free(buf);
    free(spec);
    return 0;
}

int orc_fft_c2r(const float* in, float* out, size_t n) {
    if (!in || !out || n == 0) return 1;
    const size_t nh = n / 2 + 1;
    const ocpx* half = (const ocpx*)in;
    ocpx* full = (ocpx*)malloc(sizeof(ocpx) * n);
    ocpx* tim = (ocpx*)malloc(sizeof(ocpx) * n);
    if (!full || !tim) { free(full); free(tim); return 4; }
    for (size_t k = 0; k < n; ++k) {
        if (k < nh) {
            full[k] = half[k];
        } else {
            const size_t m = n - k;
            if (m > 0 && m < nh) { full[k].re = half[m].re; full[k].im = -half[m].im; }
            else { full[k].re = 0.0f; full[k].im = 0.0f; }
        }
    }
    naive_dft(full, tim, n, -1);   /* the reference always takes the O(n^2) path here */
    for (size_t i = 0; i < n; ++i) out[i] = tim[i].re;
    free(full);
    free(tim);
    return 0;
}

/* window.c:16-49 (boxcar / hann / hamming, symmetric, N==1 -> 1) */
int orc_window(int kind, size_t n, float* out) {
    if (!out || n == 0) return 1;
    if (kind == 0) { for (size_t i = 0; i < n; ++i) out[i] = 1.0f; return 0; }
    if (kind != 1 && kind != 2) return 3;
    if (n == 1) { out[0] = 1.0f; return 0; }
    const float a = (kind == 1) ? 0.5f : 0.54f;
    const float b = (kind == 1) ? 0.5f : 0.46f;
    const float step = kTwoPi / (float)(n - 1);
    for (size_t i = 0; i < n; ++i) {
        const float c = cosf(step * (float)i);
        out[i] = a - b * c;
    }
    return 0;
}

/* stft.c:74-92 -- window (vectorized_math_fallback.c:13-29) then C2C forward. */
int orc_stft_process(const float* win, size_t nfft, const float* frame, float* spec_out) {
    if (!win || !frame || !spec_out || nfft == 0) return 1;
    float* cin = (float*)malloc(sizeof(float) * 2 * nfft);
    if (!cin) return 4;
    for (size_t i = 0; i < nfft; ++i) { cin[2 * i] = frame[i] * win[i]; cin[2 * i + 1] = 0.0f; }
    int rc = orc_fft_c2c(cin, spec_out, nfft, +1);
    free(cin);
    return rc;
}

size_t orc_stft_num_frames(size_t n, size_t nfft, size_t hop) {
    return (n < nfft) ? 1 : (1 + (n - nfft + hop) / hop);
}

/* stft.c:112-144 */
int orc_stft_spectrogram(const float* win, size_t nfft, size_t hop,
                         const float* signal, size_t n, float* out_mag, size_t* frames) {
    if (!win || !signal || !out_mag || !frames) return 1;
    if (nfft == 0 || hop == 0) return 2;
    const size_t nf = orc_stft_num_frames(n, nfft, hop);
    *frames = nf;
    float* frame = (float*)malloc(sizeof(float) * nfft);
    float* spec = (float*)malloc(sizeof(float) * 2 * nfft);
    if (!frame || !spec) { free(frame); free(spec); return 4; }
    for (size_t f = 0; f < nf; ++f) {
        const size_t s0 = f * hop;
        for (size_t i = 0; i < nfft; ++i) frame[i] = (s0 + i < n) ? signal[s0 + i] : 0.0f;
        orc_stft_process(win, nfft, frame, spec);
        float* row = out_mag + f * nfft;
        for (size_t k = 0; k < nfft; ++k) {
            const float re = spec[2 * k], im = spec[2 * k + 1];
            row[k] = sqrtf(re * re + im * im);
        }
    }
    free(frame);
    free(spec);
    return 0;
}

/* stft.c:95-110 -- inverse C2C (1/n) then out_add += re*w, norm_add += w*w */
int orc_stft_reconstruct(const float* win, size_t nfft, const float* spec,
                         float* out_add, float* norm_add) {
    if (!win || !spec || !out_add) return 1;
    float* t = (float*)malloc(sizeof(float) * 2 * nfft);
    if (!t) return 4;
    orc_fft_c2c(spec, t, nfft, -1);
    for (size_t i = 0; i < nfft; ++i) {
        const float w = win[i];
        out_add[i] += t[2 * i] * w;
        if (norm_add) norm_add[i] += w * w;
    }
    free(t);
    return 0;
}

/* hilbert.c:14-75 -- R2C, Hermitian expand, one-sided mask, inverse C2C. */
int orc_hilbert_analytic(const float* x, size_t n, float* z_out) {
    if (!x || !z_out) return 1;
    if (n == 0) return 2;
    const size_t nh = n / 2 + 1;
    float* half = (float*)malloc(sizeof(float) * 2 * nh);
    float* zs = (float*)calloc(2 * n, sizeof(float));
    if (!half || !zs) { free(half); free(zs); return 4; }
    orc_fft_r2c(x, half, n);
    /* Z[k]: DC (and N/2 for even N) pass, positive bins doubled, negatives zero.
     * The mirrored Xfull entries only feed bins the mask zeroes. */
    zs[0] = half[0];
    zs[1] = half[1];
    const size_t kpos_end = (n % 2 == 0) ? n / 2 : nh;
    for (size_t k = 1; k < kpos_end; ++k) {
        zs[2 * k] = 2.0f * half[2 * k];
        zs[2 * k + 1] = 2.0f * half[2 * k + 1];
    }
    if (n % 2 == 0) { zs[n] = half[n]; zs[n + 1] = half[n + 1]; }
    orc_fft_c2c(zs, z_out, n, -1);
    free(half);
    free(zs);
    return 0;
}

/* hilbert.c:77-96: principal phase of z[0], then f64 increments
 * atan2(Im(z_i conj z_{i-1}), Re(z_i conj z_{i-1})) summed left to right */
int orc_inst_phase(const float* z, size_t n, float* phase) {
    if (!z || !phase) return 1;
    if (n == 0) return 2;
    double acc = atan2((double)z[1], (double)z[0]);
    phase[0] = (float)acc;
    for (size_t i = 1; i < n; ++i) {
        const double cr = z[2 * i], ci = z[2 * i + 1], pr = z[2 * i - 2], pi = z[2 * i - 1];
        const double re = cr * pr + ci * pi;
        const double im = ci * pr - cr * pi;
        acc += atan2(im, re);
        phase[i] = (float)acc;
    }
    return 0;
}

/* hilbert.c:98-113: freq[0] = 0, freq[i] = (p[i] - p[i-1]) * fs / (2 pi) in f64 */
int orc_inst_freq(const float* phase, size_t n, double fs, float* freq) {
    if (!phase || !freq) return 1;
    if (n == 0) return 2;
    const double scale = fs / (2.0 * 3.141592653589793238462643383279502884);
    freq[0] = 0.0f;
    for (size_t i = 1; i < n; ++i) freq[i] = (float)(((double)phase[i] - (double)phase[i - 1]) * scale);
    return 0;
}

/* dct.c:21-68 naive kernels; :86-136 dispatch (NaN policy PROPAGATE = identity) */
int orc_dct(const float* in, float* out, size_t n, int type, int dir) {
    if (!in || !out) return 1;
    if (n == 0) return 2;
    const float N = (float)n;
    if ((type == 2 && dir > 0)) {
        for (size_t k = 0; k < n; ++k) {
            float acc = 0;
            for (size_t i = 0; i < n; ++i) {
                const float ang = kPi * ((float)i + 0.5f) * (float)k / N;
                acc += in[i] * cosf(ang);
            }
            out[k] = acc;
        }
    } else if ((type == 2 || type == 3) && dir < 0) {
        const float scale = 2.0f / N;
        for (size_t i = 0; i < n; ++i) {
            float acc = 0.5f * in[0];
            for (size_t k = 1; k < n; ++k) {
                const float ang = kPi * (float)k * ((float)i + 0.5f) / N;
                acc += in[k] * cosf(ang);
            }
            out[i] = scale * acc;
        }
    } else if (type == 3 && dir > 0) {
        for (size_t k = 0; k < n; ++k) {
            float acc = in[0];
            for (size_t i = 1; i < n; ++i) {
                const float ang = kPi * (float)k * ((float)i + 0.5f) / N;
                acc += 2.0f * in[i] * cosf(ang);
            }
            out[k] = acc;
        }
    } else if (type == 4) {
        for (size_t k = 0; k < n; ++k) {
            float acc = 0;
            for (size_t i = 0; i < n; ++i) {
                const float ang = kPi * ((float)i + 0.5f) * ((float)k + 0.5f) / N;
                acc += in[i] * cosf(ang);
            }
            if (dir < 0) acc *= 2.0f / N;
            out[k] = acc;
        }
    } else {
        return 3;
    }
    return 0;
}

/* fir.c:8-15 */
static float sinc_f(float v) {
    if (v == 0.0f) return 1.0f;
    return (float)(sinf(kPi * v) / (kPi * v));
}

/* fir.c:17-45 */
static int fir_window(float* w, size_t n, int kind) {
    const float den = (float)(n - 1);
    for (size_t i = 0; i < n; ++i) {
        switch (kind) {
        case 0: w[i] = 1.0f; break;
        case 1: w[i] = (float)(0.54f - 0.46f * cosf(kTwoPi * (float)i / den)); break;
        case 2: w[i] = (float)(0.5f - 0.5f * cosf(kTwoPi * (float)i / den)); break;
        case 3: {
            const double d1 = (float)cosf((float)((2.0 * ORC_PI_D) * (double)i / (double)(n - 1)));
            const double d2 = (float)cosf((float)(2.0 * (2.0 * ORC_PI_D) * (double)i / (double)(n - 1)));
            w[i] = (float)(0.42 - 0.5 * d1 + 0.08 * d2);
            break;
        }
        default: return 4;
        }
    }
    return 0;
}

/* fir.c:47-73 */
int orc_fir_design_lowpass(float* h, size_t taps, float fc, int wkind) {
    if (!h) return 1;
    if (taps == 0) return 2;
    if (!(fc > 0.0f && fc < 1.0f)) return 3;
    const float centre = (float)(taps - 1) / 2.0f;
    for (size_t i = 0; i < taps; ++i) {
        const float m = (float)i - centre;
        h[i] = 2 * fc * sinc_f(2 * fc * m);
    }
    float* w = (float*)malloc(sizeof(float) * taps);
    if (!w) return 4;
    int rc = fir_window(w, taps, wkind);
    if (rc) { free(w); return rc; }
    for (size_t i = 0; i < taps; ++i) h[i] *= w[i];
    free(w);
    return 0;
}

/* fir.c:160-196 */
int orc_fir_apply(const float* h, size_t taps, float* history, size_t* hist_idx,
                  const float* x, float* y, size_t n) {
    if (!h || !x || !y || !hist_idx) return 1;
    if (taps == 0) return 2;
    const size_t hs = taps - 1;
    for (size_t i = 0; i < n; ++i) {
        float acc = 0;
        acc += h[0] * x[i];
        if (hs) {
            size_t r = (*hist_idx == 0) ? hs - 1 : *hist_idx - 1;
            for (size_t t = 1; t < taps; ++t) {
                acc += h[t] * history[r];
                r = (r == 0) ? hs - 1 : r - 1;
            }
        }
        y[i] = acc;
        if (hs) {
            history[*hist_idx] = x[i];
            *hist_idx = (*hist_idx + 1) % hs;
        }
    }
    return 0;
}

/* fir.c:75-135 */
int orc_fir_apply_fft(const float* h, size_t taps, const float* x, float* y, size_t n) {
    if (!h || !x || !y) return 1;
    if (taps == 0) return 2;
    size_t nfft = 1;
    while (nfft < n + taps - 1) nfft <<= 1;
    const size_t nc = nfft / 2 + 1;
    float* xb = (float*)calloc(nfft, sizeof(float));
    float* hb = (float*)calloc(nfft, sizeof(float));
    float* X = (float*)calloc(2 * nc, sizeof(float));
    float* H = (float*)calloc(2 * nc, sizeof(float));
    float* Y = (float*)calloc(2 * nc, sizeof(float));
    if (!xb || !hb || !X || !H || !Y) { free(xb); free(hb); free(X); free(H); free(Y); return 4; }
    memcpy(xb, x, n * sizeof(float));
    memcpy(hb, h, taps * sizeof(float));
    orc_fft_r2c(xb, X, nfft);
    orc_fft_r2c(hb, H, nfft);
    for (size_t k = 0; k < nc; ++k) {   /* vectorized_math_fallback.c:31-53 */
        const float ar = X[2 * k], ai = X[2 * k + 1], br = H[2 * k], bi = H[2 * k + 1];
        Y[2 * k] = ar * br - ai * bi;
        Y[2 * k + 1] = ar * bi + ai * br;
    }
    orc_fft_c2r(Y, xb, nfft);
    for (size_t i = 0; i < n; ++i) y[i] = xb[i];
    free(xb); free(hb); free(X); free(H); free(Y);
    return 0;
}

/* common.c:6-80 -- zero-phase FIR: reflection padding of num_taps-1 samples,
 * the stateless direct form forward, reverse, again, reverse, centre.  Written
 * as a restatement of the published algorithm, index by index (the reflection
 * clamps to x[n-1] / x[0] once the pad exceeds the signal). */
int orc_filtfilt_fir(const float* h, size_t taps, const float* x, float* y, size_t n) {
    if (!h || !x || !y) return 1;
    if (taps == 0) return 2;
    if (n == 0) return 0;   /* the reference reads x[-1] here; nothing to produce */
    const size_t pad = taps - 1, m = n + 2 * pad;
    float* e = (float*)malloc(m * sizeof(float));
    float* a = (float*)malloc(m * sizeof(float));
    float* b = (float*)malloc(m * sizeof(float));
    if (!e || !a || !b) { free(e); free(a); free(b); return 4; }
    for (size_t i = 0; i < n; ++i) e[pad + i] = x[i];
    for (size_t i = 0; i < pad; ++i) {
        e[pad - 1 - i] = x[(i + 1 <= n ? i + 1 : n) - 1];
        e[pad + n + i] = x[i + 1 <= n ? n - 1 - i : 0];
    }
    for (int pass = 0; pass < 2; ++pass) {
        const float* s = pass ? b : e;
        float* d = a;
        float* tmp = (float*)malloc(m * sizeof(float));
        if (!tmp) { free(e); free(a); free(b); return 4; }
        for (size_t i = 0; i < m; ++i) {
            float acc = 0;
            const size_t kmax = i + 1 < taps ? i + 1 : taps;
            for (size_t k = 0; k < kmax; ++k) acc += h[k] * s[i - k];
            tmp[i] = acc;
        }
        for (size_t i = 0; i < m; ++i) d[i] = tmp[m - 1 - i];   /* reverse */
        free(tmp);
        if (!pass) memcpy(b, a, m * sizeof(float));
    }
    memcpy(y, a + pad, n * sizeof(float));
    free(e); free(a); free(b);
    return 0;
}

/* ---- mel / MFCC (src/features/mel.c) ------------------------------------- */
/* mel.c:14-20 */
float orc_hz_to_mel(float hz) {
    if (hz < 0.0f) return 0.0f;
    return 2595.0f * log10f(1.0f + hz / 700.0f);
}

/* mel.c:22-28 (VV_DSP_POW = powf, vv_dsp_math.h:48) */
float orc_mel_to_hz(float mel) {
    if (mel < 0.0f) return 0.0f;
    return 700.0f * (powf(10.0f, mel / 2595.0f) - 1.0f);
}

/* mel.c:51-62 */
static size_t orc_searchsorted(const float* a, size_t n, float v) {
    size_t lo = 0, hi = n;
    while (lo < hi) {
        const size_t mid = lo + (hi - lo) / 2;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

/* mel.c:66-193 (HTK only, as the reference).  fb: n_mels x (n_fft/2+1), caller-owned. */
int orc_mel_filterbank(size_t n_fft, size_t n_mels, float sample_rate, float fmin, float fmax, float* fb) {
    if (!fb) return 1;
    if (n_fft == 0 || n_mels == 0 || sample_rate <= 0.0f || fmin < 0.0f || fmax <= fmin) return 2;
    if (fmax > sample_rate / 2.0f) return 3;
    const size_t nb = n_fft / 2 + 1;
    if (n_mels >= nb) return 2;
    memset(fb, 0, n_mels * nb * sizeof(float));
    const float mel_min = orc_hz_to_mel(fmin), mel_max = orc_hz_to_mel(fmax);
    const size_t np = n_mels + 2;
    float* mel = (float*)malloc(np * sizeof(float));
    float* hz = (float*)malloc(np * sizeof(float));
    float* ff = (float*)malloc(nb * sizeof(float));
    if (!mel || !hz || !ff) { free(mel); free(hz); free(ff); return 4; }
    const float step = (mel_max - mel_min) / (float)(np - 1);   /* linspace, mel.c:35-46 */
    for (size_t i = 0; i < np; ++i) mel[i] = mel_min + step * (float)i;
    for (size_t i = 0; i < np; ++i) hz[i] = orc_mel_to_hz(mel[i]);
    for (size_t i = 0; i < nb; ++i) ff[i] = (float)i * sample_rate / (float)n_fft;
    for (size_t m = 0; m < n_mels; ++m) {
        const float left = hz[m], center = hz[m + 1], right = hz[m + 2];
        const size_t li = orc_searchsorted(ff, nb, left), ci = orc_searchsorted(ff, nb, center),
                     ri = orc_searchsorted(ff, nb, right);
        float* row = fb + m * nb;
        for (size_t k = li; k < ci && k < nb; ++k) row[k] = (ff[k] - left) / (center - left);
        for (size_t k = ci; k < ri && k < nb; ++k) row[k] = (right - ff[k]) / (right - center);
        float sum = 0.0f;
        for (size_t k = 0; k < nb; ++k) sum += row[k];
        if (sum > 0.0f)
            for (size_t k = 0; k < nb; ++k) row[k] /= sum;
    }
    free(mel); free(hz); free(ff);
    return 0;
}

/* mel.c:204-245 (VV_DSP_LOG = logf) */
int orc_log_mel(const float* power, size_t frames, size_t nb, const float* fb, size_t n_mels, float eps,
                float* out) {
    if (!power || !fb || !out) return 1;
    if (frames == 0 || nb == 0 || n_mels == 0) return 2;
    if (eps < 0.0f) return 3;
    for (size_t f = 0; f < frames; ++f)
        for (size_t m = 0; m < n_mels; ++m) {
            float e = 0.0f;
            for (size_t k = 0; k < nb; ++k) e += power[f * nb + k] * fb[m * nb + k];
            out[f * n_mels + m] = logf(e + eps);
        }
    return 0;
}

/* mel.c:249-309: DCT-II (dct.c forward) per frame, first n_coeffs, lifter (VV_DSP_SIN = sinf) */
int orc_mfcc(const float* log_mel, size_t frames, size_t n_mels, size_t n_coeffs, float lifter, float* out) {
    if (!log_mel || !out) return 1;
    if (frames == 0 || n_mels == 0 || n_coeffs == 0 || n_coeffs > n_mels) return 2;
    if (lifter < 0.0f) return 3;
    float* d = (float*)malloc(n_mels * sizeof(float));
    if (!d) return 4;
    for (size_t f = 0; f < frames; ++f) {
        const int st = orc_dct(log_mel + f * n_mels, d, n_mels, 2, 1);
        if (st) { free(d); return st; }
        float* o = out + f * n_coeffs;
        for (size_t i = 0; i < n_coeffs; ++i) o[i] = d[i];
        if (lifter > 0.0f)
            for (size_t i = 1; i < n_coeffs; ++i)
                o[i] *= 1.0f + (lifter / 2.0f) * sinf((float)M_PI * (float)i / lifter);
    }
    free(d);
    return 0;
}

/* ------------------------------------------------------------------ framing
 * src/core/framing.c.  Non-centred frames start at f*hop and are zero-padded
 * outside the signal; centred frames start at f*hop - len/2 and mirror the
 * signal about its ends (sample -1 -> 0, -2 -> 1, n -> n-1; repeated
 * reflections with period 2n). */
static size_t orc_reflect(long idx, size_t n) {   /* framing.c:21-56 */
    if (n == 0) return 0;
    if (idx < 0) {
        long a = -idx - 1;
        if (a >= (long)n) {
            const long period = 2 * (long)n;
            a %= period;
            if (a >= (long)n) a = period - 1 - a;
        }
        return (size_t)a;
    }
    if (idx >= (long)n) {
        long r = (long)n - 1 - (idx - (long)n);
        if (r < 0) {
            r = -r - 1;
            if (r >= (long)n) {
                const long period = 2 * (long)n;
                r %= period;
                if (r >= (long)n) r = period - 1 - r;
            }
        }
        if (r < 0) r = 0;
        if (r > (long)n - 1) r = (long)n - 1;
        return (size_t)r;
    }
    return (size_t)idx;
}

size_t orc_get_num_frames(size_t signal_len, size_t frame_len, size_t hop_len, int center) {
    if (hop_len == 0) return 0;
    if (center) return (signal_len + hop_len - 1) / hop_len;
    if (signal_len < frame_len) return 0;
    return 1 + (signal_len - frame_len) / hop_len;
}

int orc_fetch_frame(const float* signal, size_t signal_len, float* frame, size_t frame_len,
                    size_t hop_len, size_t frame_index, int center, const float* window) {
    if (!signal || !frame) return 1;
    if (signal_len == 0 || frame_len == 0 || hop_len == 0) return 2;
    const long start = center ? (long)(frame_index * hop_len) - (long)(frame_len / 2) : (long)(frame_index * hop_len);
    for (size_t i = 0; i < frame_len; ++i) {
        const long k = start + (long)i;
        float v;
        if (center) v = signal[orc_reflect(k, signal_len)];
        else v = (k < 0 || k >= (long)signal_len) ? 0.0f : signal[k];
        frame[i] = window ? v * window[i] : v;
    }
    return 0;
}

int orc_overlap_add(const float* frame, float* out, size_t out_len, size_t frame_len,
                    size_t hop_len, size_t frame_index) {
    if (!frame || !out) return 1;
    if (out_len == 0 || frame_len == 0 || hop_len == 0) return 2;
    const size_t s0 = frame_index * hop_len;
    for (size_t i = 0; i < frame_len; ++i)
        if (s0 + i < out_len) out[s0 + i] += frame[i];
    return 0;
}

/* ---- CZT (src/spectral/czt.c) ------------------------------------------ */
/* czt.c:10-12 -- product without FMA contraction (the file is built -ffp-contract=off) */
static ocpx orc_cmul(ocpx a, ocpx b) {
    ocpx r;
    r.re = a.re * b.re - a.im * b.im;
    r.im = a.re * b.im + a.im * b.re;
    return r;
}

/* czt.c:22-42 */
int orc_czt_params(float f_start, float f_end, size_t M, float fs, float* w, float* a) {
    if (!w || !a) return 1;
    if (M == 0 || fs <= 0.0f) return 2;
    const float delta = (f_end - f_start) / (float)M;
    const float theta = (float)(-2.0 * ORC_PI_D * (double)delta / (double)fs);
    w[0] = cosf(theta);
    w[1] = sinf(theta);
    const float phi0 = (float)(-2.0 * ORC_PI_D * (double)f_start / (double)fs);
    a[0] = cosf(phi0);
    a[1] = sinf(phi0);
    return 0;
}

/* W^{+-e}: czt.c:96-101 / 147-153 (e, ang, mag rounded to float, powf/cosf/sinf) */
static ocpx czt_chirp(float e, float argW, float magW, int sign) {
    const float ang = sign > 0 ? e * argW : -e * argW;
    const float mag = powf(magW, sign > 0 ? e : -e);
    ocpx z;
    z.re = mag * cosf(ang);
    z.im = mag * sinf(ang);
    return z;
}

/* czt.c:58-178: Bluestein with P = next_pow2(N + M - 1), Kiss FFTs (orc_fft_c2c) */
int orc_czt_cpx(const float* x, size_t N, size_t M, float w_re, float w_im, float a_re, float a_im, float* X) {
    if (!x || !X) return 1;
    if (N == 0 || M == 0) return 2;
    const ocpx* xc = (const ocpx*)x;
    ocpx A = {a_re, a_im};
    ocpx A_inv = {A.re, -A.im};
    const float denom = A.re * A.re + A.im * A.im;
    if (denom != 0.0f) { A_inv.re = A.re / denom; A_inv.im = -A.im / denom; }
    const float argW = (float)atan2f((float)(double)w_im, (float)(double)w_re);
    const float magW = (float)hypot((double)w_re, (double)w_im);
    size_t L = N + M - 1, P = 1;
    while (P < L) P <<= 1;
    ocpx* a = (ocpx*)calloc(P, sizeof(ocpx));
    ocpx* b = (ocpx*)calloc(P, sizeof(ocpx));
    ocpx* Af = (ocpx*)malloc(P * sizeof(ocpx));
    ocpx* Bf = (ocpx*)malloc(P * sizeof(ocpx));
    if (!a || !b || !Af || !Bf) { free(a); free(b); free(Af); free(Bf); return 4; }
    ocpx A_inv_pow = {1.0f, 0.0f};
    for (size_t n = 0; n < N; ++n) {   /* :90-108, g[n] = A^-n W^(n^2/2) by recurrence */
        const float e = 0.5f * (float)((double)n * (double)n);
        const ocpx Wn2 = czt_chirp(e, argW, magW, +1);
        if (n == 0) { A_inv_pow.re = 1.0f; A_inv_pow.im = 0.0f; }
        else A_inv_pow = orc_cmul(A_inv_pow, A_inv);
        a[n] = orc_cmul(xc[n], orc_cmul(A_inv_pow, Wn2));   /* :140 */
    }
    for (size_t i = 0; i < L; ++i) {   /* :142-150 b[i] = W^(-(i-(N-1))^2/2) */
        const long m = (long)i - (long)(N - 1);
        const float dm = (float)m;
        b[i] = czt_chirp(0.5f * dm * dm, argW, magW, -1);
    }
    orc_fft_c2c((const float*)a, (float*)Af, P, 1);
    orc_fft_c2c((const float*)b, (float*)Bf, P, 1);
    for (size_t i = 0; i < P; ++i) Af[i] = orc_cmul(Af[i], Bf[i]);   /* :161-163 */
    orc_fft_c2c((const float*)Af, (float*)a, P, -1);                  /* :166, x 1/P */
    ocpx* Xc = (ocpx*)X;
    for (size_t k = 0; k < M; ++k) {   /* :169-178 */
        const float e = 0.5f * (float)(k * (double)k);
        Xc[k] = orc_cmul(a[(N - 1) + k], czt_chirp(e, argW, magW, +1));
    }
    free(a); free(b); free(Af); free(Bf);
    return 0;
}

/* czt.c:44-56: real input promoted to complex */
int orc_czt_real(const float* x, size_t N, size_t M, float w_re, float w_im, float a_re, float a_im, float* X) {
    if (!x || !X) return 1;
    float* xc = (float*)calloc(2 * (N ? N : 1), sizeof(float));
    if (!xc) return 4;
    for (size_t n = 0; n < N; ++n) xc[2 * n] = x[n];
    const int st = orc_czt_cpx(xc, N, M, w_re, w_im, a_re, a_im, X);
    free(xc);
    return st;
}

/* ---- cepstrum / minimum phase (src/envelope/cepstrum.c, minphase.c) ---- */
/* cepstrum.c:7-41: Re(IFFT(log(|FFT(x)| + 1e-12))) with C2C transforms */
int orc_cepstrum_real(const float* x, size_t n, float* c) {
    if (!x || !c) return 1;
    ocpx* t = (ocpx*)calloc(3 * (n ? n : 1), sizeof(ocpx));
    if (!t) return 4;
    ocpx *xin = t, *X = t + n, *Y = t + 2 * n;
    for (size_t i = 0; i < n; ++i) { xin[i].re = x[i]; xin[i].im = 0.0f; }
    orc_fft_c2c((const float*)xin, (float*)X, n, 1);
    for (size_t k = 0; k < n; ++k) {
        const float mag = sqrtf(X[k].re * X[k].re + X[k].im * X[k].im);
        Y[k].re = logf(mag + 1e-12f);
        Y[k].im = 0.0f;
    }
    orc_fft_c2c((const float*)Y, (float*)xin, n, -1);
    for (size_t i = 0; i < n; ++i) c[i] = xin[i].re;
    free(t);
    return 0;
}

/* cepstrum.c:48-57 / minphase.c:15-19: the causal fold of a cepstrum */
static void ceps_fold(const float* c, size_t n, ocpx* C) {
    const size_t nh = n / 2;
    for (size_t i = 0; i < n; ++i) { C[i].re = 0.0f; C[i].im = 0.0f; }
    if (n > 0) C[0].re = c[0];
    for (size_t i = 1; i < nh; ++i) C[i].re = 2 * c[i];
    if (n % 2 == 0 && nh < n) C[nh].re = 0.0f;
}

/* cepstrum.c:43-78: Re(IFFT(expf(Re FFT(fold(c))))) */
int orc_icepstrum_minphase(const float* c, size_t n, float* x) {
    if (!c || !x) return 1;
    ocpx* t = (ocpx*)calloc(3 * (n ? n : 1), sizeof(ocpx));
    if (!t) return 4;
    ocpx *C = t, *H = t + n, *h = t + 2 * n;
    ceps_fold(c, n, C);
    orc_fft_c2c((const float*)C, (float*)H, n, 1);
    for (size_t k = 0; k < n; ++k) { H[k].re = expf(H[k].re); H[k].im = 0.0f; }
    orc_fft_c2c((const float*)H, (float*)h, n, -1);
    for (size_t i = 0; i < n; ++i) x[i] = h[i].re;
    free(t);
    return 0;
}

/* minphase.c:7-31: spec[k] = ((float)exp((double)Re FFT(fold(c))[k]), 0) */
int orc_minphase_from_cepstrum(const float* c, size_t n, float* spec) {
    if (!c || !spec) return 1;
    ocpx* t = (ocpx*)calloc(2 * (n ? n : 1), sizeof(ocpx));
    if (!t) return 4;
    ocpx *C = t, *H = t + n;
    ceps_fold(c, n, C);
    orc_fft_c2c((const float*)C, (float*)H, n, 1);
    for (size_t k = 0; k < n; ++k) {
        spec[2 * k] = (float)exp((double)H[k].re);
        spec[2 * k + 1] = 0.0f;
    }
    free(t);
    return 0;
}

/* ---- spectral utilities (src/spectral/utils.c) ------------------------- */
/* :5-49 -- k = n/2; fftshift out = in[k..n) ++ in[0..k), ifftshift out = in[n-k..n) ++ in[0..n-k) */
int orc_fftshift(const float* in, float* out, size_t n, int cpx, int inverse) {
    if (!in || !out) return 1;
    if (n == 0) return 2;
    const size_t k = n / 2, w = cpx ? 2 : 1;
    const size_t first = inverse ? n - k : k;   /* index of in[] that lands at out[0] */
    memcpy(out, in + w * first, sizeof(float) * w * (n - first));
    memcpy(out + w * (n - first), in, sizeof(float) * w * first);
    return 0;
}

/* :51-61 */
int orc_phase_wrap(const float* in, float* out, size_t n) {
    if (!in || !out) return 1;
    for (size_t i = 0; i < n; ++i) {
        float x = in[i];
        while (x <= -kPi) x += kTwoPi;
        while (x > kPi) x -= kTwoPi;
        out[i] = x;
    }
    return 0;
}

/* :63-73 -- float accumulation left to right */
int orc_phase_unwrap(const float* in, float* out, size_t n) {
    if (!in || !out) return 1;
    if (n == 0) return 2;
    out[0] = in[0];
    for (size_t i = 1; i < n; ++i) {
        float delta = in[i] - in[i - 1];
        if (delta > kPi) delta -= kTwoPi;
        else if (delta < -kPi) delta += kTwoPi;
        out[i] = out[i - 1] + delta;
    }
    return 0;
}
