/* fir.c -- FIR filtering on the MI355X backend (C99).
 *
 * vv_dsp_fir_design_lowpass and the state helpers keep the reference's
 * arithmetic and semantics (src/filter/fir.c:8-73, 137-158): coefficient
 * design is one-time host setup.  The filtering itself runs on the GPU:
 *   vv_dsp_fir_apply_fft (:75-135)  -> overlap-save FFT convolution, zero state;
 *   vv_dsp_fir_apply     (:160-196) -> direct form in the reference's summation
 *                                      order (bit-identical), continuing from and
 *                                      updating the ring-buffer history;
 *   vv_dsp_filtfilt_fir  (filter/common.c:23-80) -> reflection-padded forward and
 *                                      backward direct form, bit-identical. */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "vv_dsp/vv_dsp_amd.h"
#include "vv_dsp/filter/common.h"
#include "vv_dsp/filter/fir.h"
#include "vv_dsp_hip.h"

static const vv_dsp_real kPiF = (vv_dsp_real)3.141592653589793238462643383279502884;
static const double kTwoPiD = 2.0 * 3.141592653589793238462643383279502884;

static vv_dsp_real sinc_r(vv_dsp_real v) {
    if (v == (vv_dsp_real)0) return 1.0f;
    return (vv_dsp_real)(sinf(kPiF * v) / (kPiF * v));
}

static vv_dsp_status design_window(vv_dsp_real* w, size_t N, vv_dsp_window_type type) {
    const vv_dsp_real twopi = (vv_dsp_real)kTwoPiD;
    for (size_t n = 0; n < N; ++n) {
        switch (type) {
            case VV_DSP_WINDOW_RECTANGULAR: w[n] = 1.0f; break;
            case VV_DSP_WINDOW_HAMMING:
                w[n] = (vv_dsp_real)(0.54f - 0.46f * cosf(twopi * (vv_dsp_real)n / (vv_dsp_real)(N - 1)));
                break;
            case VV_DSP_WINDOW_HANNING:
                w[n] = (vv_dsp_real)(0.5f - 0.5f * cosf(twopi * (vv_dsp_real)n / (vv_dsp_real)(N - 1)));
                break;
            case VV_DSP_WINDOW_BLACKMAN: {
                const double c1 = (vv_dsp_real)cosf((vv_dsp_real)(kTwoPiD * (double)n / (double)(N - 1)));
                const double c2 = (vv_dsp_real)cosf((vv_dsp_real)(2.0 * kTwoPiD * (double)n / (double)(N - 1)));
                w[n] = (vv_dsp_real)(0.42 - 0.5 * c1 + 0.08 * c2);
                break;
            }
            default: return VV_DSP_ERROR_INTERNAL;
        }
    }
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_fir_design_lowpass(vv_dsp_real* h, size_t M, vv_dsp_real fc, vv_dsp_window_type wt) {
    if (!h) return VV_DSP_ERROR_NULL_POINTER;
    if (M == 0) return VV_DSP_ERROR_INVALID_SIZE;
    if (!(fc > (vv_dsp_real)0 && fc < (vv_dsp_real)1)) return VV_DSP_ERROR_OUT_OF_RANGE;
    const vv_dsp_real centre = (vv_dsp_real)(M - 1) / (vv_dsp_real)2;
    for (size_t n = 0; n < M; ++n) h[n] = 2 * fc * sinc_r(2 * fc * ((vv_dsp_real)n - centre));
    vv_dsp_real* w = (vv_dsp_real*)malloc(M * sizeof(vv_dsp_real));
    if (!w) return VV_DSP_ERROR_INTERNAL;
    vv_dsp_status s = design_window(w, M, wt);
    if (s == VV_DSP_OK)
        for (size_t n = 0; n < M; ++n) h[n] *= w[n];
    free(w);
    return s;
}

vv_dsp_status vv_dsp_fir_state_init(vv_dsp_fir_state* st, size_t num_taps) {
    if (!st) return VV_DSP_ERROR_NULL_POINTER;
    if (num_taps == 0) return VV_DSP_ERROR_INVALID_SIZE;
    memset(st, 0, sizeof(*st));
    st->num_taps = num_taps;
    st->history_size = num_taps - 1;
    if (st->history_size) {
        st->history = (vv_dsp_real*)calloc(st->history_size, sizeof(vv_dsp_real));
        if (!st->history) return VV_DSP_ERROR_INTERNAL;
    }
    return VV_DSP_OK;
}

void vv_dsp_fir_state_free(vv_dsp_fir_state* st) {
    if (!st) return;
    free(st->history);
    st->history = NULL;
    st->history_size = 0;
    st->history_idx = 0;
    st->num_taps = 0;
}

vv_dsp_status vv_dsp_fir_apply_fft(vv_dsp_fir_state* st, const vv_dsp_real* h, const vv_dsp_real* x,
                                   vv_dsp_real* y, size_t n) {
    if (!st || !h || !x || !y) return VV_DSP_ERROR_NULL_POINTER;
    if (st->num_taps == 0) return VV_DSP_ERROR_INVALID_SIZE;
    vvhip_fir* f = NULL;
    vv_dsp_status s = (vv_dsp_status)vvhip_fir_create(h, st->num_taps, &f);
    if (s != VV_DSP_OK) return s;
    s = (vv_dsp_status)vvhip_fir_apply_host(f, x, y, n, NULL, 0);
    vvhip_fir_destroy(f);
    return s;
}

vv_dsp_status vv_dsp_fir_apply(vv_dsp_fir_state* st, const vv_dsp_real* h, const vv_dsp_real* x, vv_dsp_real* y,
                               size_t n) {
    if (!st || !h || !x || !y) return VV_DSP_ERROR_NULL_POINTER;
    if (st->num_taps == 0) return VV_DSP_ERROR_INVALID_SIZE;
    const size_t hs = st->history_size;
    /* with no history the reference uses h[0] only (fir.c:176-185) */
    const size_t taps = hs ? st->num_taps : 1;
    if (hs && (hs != st->num_taps - 1 || !st->history)) return VV_DSP_ERROR_INVALID_SIZE;
    if (n == 0) return VV_DSP_OK;
    vv_dsp_real* prefix = NULL;
    if (hs) {
        prefix = (vv_dsp_real*)malloc(hs * sizeof(vv_dsp_real));
        if (!prefix) return VV_DSP_ERROR_INTERNAL;
        for (size_t j = 0; j < hs; ++j) prefix[j] = st->history[(st->history_idx + j) % hs]; /* oldest first */
    }
    vvhip_fir* f = NULL;
    vv_dsp_status s = (vv_dsp_status)vvhip_fir_create(h, taps, &f);
    if (s == VV_DSP_OK) s = (vv_dsp_status)vvhip_fir_apply_host(f, x, y, n, prefix, 1);
    vvhip_fir_destroy(f);
    free(prefix);
    if (s != VV_DSP_OK) return s;
    if (hs) { /* the ring after n pushes, exactly as the reference leaves it */
        const size_t first = (n > hs) ? n - hs : 0;
        for (size_t i = first; i < n; ++i) st->history[(st->history_idx + i) % hs] = x[i];
        st->history_idx = (st->history_idx + n) % hs;
    }
    return VV_DSP_OK;
}

/* ---- additive device plan (vv_dsp_amd.h) ---- */
struct vv_dsp_fir_plan {
    vvhip_fir* dev;
};

vv_dsp_status vv_dsp_fir_plan_create(const vv_dsp_real* coeffs, size_t num_taps, vv_dsp_fir_plan** out) {
    if (!out || !coeffs) return VV_DSP_ERROR_NULL_POINTER;
    *out = NULL;
    if (num_taps == 0) return VV_DSP_ERROR_INVALID_SIZE;
    vv_dsp_fir_plan* p = (vv_dsp_fir_plan*)calloc(1, sizeof(*p));
    if (!p) return VV_DSP_ERROR_INTERNAL;
    vv_dsp_status s = (vv_dsp_status)vvhip_fir_create(coeffs, num_taps, &p->dev);
    if (s != VV_DSP_OK) {
        free(p);
        return s;
    }
    *out = p;
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_fir_plan_destroy(vv_dsp_fir_plan* p) {
    if (!p) return VV_DSP_ERROR_NULL_POINTER;
    vvhip_fir_destroy(p->dev);
    free(p);
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_fir_apply_fft_device(vv_dsp_fir_plan* p, const vv_dsp_real* d_x, vv_dsp_real* d_y, size_t n,
                                          size_t nch, size_t x_stride, size_t y_stride, void* stream) {
    if (!p || !d_x || !d_y) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_fir_apply_device(p->dev, d_x, d_y, n, nch, x_stride, y_stride, NULL, 0, stream);
}

vv_dsp_status vv_dsp_fir_apply_direct_device(vv_dsp_fir_plan* p, const vv_dsp_real* d_x, vv_dsp_real* d_y,
                                             size_t n, size_t nch, size_t x_stride, size_t y_stride,
                                             void* stream) {
    if (!p || !d_x || !d_y) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_fir_apply_device(p->dev, d_x, d_y, n, nch, x_stride, y_stride, NULL, 1, stream);
}

vv_dsp_status vv_dsp_filtfilt_fir_device(vv_dsp_fir_plan* p, const vv_dsp_real* d_x, vv_dsp_real* d_y, size_t n,
                                         size_t nch, size_t x_stride, size_t y_stride, void* stream) {
    if (!p || !d_x || !d_y) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_fir_filtfilt_device(p->dev, d_x, d_y, n, nch, x_stride, y_stride, stream);
}

/* filter/common.c:23-80.  Argument checks in the reference's order; an empty
 * signal is a no-op (the reference's reflection would read input[-1]). */
vv_dsp_status vv_dsp_filtfilt_fir(const vv_dsp_real* coeffs, size_t num_taps, const vv_dsp_real* input,
                                  vv_dsp_real* output, size_t num_samples) {
    if (!coeffs || !input || !output) return VV_DSP_ERROR_NULL_POINTER;
    if (num_taps == 0) return VV_DSP_ERROR_INVALID_SIZE;
    if (num_samples == 0) return VV_DSP_OK;
    vvhip_fir* f = NULL;
    vv_dsp_status s = (vv_dsp_status)vvhip_fir_create(coeffs, num_taps, &f);
    if (s != VV_DSP_OK) return s;
    s = (vv_dsp_status)vvhip_fir_filtfilt_host(f, input, output, num_samples);
    vvhip_fir_destroy(f);
    return s;
}
