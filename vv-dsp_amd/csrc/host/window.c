/* window.c -- boxcar / Hann / Hamming tables (C99), the windows the STFT
 * handle uses.  One-time host setup with the reference's own f32 arithmetic
 * (src/window/window.c:9-49: validation order, N == 1 -> 1, the step
 * (float)(2 pi) / (float)(N-1) times (float)n through cosf), so the tables are
 * bit-identical to the reference's and every STFT frame is windowed by the same
 * bits.  The tables are applied on the GPU inside the STFT kernels. */
#include <math.h>

#include "vv_dsp/window.h"

static vv_dsp_status check_args(size_t N, const vv_dsp_real* out) {
    if (!out) return VV_DSP_ERROR_NULL_POINTER;
    if (N == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return VV_DSP_OK;
}

static vv_dsp_status raised_cosine(size_t N, vv_dsp_real* out, vv_dsp_real a, vv_dsp_real b) {
    vv_dsp_status s = check_args(N, out);
    if (s != VV_DSP_OK) return s;
    if (N == 1) {
        out[0] = (vv_dsp_real)1.0;
        return VV_DSP_OK;
    }
    const vv_dsp_real step = (vv_dsp_real)(2.0 * 3.141592653589793238462643383279502884) / (vv_dsp_real)(N - 1);
    for (size_t n = 0; n < N; ++n) out[n] = a - b * cosf(step * (vv_dsp_real)n);
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_window_boxcar(size_t N, vv_dsp_real* out) {
    vv_dsp_status s = check_args(N, out);
    if (s != VV_DSP_OK) return s;
    for (size_t n = 0; n < N; ++n) out[n] = (vv_dsp_real)1.0;
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_window_hann(size_t N, vv_dsp_real* out) {
    return raised_cosine(N, out, (vv_dsp_real)0.5, (vv_dsp_real)0.5);
}

vv_dsp_status vv_dsp_window_hamming(size_t N, vv_dsp_real* out) {
    return raised_cosine(N, out, (vv_dsp_real)0.54, (vv_dsp_real)0.46);
}
