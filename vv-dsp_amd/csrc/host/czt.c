/* czt.c -- chirp-z transform on the MI355X backend (C99).
 * Semantics of the reference's src/spectral/czt.c: the arc parameters
 * (:22-42) are scalar setup and restate the reference's float arithmetic; the
 * transform (:44-178) runs on the GPU (vvhip_czt_*: chirp pre-multiply, FFT,
 * chirp-spectrum product, inverse FFT, post-multiply; czt_kernels.hip), with
 * chirps tabulated in extended precision. */
#include <math.h>
#include <stdlib.h>

#include "vv_dsp/vv_dsp_amd.h"
#include "vv_dsp/spectral/czt.h"
#include "vv_dsp_hip.h"

#define CZT_PI_D 3.141592653589793238462643383279502884

/* czt.c:22-42 */
vv_dsp_status vv_dsp_czt_params_for_freq_range(vv_dsp_real f_start, vv_dsp_real f_end, size_t M, vv_dsp_real fs,
                                               vv_dsp_real* W_real, vv_dsp_real* W_imag, vv_dsp_real* A_real,
                                               vv_dsp_real* A_imag) {
    if (!W_real || !W_imag || !A_real || !A_imag) return VV_DSP_ERROR_NULL_POINTER;
    if (M == 0 || fs <= (vv_dsp_real)0) return VV_DSP_ERROR_INVALID_SIZE;
    const vv_dsp_real delta = (f_end - f_start) / (vv_dsp_real)M;
    const vv_dsp_real theta = (vv_dsp_real)(-2.0 * CZT_PI_D * (double)delta / (double)fs);
    *W_real = cosf(theta);
    *W_imag = sinf(theta);
    const vv_dsp_real phi0 = (vv_dsp_real)(-2.0 * CZT_PI_D * (double)f_start / (double)fs);
    *A_real = cosf(phi0);
    *A_imag = sinf(phi0);
    return VV_DSP_OK;
}

/* czt.c:58-63 argument checks, then the GPU transform */
vv_dsp_status vv_dsp_czt_exec_cpx(const vv_dsp_cpx* x, size_t N, size_t M, vv_dsp_real W_re, vv_dsp_real W_im,
                                  vv_dsp_real A_re, vv_dsp_real A_im, vv_dsp_cpx* X) {
    if (!x || !X) return VV_DSP_ERROR_NULL_POINTER;
    if (N == 0 || M == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_czt_exec_host(x, 0, N, M, W_re, W_im, A_re, A_im, X);
}

/* czt.c:44-56 */
vv_dsp_status vv_dsp_czt_exec_real(const vv_dsp_real* x, size_t N, size_t M, vv_dsp_real W_re, vv_dsp_real W_im,
                                   vv_dsp_real A_re, vv_dsp_real A_im, vv_dsp_cpx* X) {
    if (!x || !X) return VV_DSP_ERROR_NULL_POINTER;
    if (N == 0 || M == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_czt_exec_host(x, 1, N, M, W_re, W_im, A_re, A_im, X);
}

/* batched device plan (vv_dsp_amd.h) */
struct vv_dsp_czt_plan {
    vvhip_czt* h;
};

vv_dsp_status vv_dsp_czt_plan_create(size_t N, size_t M, vv_dsp_real W_re, vv_dsp_real W_im, vv_dsp_real A_re,
                                     vv_dsp_real A_im, vv_dsp_czt_plan** out) {
    if (!out) return VV_DSP_ERROR_NULL_POINTER;
    *out = NULL;
    vvhip_czt* h = NULL;
    const int st = vvhip_czt_create(N, M, W_re, W_im, A_re, A_im, &h);
    if (st) return (vv_dsp_status)st;
    vv_dsp_czt_plan* p = (vv_dsp_czt_plan*)malloc(sizeof(*p));
    if (!p) {
        vvhip_czt_destroy(h);
        return VV_DSP_ERROR_INTERNAL;
    }
    p->h = h;
    *out = p;
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_czt_plan_destroy(vv_dsp_czt_plan* p) {
    if (p) {
        vvhip_czt_destroy(p->h);
        free(p);
    }
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_czt_execute_device(const vv_dsp_czt_plan* p, const void* d_x, int real_input, size_t batch,
                                        vv_dsp_cpx* d_X, void* stream) {
    if (!p || !d_x || !d_X) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_czt_exec_device(p->h, d_x, real_input ? 1 : 0, batch, d_X, stream);
}
