/* cepstrum.c -- real cepstrum and minimum phase on the MI355X backend (C99).
 * Semantics of the reference's src/envelope/cepstrum.c:7-78 and
 * src/envelope/minphase.c:7-31; every transform and element-wise step runs on
 * the GPU (vvhip_cepstrum_*, czt_kernels.hip).  The reference reports any FFT
 * plan failure, n = 0 included, as VV_DSP_ERROR_INTERNAL (cepstrum.c:10-11,
 * minphase.c:10). */
#include "vv_dsp/vv_dsp_amd.h"
#include "vv_dsp/envelope/cepstrum.h"
#include "vv_dsp/envelope/minphase.h"
#include "vv_dsp_hip.h"

vv_dsp_status vv_dsp_cepstrum_real(const vv_dsp_real* x, size_t n, vv_dsp_real* out_cep) {
    if (!x || !out_cep) return VV_DSP_ERROR_NULL_POINTER;
    if (n == 0) return VV_DSP_ERROR_INTERNAL;
    return (vv_dsp_status)vvhip_cepstrum_host(x, n, out_cep);
}

vv_dsp_status vv_dsp_icepstrum_minphase(const vv_dsp_real* c, size_t n, vv_dsp_real* out_x) {
    if (!c || !out_x) return VV_DSP_ERROR_NULL_POINTER;
    if (n == 0) return VV_DSP_ERROR_INTERNAL;
    return (vv_dsp_status)vvhip_icepstrum_minphase_host(c, n, out_x);
}

vv_dsp_status vv_dsp_minphase_from_cepstrum(const vv_dsp_real* c, size_t n, vv_dsp_cpx* out_spec) {
    if (!c || !out_spec) return VV_DSP_ERROR_NULL_POINTER;
    if (n == 0) return VV_DSP_ERROR_INTERNAL;
    return (vv_dsp_status)vvhip_minphase_from_cepstrum_host(c, n, (float*)out_spec);
}

/* batched device rows (vv_dsp_amd.h) */
vv_dsp_status vv_dsp_cepstrum_real_device(const vv_dsp_real* d_x, size_t n, size_t batch, vv_dsp_real* d_cep,
                                          void* stream) {
    if (!d_x || !d_cep) return VV_DSP_ERROR_NULL_POINTER;
    if (n == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_cepstrum_device(d_x, n, batch, d_cep, stream);
}

vv_dsp_status vv_dsp_icepstrum_minphase_device(const vv_dsp_real* d_c, size_t n, size_t batch, vv_dsp_real* d_x,
                                               void* stream) {
    if (!d_c || !d_x) return VV_DSP_ERROR_NULL_POINTER;
    if (n == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_icepstrum_minphase_device(d_c, n, batch, d_x, stream);
}

vv_dsp_status vv_dsp_minphase_from_cepstrum_device(const vv_dsp_real* d_c, size_t n, size_t batch,
                                                   vv_dsp_cpx* d_spec, void* stream) {
    if (!d_c || !d_spec) return VV_DSP_ERROR_NULL_POINTER;
    if (n == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_minphase_from_cepstrum_device(d_c, n, batch, (float*)d_spec, stream);
}
