/* hilbert.c -- analytic signal on the MI355X backend (C99).
 * Semantics of the reference's src/spectral/hilbert.c:14-75 (R2C, one-sided
 * mask, inverse C2C scaled 1/N); instantaneous phase/frequency (:77-113) run
 * as a GPU scan over the same double-precision increments. */
#include "vv_dsp/vv_dsp_amd.h"
#include "vv_dsp/spectral/hilbert.h"
#include "vv_dsp_hip.h"

vv_dsp_status vv_dsp_hilbert_analytic(const vv_dsp_real* input, size_t N, vv_dsp_cpx* analytic_output) {
    if (!input || !analytic_output) return VV_DSP_ERROR_NULL_POINTER;
    if (N == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_hilbert_host(input, N, (float*)analytic_output);
}

vv_dsp_status vv_dsp_hilbert_analytic_device(const vv_dsp_real* d_x, size_t N, size_t batch, vv_dsp_cpx* d_z,
                                             void* stream) {
    if (!d_x || !d_z) return VV_DSP_ERROR_NULL_POINTER;
    if (N == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_hilbert_device(d_x, N, batch, (float*)d_z, stream);
}
