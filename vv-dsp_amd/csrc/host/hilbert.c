/* hilbert.c -- analytic signal on the MI355X backend (C99).
 * Semantics of the reference's src/spectral/hilbert.c:14-75 (R2C, one-sided
 * mask, inverse C2C scaled 1/N); instantaneous phase (:77-96) runs as a GPU
 * prefix sum over the same double-precision increments (phase_kernels.hip),
 * instantaneous frequency (:98-113) as a GPU elementwise difference. */
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

/* hilbert.c:77-96 */
vv_dsp_status vv_dsp_instantaneous_phase(const vv_dsp_cpx* analytic_input, size_t N, vv_dsp_real* phase_output) {
    if (!analytic_input || !phase_output) return VV_DSP_ERROR_NULL_POINTER;
    if (N == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_inst_phase_host((const float*)analytic_input, N, phase_output);
}

/* hilbert.c:98-113 */
vv_dsp_status vv_dsp_instantaneous_frequency(const vv_dsp_real* unwrapped_phase_input, size_t N, double sample_rate,
                                             vv_dsp_real* freq_output) {
    if (!unwrapped_phase_input || !freq_output) return VV_DSP_ERROR_NULL_POINTER;
    if (N == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_inst_freq_host(unwrapped_phase_input, N, sample_rate, freq_output);
}

vv_dsp_status vv_dsp_instantaneous_phase_device(const vv_dsp_cpx* d_analytic, size_t N, size_t batch,
                                                vv_dsp_real* d_phase, void* stream) {
    if (!d_analytic || !d_phase) return VV_DSP_ERROR_NULL_POINTER;
    if (N == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_inst_phase_device((const float*)d_analytic, N, batch, d_phase, stream);
}

vv_dsp_status vv_dsp_instantaneous_frequency_device(const vv_dsp_real* d_phase, size_t N, size_t batch,
                                                    double sample_rate, vv_dsp_real* d_freq, void* stream) {
    if (!d_phase || !d_freq) return VV_DSP_ERROR_NULL_POINTER;
    if (N == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_inst_freq_device(d_phase, N, batch, sample_rate, d_freq, stream);
}
