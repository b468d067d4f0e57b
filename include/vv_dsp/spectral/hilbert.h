/* hilbert.h -- analytic signal, instantaneous phase and frequency
 * (reference include/vv_dsp/spectral/hilbert.h:11-28). */
#ifndef VV_DSP_SPECTRAL_HILBERT_H
#define VV_DSP_SPECTRAL_HILBERT_H
#include "vv_dsp/vv_dsp_types.h"
#ifdef __cplusplus
extern "C" {
#endif
/* input real[N] -> analytic_output complex[N] */
vv_dsp_status vv_dsp_hilbert_analytic(const vv_dsp_real* input, size_t N, vv_dsp_cpx* analytic_output);
/* analytic_input complex[N] -> phase_output real[N], unwrapped (radians) */
vv_dsp_status vv_dsp_instantaneous_phase(const vv_dsp_cpx* analytic_input, size_t N, vv_dsp_real* phase_output);
/* unwrapped_phase_input real[N] -> freq_output real[N] in Hz, freq_output[0] = 0 */
vv_dsp_status vv_dsp_instantaneous_frequency(const vv_dsp_real* unwrapped_phase_input, size_t N,
                                             double sample_rate, vv_dsp_real* freq_output);
#ifdef __cplusplus
}
#endif
#endif
