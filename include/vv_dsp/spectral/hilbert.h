/* hilbert.h -- analytic signal (reference include/vv_dsp/spectral/hilbert.h:15). */
#ifndef VV_DSP_SPECTRAL_HILBERT_H
#define VV_DSP_SPECTRAL_HILBERT_H
#include "vv_dsp/vv_dsp_types.h"
#ifdef __cplusplus
extern "C" {
#endif
vv_dsp_status vv_dsp_hilbert_analytic(const vv_dsp_real* input, size_t N, vv_dsp_cpx* analytic_output);
#ifdef __cplusplus
}
#endif
#endif
