/* minphase.h -- minimum-phase spectrum from a real cepstrum
 * (reference include/vv_dsp/envelope/minphase.h:10-16). */
#ifndef VV_DSP_ENVELOPE_MINPHASE_H
#define VV_DSP_ENVELOPE_MINPHASE_H
#include <stddef.h>
#include "vv_dsp/vv_dsp_types.h"
#ifdef __cplusplus
extern "C" {
#endif
/* out_spec[k] = (exp(Re FFT(fold(c))[k]), 0), k < n */
vv_dsp_status vv_dsp_minphase_from_cepstrum(const vv_dsp_real* c, size_t n, vv_dsp_cpx* out_spec);
#ifdef __cplusplus
}
#endif
#endif
