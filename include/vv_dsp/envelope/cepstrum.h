/* cepstrum.h -- real cepstrum and its minimum-phase inverse
 * (reference include/vv_dsp/envelope/cepstrum.h:10-18). */
#ifndef VV_DSP_ENVELOPE_CEPSTRUM_H
#define VV_DSP_ENVELOPE_CEPSTRUM_H
#include <stddef.h>
#include "vv_dsp/vv_dsp_types.h"
#ifdef __cplusplus
extern "C" {
#endif
/* out_cep[n] = Re IFFT(log(|FFT(x)| + 1e-12)) */
vv_dsp_status vv_dsp_cepstrum_real(const vv_dsp_real* x, size_t n, vv_dsp_real* out_cep);
/* out_x[n] = Re IFFT(exp(Re FFT(fold(c)))), fold(c) = (c0, 2 c1 .. 2 c(n/2-1), 0 ..) */
vv_dsp_status vv_dsp_icepstrum_minphase(const vv_dsp_real* c, size_t n, vv_dsp_real* out_x);
#ifdef __cplusplus
}
#endif
#endif
