/* spectral.h -- umbrella header of the spectral module (reference
 * include/vv_dsp/spectral.h:14-60): FFT, spectral utilities, STFT, DCT, CZT and
 * Hilbert. */
#ifndef VV_DSP_SPECTRAL_H
#define VV_DSP_SPECTRAL_H
#ifdef __cplusplus
extern "C" {
#endif
/* build check of the module, returns 42 as the reference's (spectral.c:3-5) */
int vv_dsp_spectral_dummy(void);
#ifdef __cplusplus
}
#endif
#include "vv_dsp/spectral/fft.h"
#include "vv_dsp/spectral/utils.h"
#include "vv_dsp/spectral/stft.h"
#include "vv_dsp/spectral/dct.h"
#include "vv_dsp/spectral/czt.h"
#include "vv_dsp/spectral/hilbert.h"
#endif
