/* window.h -- the STFT's analysis/synthesis windows (reference
 * include/vv_dsp/window.h, the boxcar / Hann / Hamming declarations;
 * src/window/window.c:16-49).  Symmetric windows, w[n] = w[N-1-n], N == 1 -> 1.
 * The reference's other eleven windows are not part of this backend (they
 * feed no transform on the spectral path). */
#ifndef VV_DSP_WINDOW_H
#define VV_DSP_WINDOW_H
#include "vv_dsp/vv_dsp_types.h"
#ifdef __cplusplus
extern "C" {
#endif

/* w[n] = 1 */
vv_dsp_status vv_dsp_window_boxcar(size_t N, vv_dsp_real* out);
/* w[n] = 0.5 - 0.5 cos(2 pi n / (N-1))   (f32 arithmetic, cosf) */
vv_dsp_status vv_dsp_window_hann(size_t N, vv_dsp_real* out);
/* w[n] = 0.54 - 0.46 cos(2 pi n / (N-1)) */
vv_dsp_status vv_dsp_window_hamming(size_t N, vv_dsp_real* out);

#ifdef __cplusplus
}
#endif
#endif
