/* czt.h -- chirp-z transform (reference include/vv_dsp/spectral/czt.h:10-43).
 * X[k] = sum_{n=0}^{N-1} x[n] A^-n W^(nk), k < M: the points z_k = A W^-k
 * (scipy.signal.czt convention). */
#ifndef VV_DSP_SPECTRAL_CZT_H
#define VV_DSP_SPECTRAL_CZT_H
#include <stddef.h>
#include "vv_dsp/vv_dsp_types.h"
#ifdef __cplusplus
extern "C" {
#endif
/* (W, A) sampling the unit-circle arc f_start .. f_end (Hz) at M points:
 * W = exp(-j 2 pi delta / fs), delta = (f_end - f_start) / M; A = exp(-j 2 pi f_start / fs) */
vv_dsp_status vv_dsp_czt_params_for_freq_range(vv_dsp_real f_start, vv_dsp_real f_end, size_t M,
                                               vv_dsp_real sampling_rate, vv_dsp_real* W_real, vv_dsp_real* W_imag,
                                               vv_dsp_real* A_real, vv_dsp_real* A_imag);
/* complex input x[N] -> X[M] */
vv_dsp_status vv_dsp_czt_exec_cpx(const vv_dsp_cpx* input, size_t N, size_t M, vv_dsp_real W_real,
                                  vv_dsp_real W_imag, vv_dsp_real A_real, vv_dsp_real A_imag, vv_dsp_cpx* output);
/* real input x[N] (imaginary parts 0) -> X[M] */
vv_dsp_status vv_dsp_czt_exec_real(const vv_dsp_real* input, size_t N, size_t M, vv_dsp_real W_real,
                                   vv_dsp_real W_imag, vv_dsp_real A_real, vv_dsp_real A_imag, vv_dsp_cpx* output);
#ifdef __cplusplus
}
#endif
#endif
