/* common.h -- filter utilities (reference include/vv_dsp/filter/common.h:14-31):
 * the FIR design window enum and zero-phase FIR filtering. */
#ifndef VV_DSP_FILTER_COMMON_H
#define VV_DSP_FILTER_COMMON_H
#include "vv_dsp/vv_dsp_types.h"
#ifdef __cplusplus
extern "C" {
#endif
#ifndef VV_DSP_WINDOW_TYPE_DEFINED
#define VV_DSP_WINDOW_TYPE_DEFINED
typedef enum {
    VV_DSP_WINDOW_RECTANGULAR = 0,
    VV_DSP_WINDOW_HAMMING = 1,
    VV_DSP_WINDOW_HANNING = 2,
    VV_DSP_WINDOW_BLACKMAN = 3
} vv_dsp_window_type;
#endif

/* Zero-phase FIR: reflection padding of num_taps-1 samples, the filter forward,
 * reversed, forward again, reversed back; output = the centre num_samples.
 * Runs on the GPU with the reference's summation order (bit-identical). */
vv_dsp_status vv_dsp_filtfilt_fir(const vv_dsp_real* coeffs, size_t num_taps, const vv_dsp_real* input,
                                  vv_dsp_real* output, size_t num_samples);

#ifdef __cplusplus
}
#endif
#endif
