/* fir.h -- FIR API (reference include/vv_dsp/filter/fir.h:22-53 and the window
 * enum of filter/common.h:14-19). */
#ifndef VV_DSP_FILTER_FIR_H
#define VV_DSP_FILTER_FIR_H
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

typedef struct {
    vv_dsp_real* history;  /* ring buffer of the last num_taps-1 inputs */
    size_t history_size;
    size_t history_idx;    /* next write position (= oldest sample) */
    size_t num_taps;
} vv_dsp_fir_state;

vv_dsp_status vv_dsp_fir_design_lowpass(vv_dsp_real* coeffs, size_t num_taps, vv_dsp_real cutoff_norm,
                                        vv_dsp_window_type window_type);
vv_dsp_status vv_dsp_fir_state_init(vv_dsp_fir_state* state, size_t num_taps);
void vv_dsp_fir_state_free(vv_dsp_fir_state* state);
/* streaming direct form; continues from and updates state->history */
vv_dsp_status vv_dsp_fir_apply(vv_dsp_fir_state* state, const vv_dsp_real* coeffs, const vv_dsp_real* input,
                               vv_dsp_real* output, size_t num_samples);
/* zero-state linear convolution, first num_samples outputs (state->num_taps used only) */
vv_dsp_status vv_dsp_fir_apply_fft(vv_dsp_fir_state* state, const vv_dsp_real* coeffs,
                                   const vv_dsp_real* input, vv_dsp_real* output, size_t num_samples);
#ifdef __cplusplus
}
#endif
#endif
