/* utils.h -- spectral data-format helpers (reference include/vv_dsp/spectral/utils.h:13-28). */
#ifndef VV_DSP_SPECTRAL_UTILS_H
#define VV_DSP_SPECTRAL_UTILS_H
#include <stddef.h>
#include "vv_dsp/vv_dsp_types.h"
#ifdef __cplusplus
extern "C" {
#endif
/* out-of-place half-length rotations: fftshift moves bin n/2 to index 0, ifftshift undoes it */
vv_dsp_status vv_dsp_fftshift_real(const vv_dsp_real* in, vv_dsp_real* out, size_t n);
vv_dsp_status vv_dsp_ifftshift_real(const vv_dsp_real* in, vv_dsp_real* out, size_t n);
vv_dsp_status vv_dsp_fftshift_cpx(const vv_dsp_cpx* in, vv_dsp_cpx* out, size_t n);
vv_dsp_status vv_dsp_ifftshift_cpx(const vv_dsp_cpx* in, vv_dsp_cpx* out, size_t n);
/* wrap to (-pi, pi] */
vv_dsp_status vv_dsp_phase_wrap(const vv_dsp_real* in, vv_dsp_real* out, size_t n);
/* continuous phase from wrapped input: out[0] = in[0], neighbour steps wrapped once */
vv_dsp_status vv_dsp_phase_unwrap(const vv_dsp_real* in, vv_dsp_real* out, size_t n);
#ifdef __cplusplus
}
#endif
#endif
