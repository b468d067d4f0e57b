/* spectral_utils.c -- fftshift / ifftshift and phase wrap / unwrap on the
 * MI355X backend (C99).  Semantics and error codes of the reference's
 * src/spectral/utils.c:5-73; the element work runs on the GPU
 * (spectral_utils_kernels.hip, and phase_kernels.hip for the unwrap scan). */
#include "vv_dsp/vv_dsp_amd.h"
#include "vv_dsp/spectral.h"
#include "vv_dsp_hip.h"

int vv_dsp_spectral_dummy(void) { return 42; }

/* utils.c:5-19 / 21-33: NULL -> NULL_POINTER, n == 0 -> INVALID_SIZE */
static vv_dsp_status shift(const void* in, void* out, size_t n, int cpx, int inverse) {
    if (!in || !out) return VV_DSP_ERROR_NULL_POINTER;
    if (n == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_fftshift_host(in, out, n, cpx, inverse);
}

vv_dsp_status vv_dsp_fftshift_real(const vv_dsp_real* in, vv_dsp_real* out, size_t n) { return shift(in, out, n, 0, 0); }
vv_dsp_status vv_dsp_ifftshift_real(const vv_dsp_real* in, vv_dsp_real* out, size_t n) { return shift(in, out, n, 0, 1); }
vv_dsp_status vv_dsp_fftshift_cpx(const vv_dsp_cpx* in, vv_dsp_cpx* out, size_t n) { return shift(in, out, n, 1, 0); }
vv_dsp_status vv_dsp_ifftshift_cpx(const vv_dsp_cpx* in, vv_dsp_cpx* out, size_t n) { return shift(in, out, n, 1, 1); }

/* utils.c:51-61: n == 0 is OK (nothing to do) */
vv_dsp_status vv_dsp_phase_wrap(const vv_dsp_real* in, vv_dsp_real* out, size_t n) {
    if (!in || !out) return VV_DSP_ERROR_NULL_POINTER;
    if (n == 0) return VV_DSP_OK;
    return (vv_dsp_status)vvhip_phase_wrap_host(in, out, n);
}

/* utils.c:63-73 */
vv_dsp_status vv_dsp_phase_unwrap(const vv_dsp_real* in, vv_dsp_real* out, size_t n) {
    if (!in || !out) return VV_DSP_ERROR_NULL_POINTER;
    if (n == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_phase_unwrap_host(in, out, n);
}

/* batched device rows (vv_dsp_amd.h) */
vv_dsp_status vv_dsp_fftshift_device(const void* d_in, void* d_out, size_t n, size_t batch, int is_complex,
                                     int inverse, void* stream) {
    if (!d_in || !d_out) return VV_DSP_ERROR_NULL_POINTER;
    if (n == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_fftshift_device(d_in, d_out, n, batch, is_complex ? 1 : 0, inverse ? 1 : 0, stream);
}

vv_dsp_status vv_dsp_phase_wrap_device(const vv_dsp_real* d_in, vv_dsp_real* d_out, size_t count, void* stream) {
    if (!d_in || !d_out) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_phase_wrap_device(d_in, d_out, count, stream);
}

vv_dsp_status vv_dsp_phase_unwrap_device(const vv_dsp_real* d_in, vv_dsp_real* d_out, size_t n, size_t batch,
                                         void* stream) {
    if (!d_in || !d_out) return VV_DSP_ERROR_NULL_POINTER;
    if (n == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_phase_unwrap_device(d_in, d_out, n, batch, stream);
}
