/* fft_hip.c -- the HIP (gfx950) backend behind the FFT vtable.
 * Slot VV_DSP_FFT_BACKEND_HIP of the dispatcher; the vtable shape is the
 * reference's src/spectral/fft_backend.h:32-38.  Every call goes to the
 * extern "C" shim (include/vv_dsp_hip.h); there is no CPU path here.
 *
 * make_plan reads only the fields of the reference's 32-byte plan
 * (fft_backend.h:17-29), so this vtable can be registered in the reference's
 * own dispatcher; the batch comes from our
 * dispatcher through vv_amd_fft_pending_batch(), 1 otherwise. */
#include "fft_backend.h"
#include "vv_dsp_hip.h"

static vv_dsp_status hip_make_plan(const struct vv_dsp_fft_plan* spec, void** backend_data) {
    if (!spec || !backend_data) return VV_DSP_ERROR_NULL_POINTER;
    vvhip_fft* p = 0;
    int st = vvhip_fft_plan_create(spec->n, (int)spec->type, (int)spec->dir, vv_amd_fft_pending_batch(spec), &p);
    *backend_data = p;
    return (vv_dsp_status)st;
}

static vv_dsp_status hip_execute(const struct vv_dsp_fft_plan* spec, void* backend_data, const void* in, void* out) {
    if (!spec || !backend_data || !in || !out) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_fft_exec_host((vvhip_fft*)backend_data, in, out);
}

static void hip_free_plan(void* backend_data) {
    if (backend_data) vvhip_fft_plan_destroy((vvhip_fft*)backend_data);
}

static int hip_is_available(void) { return vvhip_available() > 0; }

const vv_dsp_fft_backend_vtable vv_dsp_fft_hip_vtable = {
    hip_make_plan, hip_execute, hip_free_plan, hip_is_available, "HIP-gfx950",
};
