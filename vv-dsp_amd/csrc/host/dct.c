/* dct.c -- DCT plans on the MI355X backend (C99).
 * Validation and NaN-policy behaviour of the reference's src/spectral/dct.c:70-153;
 * power-of-two DCT-II (and its DCT-III inverse) run as an N-point real FFT with
 * Makhoul's permutation, other sizes/types as a GPU O(N^2) kernel with f64
 * accumulation. */
#include <stdlib.h>

#include "vv_dsp/vv_dsp_amd.h"
#include "vv_dsp/spectral/dct.h"
#include "vv_dsp_hip.h"

struct vv_dsp_dct_plan {
    size_t n;
    vv_dsp_dct_type type;
    vv_dsp_dct_dir dir;
};

/* NaN policy, per thread as the reference's (src/core/nan_policy.c:11-31,
 * _Thread_local under gnu99).  Weak so that the reference's core module, when
 * linked too, provides the single definition. */
static __thread vv_dsp_nan_policy_e g_policy = VV_DSP_NAN_POLICY_PROPAGATE;
__attribute__((weak)) void vv_dsp_set_nan_policy(vv_dsp_nan_policy_e policy) {
    if (policy >= VV_DSP_NAN_POLICY_PROPAGATE && policy <= VV_DSP_NAN_POLICY_CLAMP) g_policy = policy;
}
__attribute__((weak)) vv_dsp_nan_policy_e vv_dsp_get_nan_policy(void) { return g_policy; }

vv_dsp_status vv_dsp_dct_make_plan(size_t n, vv_dsp_dct_type type, vv_dsp_dct_dir dir, vv_dsp_dct_plan** out_plan) {
    if (!out_plan) return VV_DSP_ERROR_NULL_POINTER;
    *out_plan = NULL;
    if (n == 0) return VV_DSP_ERROR_INVALID_SIZE;
    if (type != VV_DSP_DCT_II && type != VV_DSP_DCT_III && type != VV_DSP_DCT_IV) return VV_DSP_ERROR_OUT_OF_RANGE;
    if (dir != VV_DSP_DCT_FORWARD && dir != VV_DSP_DCT_BACKWARD) return VV_DSP_ERROR_OUT_OF_RANGE;
    vv_dsp_dct_plan* p = (vv_dsp_dct_plan*)malloc(sizeof(*p));
    if (!p) return VV_DSP_ERROR_INTERNAL;
    p->n = n;
    p->type = type;
    p->dir = dir;
    *out_plan = p;
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_dct_execute(const vv_dsp_dct_plan* plan, const vv_dsp_real* in, vv_dsp_real* out) {
    if (!plan || !in || !out) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_dct_host(in, out, plan->n, (int)plan->type, (int)plan->dir,
                                         (int)vv_dsp_get_nan_policy());
}

vv_dsp_status vv_dsp_dct_execute_device(const vv_dsp_dct_plan* plan, const vv_dsp_real* d_in, vv_dsp_real* d_out,
                                        size_t batch, void* stream) {
    if (!plan || !d_in || !d_out) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_dct_device(d_in, d_out, plan->n, batch, (int)plan->type, (int)plan->dir,
                                           (int)vv_dsp_get_nan_policy(), stream);
}

vv_dsp_status vv_dsp_dct_destroy(vv_dsp_dct_plan* plan) {
    if (!plan) return VV_DSP_ERROR_NULL_POINTER;
    free(plan);
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_dct_forward(size_t n, vv_dsp_dct_type type, const vv_dsp_real* in, vv_dsp_real* out) {
    vv_dsp_dct_plan* p = NULL;
    vv_dsp_status s = vv_dsp_dct_make_plan(n, type, VV_DSP_DCT_FORWARD, &p);
    if (s != VV_DSP_OK) return s;
    s = vv_dsp_dct_execute(p, in, out);
    (void)vv_dsp_dct_destroy(p);
    return s;
}

vv_dsp_status vv_dsp_dct_inverse(size_t n, vv_dsp_dct_type type, const vv_dsp_real* in, vv_dsp_real* out) {
    vv_dsp_dct_plan* p = NULL;
    vv_dsp_status s = vv_dsp_dct_make_plan(n, type, VV_DSP_DCT_BACKWARD, &p);
    if (s != VV_DSP_OK) return s;
    s = vv_dsp_dct_execute(p, in, out);
    (void)vv_dsp_dct_destroy(p);
    return s;
}
