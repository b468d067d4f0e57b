/* nan_policy.h -- NaN/Inf policy used by the DCT (reference
 * include/vv_dsp/core/nan_policy.h:33-38).  Exported weakly by the MI355X
 * library so a program that also links the reference's core module keeps one
 * policy global. */
#ifndef VV_DSP_CORE_NAN_POLICY_H
#define VV_DSP_CORE_NAN_POLICY_H
#include "vv_dsp/vv_dsp_types.h"
#ifdef __cplusplus
extern "C" {
#endif
typedef enum vv_dsp_nan_policy {
    VV_DSP_NAN_POLICY_PROPAGATE = 0,
    VV_DSP_NAN_POLICY_IGNORE = 1,
    VV_DSP_NAN_POLICY_ERROR = 2,
    VV_DSP_NAN_POLICY_CLAMP = 3
} vv_dsp_nan_policy_e;
void vv_dsp_set_nan_policy(vv_dsp_nan_policy_e policy);
vv_dsp_nan_policy_e vv_dsp_get_nan_policy(void);
#ifdef __cplusplus
}
#endif
#endif
