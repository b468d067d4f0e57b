/* dct.h -- DCT plans (reference include/vv_dsp/spectral/dct.h:13-53).
 * DCT-II forward: X[k] = sum x[n] cos(pi (n+1/2) k / N) (unnormalized);
 * BACKWARD of DCT-II/III is (2/N)(X0/2 + sum_k>=1 X[k] cos(pi k (n+1/2)/N)). */
#ifndef VV_DSP_SPECTRAL_DCT_H
#define VV_DSP_SPECTRAL_DCT_H
#include "vv_dsp/vv_dsp_types.h"
#include "vv_dsp/core/nan_policy.h"
#ifdef __cplusplus
extern "C" {
#endif
typedef enum vv_dsp_dct_type { VV_DSP_DCT_II = 2, VV_DSP_DCT_III = 3, VV_DSP_DCT_IV = 4 } vv_dsp_dct_type;
typedef enum vv_dsp_dct_dir { VV_DSP_DCT_FORWARD = +1, VV_DSP_DCT_BACKWARD = -1 } vv_dsp_dct_dir;
typedef struct vv_dsp_dct_plan vv_dsp_dct_plan;

VV_DSP_NODISCARD vv_dsp_status vv_dsp_dct_make_plan(size_t n, vv_dsp_dct_type type, vv_dsp_dct_dir dir,
                                                    vv_dsp_dct_plan** out_plan);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dct_execute(const vv_dsp_dct_plan* plan, const vv_dsp_real* in,
                                                  vv_dsp_real* out);
vv_dsp_status vv_dsp_dct_destroy(vv_dsp_dct_plan* plan);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dct_forward(size_t n, vv_dsp_dct_type type, const vv_dsp_real* in,
                                                  vv_dsp_real* out);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dct_inverse(size_t n, vv_dsp_dct_type type, const vv_dsp_real* in,
                                                  vv_dsp_real* out);
#ifdef __cplusplus
}
#endif
#endif
