/* vv_dsp_types.h -- core types of the vv-dsp C API, ABI-identical to the
 * reference (include/vv_dsp/vv_dsp_types.h:70-128): f32 real, interleaved
 * {re, im} complex, int-sized status enum. */
#ifndef VV_DSP_TYPES_H
#define VV_DSP_TYPES_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__) || defined(__clang__)
#define VV_DSP_NODISCARD __attribute__((warn_unused_result))
#else
#define VV_DSP_NODISCARD
#endif

#ifdef VV_DSP_USE_DOUBLE
#error "the MI355X backend implements the default f32 build of vv-dsp only"
#endif
typedef float vv_dsp_real;

typedef struct vv_dsp_cpx {
    vv_dsp_real re;
    vv_dsp_real im;
} vv_dsp_cpx;

typedef enum vv_dsp_status {
    VV_DSP_OK = 0,
    VV_DSP_ERROR_NULL_POINTER = 1,
    VV_DSP_ERROR_INVALID_SIZE = 2,
    VV_DSP_ERROR_OUT_OF_RANGE = 3,
    VV_DSP_ERROR_INTERNAL = 4,
    VV_DSP_ERROR_NAN_INF = 5,
    VV_DSP_ERROR_UNSUPPORTED = 6
} vv_dsp_status;

#ifdef __cplusplus
}
#endif
#endif
