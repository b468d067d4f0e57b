/* fft.h -- vv-dsp FFT API (signatures of the reference's
 * include/vv_dsp/spectral/fft.h:34-252) with a fourth backend slot,
 * VV_DSP_FFT_BACKEND_HIP, served by hand-written gfx950 kernels.
 * Buffers: C2C cpx[n]->cpx[n]; R2C real[n]->cpx[n/2+1]; C2R cpx[n/2+1]->real[n].
 * Forward unscaled, backward scaled by 1/n. */
#ifndef VV_DSP_SPECTRAL_FFT_H
#define VV_DSP_SPECTRAL_FFT_H
#include "vv_dsp/vv_dsp_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef enum vv_dsp_fft_backend {
    VV_DSP_FFT_BACKEND_KISS = 0,
    VV_DSP_FFT_BACKEND_FFTW = 1,
    VV_DSP_FFT_BACKEND_FFTS = 2,
    VV_DSP_FFT_BACKEND_HIP = 3 /* MI355X / gfx950 */
} vv_dsp_fft_backend;

typedef enum vv_dsp_fftw_flag {
    VV_DSP_FFTW_ESTIMATE = 0,
    VV_DSP_FFTW_MEASURE = 1,
    VV_DSP_FFTW_PATIENT = 2
} vv_dsp_fftw_flag;

typedef enum vv_dsp_fft_dir { VV_DSP_FFT_FORWARD = +1, VV_DSP_FFT_BACKWARD = -1 } vv_dsp_fft_dir;
typedef enum vv_dsp_fft_type { VV_DSP_FFT_C2C = 0, VV_DSP_FFT_R2C = 1, VV_DSP_FFT_C2R = 2 } vv_dsp_fft_type;

typedef struct vv_dsp_fft_plan vv_dsp_fft_plan;

VV_DSP_NODISCARD vv_dsp_status vv_dsp_fft_set_backend(vv_dsp_fft_backend backend);
vv_dsp_fft_backend vv_dsp_fft_get_backend(void);
int vv_dsp_fft_is_backend_available(vv_dsp_fft_backend backend);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_fft_set_fftw_flag(vv_dsp_fftw_flag flag);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_fft_flush_fftw_cache(void);

VV_DSP_NODISCARD vv_dsp_status vv_dsp_fft_make_plan(size_t n, vv_dsp_fft_type type,
                                                    vv_dsp_fft_dir dir, vv_dsp_fft_plan** out_plan);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_fft_execute(const vv_dsp_fft_plan* plan, const void* in,
                                                  void* out);
vv_dsp_status vv_dsp_fft_destroy(vv_dsp_fft_plan* plan);

#ifdef __cplusplus
}
#endif
#endif
