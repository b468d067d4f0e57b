/* stft.h -- vv-dsp STFT API (reference include/vv_dsp/spectral/stft.h:15-56). */
#ifndef VV_DSP_SPECTRAL_STFT_H
#define VV_DSP_SPECTRAL_STFT_H
#include "vv_dsp/vv_dsp_types.h"
#include "vv_dsp/spectral/fft.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vv_dsp_stft vv_dsp_stft;

typedef enum vv_dsp_stft_window {
    VV_DSP_STFT_WIN_BOXCAR = 0,
    VV_DSP_STFT_WIN_HANN = 1,
    VV_DSP_STFT_WIN_HAMMING = 2
} vv_dsp_stft_window;

typedef struct vv_dsp_stft_params {
    size_t fft_size;
    size_t hop_size;
    vv_dsp_stft_window window;
} vv_dsp_stft_params;

VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_create(const vv_dsp_stft_params* params, vv_dsp_stft** out);
vv_dsp_status vv_dsp_stft_destroy(vv_dsp_stft* h);
/* one frame: real[fft_size] (windowed internally) -> cpx[fft_size] */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_process(vv_dsp_stft* h, const vv_dsp_real* in, vv_dsp_cpx* out);
/* out_add[i] += Re(IFFT(in))[i] * w[i]; norm_add[i] += w[i]^2 (norm_add may be NULL) */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_reconstruct(vv_dsp_stft* h, const vv_dsp_cpx* in,
                                                       vv_dsp_real* out_add, vv_dsp_real* norm_add);
/* magnitudes [frames][fft_size]; frames = n < fft_size ? 1 : 1 + (n - fft_size + hop) / hop */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_spectrogram(vv_dsp_stft* h, const vv_dsp_real* signal,
                                                       size_t n, vv_dsp_real* out_mag, size_t* out_frames);

#ifdef __cplusplus
}
#endif
#endif
