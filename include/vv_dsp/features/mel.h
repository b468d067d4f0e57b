/* mel.h -- mel filterbank, log-mel spectrogram and MFCC (reference
 * include/vv_dsp/features/mel.h:12-170; src/features/mel.c).
 *
 * Same functions, argument meaning and error codes as the reference.  The
 * filterbank is built on the host with the reference's arithmetic (bit-identical
 * weights); the per-frame work (filterbank sums, log, DCT-II, lifter) runs on
 * the GPU.  Only the HTK mel variant exists in the reference (mel.c:88-91). */
#ifndef VV_DSP_FEATURES_MEL_H
#define VV_DSP_FEATURES_MEL_H

#include <stddef.h>

#include "vv_dsp/spectral/dct.h"
#include "vv_dsp/vv_dsp_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef enum vv_dsp_mel_variant {
    VV_DSP_MEL_VARIANT_HTK = 0,
    VV_DSP_MEL_VARIANT_SLANEY = 1 /* rejected with OUT_OF_RANGE, as in the reference */
} vv_dsp_mel_variant;

typedef struct vv_dsp_mfcc_plan vv_dsp_mfcc_plan;

/* 2595 log10(1 + hz/700); negative input -> 0 */
vv_dsp_real vv_dsp_hz_to_mel(vv_dsp_real hz);
/* 700 (10^(mel/2595) - 1); negative input -> 0 */
vv_dsp_real vv_dsp_mel_to_hz(vv_dsp_real mel);

/* n_mels triangular filters over n_fft/2+1 bins, each normalised to unit sum;
 * *out_filterbank_weights is n_mels x (n_fft/2+1), freed with
 * vv_dsp_mel_filterbank_free. */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_mel_filterbank_create(size_t n_fft, size_t n_mels,
                                                            vv_dsp_real sample_rate, vv_dsp_real fmin,
                                                            vv_dsp_real fmax, vv_dsp_mel_variant variant,
                                                            vv_dsp_real** out_filterbank_weights,
                                                            size_t* out_num_filters, size_t* out_filter_len);
void vv_dsp_mel_filterbank_free(vv_dsp_real* filterbank_weights, size_t n_mels);

/* out[f][m] = log(sum_k power[f][k] * fb[m][k] + log_epsilon) */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_compute_log_mel_spectrogram(const vv_dsp_real* power_spectrogram,
                                                                  size_t num_frames, size_t n_fft_bins,
                                                                  const vv_dsp_real* filterbank_weights,
                                                                  size_t n_mels, vv_dsp_real log_epsilon,
                                                                  vv_dsp_real* out_log_mel_spectrogram);

/* per frame: DCT-II of the log-mel row (vv_dsp_dct_forward), first
 * num_mfcc_coeffs, then c[i] *= 1 + (L/2) sin(pi i / L) for i >= 1 when L > 0 */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_mfcc(const vv_dsp_real* log_mel_spectrogram, size_t num_frames,
                                           size_t n_mels, size_t num_mfcc_coeffs, vv_dsp_dct_type dct_type,
                                           vv_dsp_real lifter_coeff, vv_dsp_real* out_mfcc_coeffs);

VV_DSP_NODISCARD vv_dsp_status vv_dsp_mfcc_init(size_t n_fft, size_t n_mels, size_t num_mfcc_coeffs,
                                                vv_dsp_real sample_rate, vv_dsp_real fmin, vv_dsp_real fmax,
                                                vv_dsp_mel_variant variant, vv_dsp_dct_type dct_type,
                                                vv_dsp_real lifter_coeff, vv_dsp_real log_epsilon,
                                                vv_dsp_mfcc_plan** out_plan);
/* power spectrogram [num_frames][n_fft/2+1] -> MFCC [num_frames][num_mfcc_coeffs] */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_mfcc_process(const vv_dsp_mfcc_plan* plan,
                                                   const vv_dsp_real* power_spectrogram, size_t num_frames,
                                                   vv_dsp_real* out_mfcc_coeffs);
vv_dsp_status vv_dsp_mfcc_destroy(vv_dsp_mfcc_plan* plan);

#ifdef __cplusplus
}
#endif
#endif
