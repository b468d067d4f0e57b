/* mel.c -- mel filterbank / log-mel / MFCC front-end (reference
 * src/features/mel.c, include/vv_dsp/features/mel.h).
 *
 * Host side: the HTK mel conversions and the triangular filterbank are setup
 * code and keep the reference's f32 arithmetic exactly (same operation order,
 * so the weights are bit-identical).  The per-frame work -- filterbank sums,
 * log, DCT-II, lifter -- runs on the GPU through the vvhip_mel_* shim
 * (mel_kernels.hip); there is no CPU compute path. */
#include "vv_dsp/features/mel.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "vv_dsp/vv_dsp_amd.h"
#include "vv_dsp_hip.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* mel.c:14-20 */
vv_dsp_real vv_dsp_hz_to_mel(vv_dsp_real hz) {
    return hz < 0.0f ? 0.0f : 2595.0f * log10f(1.0f + hz / 700.0f);
}

/* mel.c:22-28 */
vv_dsp_real vv_dsp_mel_to_hz(vv_dsp_real mel) {
    return mel < 0.0f ? 0.0f : 700.0f * (powf(10.0f, mel / 2595.0f) - 1.0f);
}

/* first index i with a[i] >= v (a ascending), mel.c:51-62 */
static size_t lower_bound_f(const float* a, size_t n, float v) {
    size_t lo = 0, hi = n;
    while (lo < hi) {
        const size_t mid = lo + (hi - lo) / 2;
        if (a[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

/* mel.c:66-193 */
vv_dsp_status vv_dsp_mel_filterbank_create(size_t n_fft, size_t n_mels, vv_dsp_real sample_rate, vv_dsp_real fmin,
                                           vv_dsp_real fmax, vv_dsp_mel_variant variant,
                                           vv_dsp_real** out_filterbank_weights, size_t* out_num_filters,
                                           size_t* out_filter_len) {
    if (!out_filterbank_weights || !out_num_filters || !out_filter_len) return VV_DSP_ERROR_NULL_POINTER;
    if (n_fft == 0 || n_mels == 0 || sample_rate <= 0.0f || fmin < 0.0f || fmax <= fmin)
        return VV_DSP_ERROR_INVALID_SIZE;
    if (fmax > sample_rate / 2.0f) return VV_DSP_ERROR_OUT_OF_RANGE;
    if (variant != VV_DSP_MEL_VARIANT_HTK) return VV_DSP_ERROR_OUT_OF_RANGE;
    const size_t nb = n_fft / 2 + 1;
    if (n_mels >= nb) return VV_DSP_ERROR_INVALID_SIZE;

    const size_t npts = n_mels + 2;
    float* fb = (float*)calloc(n_mels * nb, sizeof(float));
    float* pts = (float*)malloc(npts * sizeof(float));   /* mel points, then Hz */
    float* bins = (float*)malloc(nb * sizeof(float));
    if (!fb || !pts || !bins) {
        free(fb);
        free(pts);
        free(bins);
        return VV_DSP_ERROR_INTERNAL;
    }
    /* n_mels + 2 mel points evenly spaced over [mel(fmin), mel(fmax)] */
    const float m0 = vv_dsp_hz_to_mel(fmin), m1 = vv_dsp_hz_to_mel(fmax);
    const float dm = (m1 - m0) / (float)(npts - 1);
    for (size_t i = 0; i < npts; ++i) pts[i] = m0 + dm * (float)i;
    for (size_t i = 0; i < npts; ++i) pts[i] = vv_dsp_mel_to_hz(pts[i]);
    for (size_t k = 0; k < nb; ++k) bins[k] = (float)k * sample_rate / (float)n_fft;

    for (size_t m = 0; m < n_mels; ++m) {
        const float lo = pts[m], mid = pts[m + 1], hi = pts[m + 2];
        const size_t kl = lower_bound_f(bins, nb, lo), km = lower_bound_f(bins, nb, mid),
                     kh = lower_bound_f(bins, nb, hi);
        float* row = fb + m * nb;
        for (size_t k = kl; k < km && k < nb; ++k) row[k] = (bins[k] - lo) / (mid - lo);
        for (size_t k = km; k < kh && k < nb; ++k) row[k] = (hi - bins[k]) / (hi - mid);
        float total = 0.0f;   /* unit-sum normalisation over the whole row, in bin order */
        for (size_t k = 0; k < nb; ++k) total += row[k];
        if (total > 0.0f)
            for (size_t k = 0; k < nb; ++k) row[k] /= total;
    }
    free(pts);
    free(bins);
    *out_filterbank_weights = fb;
    *out_num_filters = n_mels;
    *out_filter_len = nb;
    return VV_DSP_OK;
}

void vv_dsp_mel_filterbank_free(vv_dsp_real* filterbank_weights, size_t n_mels) {
    (void)n_mels;
    free(filterbank_weights);
}

/* mel.c:204-245 on the GPU (vvhip_mel kind 0) */
vv_dsp_status vv_dsp_compute_log_mel_spectrogram(const vv_dsp_real* power_spectrogram, size_t num_frames,
                                                 size_t n_fft_bins, const vv_dsp_real* filterbank_weights,
                                                 size_t n_mels, vv_dsp_real log_epsilon,
                                                 vv_dsp_real* out_log_mel_spectrogram) {
    if (!power_spectrogram || !filterbank_weights || !out_log_mel_spectrogram) return VV_DSP_ERROR_NULL_POINTER;
    if (num_frames == 0 || n_fft_bins == 0 || n_mels == 0) return VV_DSP_ERROR_INVALID_SIZE;
    if (log_epsilon < 0.0f) return VV_DSP_ERROR_OUT_OF_RANGE;
    vvhip_mel* m = NULL;
    int st = vvhip_mel_create(filterbank_weights, n_mels, n_fft_bins, 0, 0.0f, log_epsilon, &m);
    if (st == VV_DSP_OK) st = vvhip_mel_host(m, power_spectrogram, num_frames, out_log_mel_spectrogram, 0);
    vvhip_mel_destroy(m);
    return (vv_dsp_status)st;
}

/* mel.c:249-309 on the GPU (vvhip_mel kind 2) */
vv_dsp_status vv_dsp_mfcc(const vv_dsp_real* log_mel_spectrogram, size_t num_frames, size_t n_mels,
                          size_t num_mfcc_coeffs, vv_dsp_dct_type dct_type, vv_dsp_real lifter_coeff,
                          vv_dsp_real* out_mfcc_coeffs) {
    if (!log_mel_spectrogram || !out_mfcc_coeffs) return VV_DSP_ERROR_NULL_POINTER;
    if (num_frames == 0 || n_mels == 0 || num_mfcc_coeffs == 0 || num_mfcc_coeffs > n_mels)
        return VV_DSP_ERROR_INVALID_SIZE;
    if (dct_type != VV_DSP_DCT_II || lifter_coeff < 0.0f) return VV_DSP_ERROR_OUT_OF_RANGE;
    vvhip_mel* m = NULL;
    int st = vvhip_mel_create(NULL, n_mels, 0, num_mfcc_coeffs, lifter_coeff, 0.0f, &m);
    if (st == VV_DSP_OK) st = vvhip_mel_host(m, log_mel_spectrogram, num_frames, out_mfcc_coeffs, 2);
    vvhip_mel_destroy(m);
    return (vv_dsp_status)st;
}

/* mel.c:314-331: the plan keeps the filterbank on the device */
struct vv_dsp_mfcc_plan {
    size_t n_fft, n_mels, num_mfcc_coeffs, n_fft_bins;
    vvhip_mel* dev;
};

/* mel.c:333-406 (same validation order and codes) */
vv_dsp_status vv_dsp_mfcc_init(size_t n_fft, size_t n_mels, size_t num_mfcc_coeffs, vv_dsp_real sample_rate,
                               vv_dsp_real fmin, vv_dsp_real fmax, vv_dsp_mel_variant variant,
                               vv_dsp_dct_type dct_type, vv_dsp_real lifter_coeff, vv_dsp_real log_epsilon,
                               vv_dsp_mfcc_plan** out_plan) {
    if (!out_plan) return VV_DSP_ERROR_NULL_POINTER;
    if (n_fft == 0 || n_mels == 0 || num_mfcc_coeffs == 0 || sample_rate <= 0.0f) return VV_DSP_ERROR_INVALID_SIZE;
    if (num_mfcc_coeffs > n_mels || fmin < 0.0f || fmax <= fmin || fmax > sample_rate / 2.0f)
        return VV_DSP_ERROR_OUT_OF_RANGE;
    vv_dsp_real* fb = NULL;
    size_t nf = 0, fl = 0;
    vv_dsp_status st = vv_dsp_mel_filterbank_create(n_fft, n_mels, sample_rate, fmin, fmax, variant, &fb, &nf, &fl);
    if (st != VV_DSP_OK) return st;
    /* the reference accepts any dct_type / lifter here and rejects them in
     * vv_dsp_mfcc at process time (mel.c:268-273); keep that split */
    vv_dsp_mfcc_plan* p = (vv_dsp_mfcc_plan*)calloc(1, sizeof(*p));
    if (!p) {
        free(fb);
        return VV_DSP_ERROR_INTERNAL;
    }
    p->n_fft = n_fft;
    p->n_mels = n_mels;
    p->num_mfcc_coeffs = num_mfcc_coeffs;
    p->n_fft_bins = fl;
    p->dev = NULL;
    int hs = VV_DSP_OK;
    if (dct_type == VV_DSP_DCT_II && lifter_coeff >= 0.0f && log_epsilon >= 0.0f)
        hs = vvhip_mel_create(fb, n_mels, fl, num_mfcc_coeffs, lifter_coeff, log_epsilon, &p->dev);
    free(fb);
    if (hs != VV_DSP_OK) {
        free(p);
        return (vv_dsp_status)hs;
    }
    *out_plan = p;
    return VV_DSP_OK;
}

/* mel.c:408-450: power [frames][n_fft/2+1] -> MFCC [frames][num_mfcc_coeffs] */
vv_dsp_status vv_dsp_mfcc_process(const vv_dsp_mfcc_plan* plan, const vv_dsp_real* power_spectrogram,
                                  size_t num_frames, vv_dsp_real* out_mfcc_coeffs) {
    if (!plan || !power_spectrogram || !out_mfcc_coeffs) return VV_DSP_ERROR_NULL_POINTER;
    if (num_frames == 0) return VV_DSP_ERROR_INVALID_SIZE;
    if (!plan->dev) return VV_DSP_ERROR_OUT_OF_RANGE;   /* dct_type / lifter / epsilon the reference rejects */
    return (vv_dsp_status)vvhip_mel_host(plan->dev, power_spectrogram, num_frames, out_mfcc_coeffs, 1);
}

vv_dsp_status vv_dsp_mfcc_destroy(vv_dsp_mfcc_plan* plan) {
    if (!plan) return VV_DSP_ERROR_NULL_POINTER;
    vvhip_mel_destroy(plan->dev);
    free(plan);
    return VV_DSP_OK;
}

/* ---- device-pointer batch API (vv_dsp_amd.h) ---- */
vv_dsp_status vv_dsp_mfcc_process_device(const vv_dsp_mfcc_plan* plan, const vv_dsp_real* d_power,
                                         size_t num_frames, vv_dsp_real* d_out_mfcc, void* stream) {
    if (!plan || !d_power || !d_out_mfcc) return VV_DSP_ERROR_NULL_POINTER;
    if (!plan->dev) return VV_DSP_ERROR_OUT_OF_RANGE;
    return (vv_dsp_status)vvhip_mel_device(plan->dev, d_power, num_frames, d_out_mfcc, 1, stream);
}

/* the plan's device tables, for the fused signal -> mel entries of stft.c */
__attribute__((visibility("hidden"))) vvhip_mel* vv_amd_mfcc_device_plan(const vv_dsp_mfcc_plan* plan) {
    return plan ? plan->dev : 0;
}

vv_dsp_status vv_dsp_log_mel_device(const vv_dsp_mfcc_plan* plan, const vv_dsp_real* d_power, size_t num_frames,
                                    vv_dsp_real* d_out_log_mel, void* stream) {
    if (!plan || !d_power || !d_out_log_mel) return VV_DSP_ERROR_NULL_POINTER;
    if (!plan->dev) return VV_DSP_ERROR_OUT_OF_RANGE;
    return (vv_dsp_status)vvhip_mel_device(plan->dev, d_power, num_frames, d_out_log_mel, 0, stream);
}

/* power rows row_pitch floats apart (vv_dsp_stft_power_pitched_device's layout) */
vv_dsp_status vv_dsp_mfcc_process_pitched_device(const vv_dsp_mfcc_plan* plan, const vv_dsp_real* d_power,
                                                 size_t num_frames, size_t row_pitch, vv_dsp_real* d_out_mfcc,
                                                 void* stream) {
    if (!plan || !d_power || !d_out_mfcc) return VV_DSP_ERROR_NULL_POINTER;
    if (!plan->dev) return VV_DSP_ERROR_OUT_OF_RANGE;
    if (row_pitch == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_mel_pitched_device(plan->dev, d_power, num_frames, row_pitch, d_out_mfcc, 1, stream);
}

vv_dsp_status vv_dsp_log_mel_pitched_device(const vv_dsp_mfcc_plan* plan, const vv_dsp_real* d_power,
                                            size_t num_frames, size_t row_pitch, vv_dsp_real* d_out_log_mel,
                                            void* stream) {
    if (!plan || !d_power || !d_out_log_mel) return VV_DSP_ERROR_NULL_POINTER;
    if (!plan->dev) return VV_DSP_ERROR_OUT_OF_RANGE;
    if (row_pitch == 0) return VV_DSP_ERROR_INVALID_SIZE;
    return (vv_dsp_status)vvhip_mel_pitched_device(plan->dev, d_power, num_frames, row_pitch, d_out_log_mel, 0,
                                                   stream);
}
