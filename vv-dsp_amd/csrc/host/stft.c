/* stft.c -- vv-dsp STFT handle on the MI355X backend (C99).
 * API and validation of the reference's src/spectral/stft.c:30-144; the window
 * table is generated here with the reference's own arithmetic
 * (src/window/window.c:16-49: symmetric, N==1 -> 1) so its bits match, and all
 * transform work (window multiply, FFT, magnitude, ISTFT accumulate) runs in
 * the fused gfx950 kernels behind include/vv_dsp_hip.h. */
#include <math.h>
#include <stdlib.h>

#include "vv_dsp/vv_dsp_amd.h"
#include "vv_dsp/spectral/stft.h"
#include "vv_dsp/window.h"
#include "vv_dsp_hip.h"

struct vv_dsp_stft {
    size_t nfft;
    size_t hop;
    vv_dsp_stft_window win_type;
    vv_dsp_real* win;
    vvhip_stft* dev;
};

/* stft.c:21-28: the window by type (window.c:16-49 arithmetic, vv_dsp/window.h) */
static vv_dsp_status make_window(vv_dsp_stft_window wt, size_t n, vv_dsp_real* w) {
    switch (wt) {
        case VV_DSP_STFT_WIN_BOXCAR: return vv_dsp_window_boxcar(n, w);
        case VV_DSP_STFT_WIN_HANN: return vv_dsp_window_hann(n, w);
        case VV_DSP_STFT_WIN_HAMMING: return vv_dsp_window_hamming(n, w);
        default: return VV_DSP_ERROR_OUT_OF_RANGE;
    }
}

vv_dsp_status vv_dsp_stft_create(const vv_dsp_stft_params* params, vv_dsp_stft** out) {
    if (!out || !params) return VV_DSP_ERROR_NULL_POINTER;
    *out = NULL;
    if (params->fft_size == 0 || params->hop_size == 0 || params->hop_size > params->fft_size)
        return VV_DSP_ERROR_INVALID_SIZE;
    vv_dsp_stft* h = (vv_dsp_stft*)calloc(1, sizeof(*h));
    if (!h) return VV_DSP_ERROR_INTERNAL;
    h->nfft = params->fft_size;
    h->hop = params->hop_size;
    h->win_type = params->window;
    h->win = (vv_dsp_real*)malloc(sizeof(vv_dsp_real) * h->nfft);
    if (!h->win) {
        free(h);
        return VV_DSP_ERROR_INTERNAL;
    }
    vv_dsp_status s = make_window(h->win_type, h->nfft, h->win);
    if (s == VV_DSP_OK) s = (vv_dsp_status)vvhip_stft_create(h->nfft, h->hop, h->win, &h->dev);
    if (s != VV_DSP_OK) {
        free(h->win);
        free(h);
        return s;
    }
    *out = h;
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_stft_destroy(vv_dsp_stft* h) {
    if (!h) return VV_DSP_ERROR_NULL_POINTER;
    vvhip_stft_destroy(h->dev);
    free(h->win);
    free(h);
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_stft_process(vv_dsp_stft* h, const vv_dsp_real* in, vv_dsp_cpx* out) {
    if (!h || !in || !out) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_stft_process_host(h->dev, in, (float*)out);
}

vv_dsp_status vv_dsp_stft_reconstruct(vv_dsp_stft* h, const vv_dsp_cpx* in, vv_dsp_real* out_add,
                                      vv_dsp_real* norm_add) {
    if (!h || !in || !out_add) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_stft_reconstruct_host(h->dev, (const float*)in, out_add, norm_add);
}

vv_dsp_status vv_dsp_stft_spectrogram(vv_dsp_stft* h, const vv_dsp_real* signal, size_t n, vv_dsp_real* out_mag,
                                      size_t* out_frames) {
    if (!h || !signal || !out_mag || !out_frames) return VV_DSP_ERROR_NULL_POINTER;
    if (h->nfft == 0 || h->hop == 0) return VV_DSP_ERROR_INVALID_SIZE;
    *out_frames = vvhip_stft_num_frames(n, h->nfft, h->hop);
    return (vv_dsp_status)vvhip_stft_spectrogram_host(h->dev, signal, n, out_mag);
}

/* ---- additive device-pointer entry points (vv_dsp_amd.h) ---- */
vv_dsp_status vv_dsp_stft_spectrogram_device(vv_dsp_stft* h, const vv_dsp_real* d_signal, size_t n, size_t nch,
                                             size_t ch_stride, vv_dsp_real* d_out_mag, size_t out_ch_stride,
                                             void* stream, size_t* out_frames) {
    if (!h || !d_signal || !d_out_mag) return VV_DSP_ERROR_NULL_POINTER;
    if (out_frames) *out_frames = vvhip_stft_num_frames(n, h->nfft, h->hop);
    return (vv_dsp_status)vvhip_stft_spectrogram_device(h->dev, d_signal, n, nch, ch_stride, d_out_mag,
                                                        out_ch_stride, 0, stream);
}

vv_dsp_status vv_dsp_stft_spectrum_device(vv_dsp_stft* h, const vv_dsp_real* d_signal, size_t n, size_t nch,
                                          size_t ch_stride, vv_dsp_cpx* d_out, size_t out_ch_stride, void* stream,
                                          size_t* out_frames) {
    if (!h || !d_signal || !d_out) return VV_DSP_ERROR_NULL_POINTER;
    if (out_frames) *out_frames = vvhip_stft_num_frames(n, h->nfft, h->hop);
    return (vv_dsp_status)vvhip_stft_spectrogram_device(h->dev, d_signal, n, nch, ch_stride, d_out,
                                                        out_ch_stride, 1, stream);
}

vv_dsp_status vv_dsp_stft_power_device(vv_dsp_stft* h, const vv_dsp_real* d_signal, size_t n, size_t nch,
                                       size_t ch_stride, vv_dsp_real* d_out_power, size_t out_ch_stride,
                                       void* stream, size_t* out_frames) {
    if (!h || !d_signal || !d_out_power) return VV_DSP_ERROR_NULL_POINTER;
    if (out_frames) *out_frames = vvhip_stft_num_frames(n, h->nfft, h->hop);
    return (vv_dsp_status)vvhip_stft_spectrogram_device(h->dev, d_signal, n, nch, ch_stride, d_out_power,
                                                        out_ch_stride, 2, stream);
}

vv_dsp_status vv_dsp_stft_power_pitched_device(vv_dsp_stft* h, const vv_dsp_real* d_signal, size_t n, size_t nch,
                                               size_t ch_stride, vv_dsp_real* d_out_power, size_t out_ch_stride,
                                               size_t row_pitch, void* stream, size_t* out_frames) {
    if (!h || !d_signal || !d_out_power) return VV_DSP_ERROR_NULL_POINTER;
    if (out_frames) *out_frames = vvhip_stft_num_frames(n, h->nfft, h->hop);
    return (vv_dsp_status)vvhip_stft_power_pitched_device(h->dev, d_signal, n, nch, ch_stride, d_out_power,
                                                          out_ch_stride, row_pitch, stream);
}

__attribute__((visibility("hidden"))) vvhip_mel* vv_amd_mfcc_device_plan(const vv_dsp_mfcc_plan* plan);

static vv_dsp_status stft_mel(vv_dsp_stft* h, const vv_dsp_mfcc_plan* plan, const vv_dsp_real* d_signal, size_t n,
                              size_t nch, size_t ch_stride, vv_dsp_real* d_out, size_t out_ch_stride, void* stream,
                              size_t* out_frames, int kind) {
    if (!h || !plan || !d_signal || !d_out) return VV_DSP_ERROR_NULL_POINTER;
    vvhip_mel* m = vv_amd_mfcc_device_plan(plan);
    if (!m) return VV_DSP_ERROR_OUT_OF_RANGE;
    if (out_frames) *out_frames = vvhip_stft_num_frames(n, h->nfft, h->hop);
    return (vv_dsp_status)vvhip_stft_mel_device(h->dev, m, d_signal, n, nch, ch_stride, d_out, out_ch_stride, kind,
                                                stream);
}

vv_dsp_status vv_dsp_stft_log_mel_device(vv_dsp_stft* h, const vv_dsp_mfcc_plan* plan, const vv_dsp_real* d_signal,
                                         size_t n, size_t nch, size_t ch_stride, vv_dsp_real* d_out,
                                         size_t out_ch_stride, void* stream, size_t* out_frames) {
    return stft_mel(h, plan, d_signal, n, nch, ch_stride, d_out, out_ch_stride, stream, out_frames, 0);
}

vv_dsp_status vv_dsp_stft_mfcc_device(vv_dsp_stft* h, const vv_dsp_mfcc_plan* plan, const vv_dsp_real* d_signal,
                                      size_t n, size_t nch, size_t ch_stride, vv_dsp_real* d_out, size_t out_ch_stride,
                                      void* stream, size_t* out_frames) {
    return stft_mel(h, plan, d_signal, n, nch, ch_stride, d_out, out_ch_stride, stream, out_frames, 1);
}

vv_dsp_status vv_dsp_stft_frames_range_device(vv_dsp_stft* h, const vv_dsp_real* d_signal, size_t n, size_t nch,
                                              size_t ch_stride, size_t frame0, size_t nframes, void* d_out,
                                              size_t out_ch_stride, int out_kind, void* stream) {
    if (!h || !d_signal || !d_out) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_stft_spectrogram_range_device(h->dev, d_signal, n, nch, ch_stride, frame0, nframes,
                                                              d_out, out_ch_stride, out_kind, stream);
}

vv_dsp_status vv_dsp_stft_process_device(vv_dsp_stft* h, const vv_dsp_real* d_frames, size_t count,
                                         vv_dsp_cpx* d_spec, void* stream) {
    if (!h || !d_frames || !d_spec) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_stft_process_device(h->dev, d_frames, count, (float*)d_spec, stream);
}

vv_dsp_status vv_dsp_stft_reconstruct_device(vv_dsp_stft* h, const vv_dsp_cpx* d_spec, size_t count,
                                             vv_dsp_real* d_out_add, vv_dsp_real* d_norm_add, void* stream) {
    if (!h || !d_spec || !d_out_add) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_stft_reconstruct_device(h->dev, (const float*)d_spec, count, h->hop, d_out_add,
                                                        d_norm_add, stream);
}

/* ---- multi-GPU layout (vv_dsp_amd.h) ---- */
vv_dsp_status vv_dsp_stft_get_sizes(const vv_dsp_stft* h, size_t* fft_size, size_t* hop_size) {
    if (!h) return VV_DSP_ERROR_NULL_POINTER;
    if (fft_size) *fft_size = h->nfft;
    if (hop_size) *hop_size = h->hop;
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_stft_channel_shard_device(vv_dsp_stft* h, int device, const vv_dsp_real* d_signal, size_t n,
                                               size_t count, size_t ch_stride, int out_kind, void* d_out,
                                               size_t out_ch_stride, void* stream, size_t* out_frames) {
    if (!h || !d_signal || !d_out) return VV_DSP_ERROR_NULL_POINTER;
    if (out_kind < 0 || out_kind > 2) return VV_DSP_ERROR_OUT_OF_RANGE;
    int prev = 0;
    vv_dsp_status st = (vv_dsp_status)vvhip_get_device(&prev);
    if (st != VV_DSP_OK) return st;
    st = (vv_dsp_status)vvhip_set_device(device);
    if (st != VV_DSP_OK) return st;
    if (out_frames) *out_frames = vvhip_stft_num_frames(n, h->nfft, h->hop);
    st = (vv_dsp_status)vvhip_stft_spectrogram_device(h->dev, d_signal, n, count, ch_stride, d_out, out_ch_stride,
                                                      out_kind, stream);
    vv_dsp_status st2 = (vv_dsp_status)vvhip_set_device(prev);
    return st != VV_DSP_OK ? st : st2;
}
