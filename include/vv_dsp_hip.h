/*
 * vv_dsp_hip.h -- the thin extern "C" HIP shim of the MI355X (gfx950) backend.
 *
 * Plain C ABI: opaque handles, raw pointers, sizes, int status codes with the
 * values of the reference's vv_dsp_status (include/vv_dsp/vv_dsp_types.h:120-128:
 * 0 OK, 1 NULL_POINTER, 2 INVALID_SIZE, 3 OUT_OF_RANGE, 4 INTERNAL,
 * 5 NAN_INF, 6 UNSUPPORTED).  No HIP or torch types appear here: streams are
 * passed as `void*` (a hipStream_t; NULL = the handle's own stream).
 *
 * Two calling conventions per operation:
 *   *_host   : host pointers, synchronous (what the reference's C API needs);
 *   *_device : device pointers, asynchronous on the given stream (the batched
 *              entry points; inputs already resident in HBM).
 *
 * The C99 front-end in vv-dsp_amd/csrc/host/ (the reference's vv_dsp_* API) is
 * the only intended caller of the *_host functions; the *_device functions are
 * also reachable through include/vv_dsp/vv_dsp_amd.h.
 *
 * Reference interfaces each group replaces:
 *   vvhip_fft_*  : the FFT backend vtable slot, src/spectral/fft_backend.h:32-38
 *                  (make_plan / execute / free_plan / is_available)
 *   vvhip_stft_* : src/spectral/stft.c:30-144 (create, process, reconstruct, spectrogram)
 *   vvhip_fir_*  : src/filter/fir.c:75-196 (apply_fft, apply), filter/common.c:23-80 (filtfilt)
 *   vvhip_hilbert_*: src/spectral/hilbert.c:14-75
 *   vvhip_dct_*  : src/spectral/dct.c:86-136
 *   vvhip_czt_*  : src/spectral/czt.c:44-178 (exec_cpx, exec_real)
 *   vvhip_fftshift_* / _phase_wrap_* / _phase_unwrap_*: src/spectral/utils.c:5-73
 *   vvhip_cepstrum_* / _icepstrum_minphase_* / _minphase_from_cepstrum_*:
 *                  src/envelope/cepstrum.c:7-78, src/envelope/minphase.c:7-31
 */
#ifndef VV_DSP_HIP_H
#define VV_DSP_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif
#pragma GCC visibility push(default)

typedef struct vvhip_fft vvhip_fft;
typedef struct vvhip_stft vvhip_stft;
typedef struct vvhip_fir vvhip_fir;
typedef struct vvhip_mel vvhip_mel;
typedef struct vvhip_czt vvhip_czt;

/* Number of usable HIP devices (0 when none: every other call then fails). */
int vvhip_available(void);
/* Text of the last error seen by this thread ("" if none). */
const char* vvhip_last_error(void);

/* A/B switches and path counters (csrc/hip/debug.hip), for tests and the
 * scripts/kbench.py timing harness; the defaults are the adopted kernels.
 *   vvhip_debug_set("STFT_DYN", 0)  selects a launcher alternative (the names
 *       are the VVHIP_* switches of DESIGN.md, with or without the prefix);
 *       0 on success, -1 for an unknown name or a negative value;
 *   vvhip_debug_clear(name)  back to the default (NULL: every knob, and every
 *       path counter to 0);
 *   vvhip_debug_get(name)  a knob's value (-1 unset) or a path counter
 *       ("STAT_STFT_DYN", "STAT_FIR_DYN", "STAT_FIR_STATIC", "STAT_MEL_FUSED",
 *       "STAT_MEL_SPLIT": launches of that path since the last clear); -2 unknown.
 * The environment is read once per process, and only with VVHIP_AB=1 set. */
int vvhip_debug_set(const char* name, long long value);
int vvhip_debug_clear(const char* name);
long long vvhip_debug_get(const char* name);
/* Build identification, e.g. "vvhip gfx950 ROCm 7.2". */
const char* vvhip_version(void);

/* ---- device memory helpers (tests / host front-end) ---- */
void* vvhip_malloc(size_t bytes);
void vvhip_free(void* p);
int vvhip_memcpy_h2d(void* dst, const void* src, size_t bytes);
int vvhip_memcpy_d2h(void* dst, const void* src, size_t bytes);
int vvhip_memset(void* dst, int value, size_t bytes);
/* stream-ordered scratch on the stream's device (hipMallocAsync / hipFreeAsync)
 * and a device-to-device copy on a stream */
int vvhip_malloc_async(void** p, size_t bytes, void* stream);
int vvhip_free_async(void* p, void* stream);
int vvhip_memcpy_d2d_async(void* dst, const void* src, size_t bytes, void* stream);
/* the device of a stream (NULL: the current device's null stream), and a
 * device-side wait of `waiter` for everything enqueued on `producer` so far
 * (an event on the producer's device; no host synchronisation) */
int vvhip_stream_device(void* stream, int* device);
int vvhip_stream_wait(void* waiter, void* producer);
/* sets the text vvhip_last_error() returns on this thread (host front-end errors) */
void vvhip_set_error(const char* what);
int vvhip_stream_sync(void* stream);
int vvhip_device_sync(void);
/* the calling thread's current HIP device (hipSetDevice / hipGetDevice) */
int vvhip_set_device(int device);
int vvhip_get_device(int* device);

/* ---- FFT: replaces the backend vtable slot (fft_backend.h:32-38) ----
 * type: 0 C2C, 1 R2C, 2 C2R (fft.h:152-156); dir: +1 forward, -1 backward.
 * Layout per transform as fft.h:169-172; `batch` transforms back to back. */
int vvhip_fft_plan_create(size_t n, int type, int dir, size_t batch, vvhip_fft** out);
int vvhip_fft_exec_host(vvhip_fft* plan, const void* in, void* out);
int vvhip_fft_exec_device(vvhip_fft* plan, const void* d_in, void* d_out, size_t batch,
                          void* stream);
void vvhip_fft_plan_destroy(vvhip_fft* plan);

/* ---- STFT (stft.c) ---- window: nfft floats computed by the caller. */
int vvhip_stft_create(size_t nfft, size_t hop, const float* window, vvhip_stft** out);
void vvhip_stft_destroy(vvhip_stft* h);
/* frames = n < nfft ? 1 : 1 + (n - nfft + hop) / hop   (stft.c:119) */
size_t vvhip_stft_num_frames(size_t n, size_t nfft, size_t hop);
int vvhip_stft_spectrogram_host(vvhip_stft* h, const float* signal, size_t n, float* out_mag);
/* nch channels at ch_stride floats; rows [ch][frame][...] at out_ch_stride elements.
 * out_kind 0: magnitudes sqrtf(re^2+im^2) of all nfft bins (stft.c:133-139);
 *          1: the full complex spectrum (float pairs, stft_process semantics);
 *          2: power re^2+im^2 of bins 0..nfft/2 (nfft/2+1 floats per row; the
 *             power spectrogram vv_dsp_compute_log_mel_spectrogram consumes). */
int vvhip_stft_spectrogram_device(vvhip_stft* h, const float* d_signal, size_t n, size_t nch,
                                  size_t ch_stride, void* d_out, size_t out_ch_stride,
                                  int out_kind, void* stream);
/* Power rows (kind 2) with rows row_pitch >= nfft/2+1 floats apart (the pad
 * floats are not written); out_ch_stride >= frames * row_pitch. */
int vvhip_stft_power_pitched_device(vvhip_stft* h, const float* d_signal, size_t n, size_t nch, size_t ch_stride,
                                    float* d_out, size_t out_ch_stride, size_t row_pitch, void* stream);
/* Frames [frame0, frame0 + nframes) of the same spectrogram (the row of frame
 * f is out + (f - frame0) * row): one shard of a long signal's frames.  With an
 * even frame0 the rows are bit-identical to the whole-signal call (frames are
 * transformed in pairs (2j, 2j+1)).  ST_RANGE if the range exceeds the frames. */
int vvhip_stft_spectrogram_range_device(vvhip_stft* h, const float* d_signal, size_t n, size_t nch,
                                        size_t ch_stride, size_t frame0, size_t nframes, void* d_out,
                                        size_t out_ch_stride, int out_kind, void* stream);
/* Half-spectrum rows for the config-5 gather: pack [rows][n] -> [rows][n/2+1]
 * (unpack 0), or expand [rows][n/2+1] -> [rows][n] by out[k] = in[n-k] above
 * n/2 (unpack 1; magnitude rows of real frames are mirror-symmetric). */
int vvhip_rows_half_device(const float* d_in, float* d_out, size_t rows, size_t n, int unpack, void* stream);
int vvhip_stft_process_host(vvhip_stft* h, const float* frame, float* spec_out);
int vvhip_stft_process_device(vvhip_stft* h, const float* d_frames, size_t count, float* d_spec,
                              void* stream);
int vvhip_stft_reconstruct_host(vvhip_stft* h, const float* spec, float* out_add, float* norm_add);
/* count frames (cpx[count][nfft]) overlap-added at `hop` into out_add/norm_add
 * (length (count-1)*hop + nfft); norm_add may be NULL. */
int vvhip_stft_reconstruct_device(vvhip_stft* h, const float* d_spec, size_t count, size_t hop,
                                  float* d_out_add, float* d_norm_add, void* stream);

/* ---- framing (src/core/framing.c:58-146) ----
 * Device: frames [frame0, frame0 + count) of an n-sample signal into
 * d_frames[count][frame_len] (zero padding, or reflection when center != 0;
 * times d_window when not NULL), and the overlap-add of count frames into
 * d_out[out_len] at (frame0 + f) * hop, each output sample summed in frame
 * order.  Host: one frame, the reference's signatures (via the device). */
int vvhip_fetch_frames_device(const float* d_signal, size_t n, float* d_frames, size_t frame_len, size_t hop,
                              size_t frame0, size_t count, int center, const float* d_window, void* stream);
int vvhip_overlap_add_device(const float* d_frames, size_t count, float* d_out, size_t out_len, size_t frame_len,
                             size_t hop, size_t frame0, void* stream);
int vvhip_fetch_frame_host(const float* signal, size_t n, float* frame, size_t frame_len, size_t hop,
                           size_t frame_index, int center, const float* window);
int vvhip_overlap_add_host(const float* frame, float* out, size_t out_len, size_t frame_len, size_t hop,
                           size_t frame_index);

/* ---- FIR (fir.c) ---- */
int vvhip_fir_create(const float* h, size_t taps, vvhip_fir** out);
void vvhip_fir_destroy(vvhip_fir* f);
/* mode 0: FFT overlap-save (fir_apply_fft semantics), mode 1: direct form,
 * same summation order as fir.c:170-186 (bit-identical to vv_dsp_fir_apply).
 * prefix: taps-1 samples preceding x[0] in time order (oldest first), or NULL
 * for zero initial state. */
int vvhip_fir_apply_host(vvhip_fir* f, const float* x, float* y, size_t n, const float* prefix,
                         int mode);
int vvhip_fir_apply_device(vvhip_fir* f, const float* d_x, float* d_y, size_t n, size_t nch,
                           size_t x_stride, size_t y_stride, const float* d_prefix, int mode,
                           void* stream);
/* ---- Mel / MFCC (src/features/mel.c:204-309) ----
 * fb: dense filterbank [n_mels][nbins] (vv_dsp_mel_filterbank_create), or NULL
 * for a plan that only maps log-mel rows to MFCC (kind 2).  n_coeffs: MFCC
 * coefficients (0 = log-mel only); lifter as mel.c:298-304; eps added before log. */
int vvhip_mel_create(const float* fb, size_t n_mels, size_t nbins, size_t n_coeffs, float lifter, float eps,
                     vvhip_mel** out);
void vvhip_mel_destroy(vvhip_mel* m);
/* kind 0: power rows [frames][nbins] -> log-mel [frames][n_mels]
 *      1: power rows -> MFCC [frames][n_coeffs]
 *      2: log-mel rows [frames][n_mels] -> MFCC [frames][n_coeffs] */
int vvhip_mel_device(vvhip_mel* m, const float* d_in, size_t frames, float* d_out, int kind, void* stream);
/* the same with power rows row_pitch >= nbins floats apart (kinds 0 / 1; 0 = nbins) */
int vvhip_mel_pitched_device(vvhip_mel* m, const float* d_in, size_t frames, size_t row_pitch, float* d_out, int kind,
                             void* stream);
/* signal [ch][n] (ch_stride floats apart) -> log-mel (kind 0) or MFCC (kind 1)
 * rows [ch][frame][n_mels | n_coeffs]: the stft's power rows feed the mel plan
 * in one kernel when nfft = 1024 (else two launches, same values) */
int vvhip_stft_mel_device(vvhip_stft* h, vvhip_mel* m, const float* d_signal, size_t n, size_t nch, size_t ch_stride,
                          float* d_out, size_t out_ch_stride, int kind, void* stream);
int vvhip_mel_host(vvhip_mel* m, const float* in, size_t frames, float* out, int kind);

/* Block length (real FFT size) the overlap-save path uses for a signal of n samples. */
/* zero-phase filtering (filter/common.c:23-80): reflection pad, direct form
 * forward and backward in the reference's summation order (bit-identical) */
int vvhip_fir_filtfilt_device(vvhip_fir* f, const float* d_x, float* d_y, size_t n, size_t nch, size_t x_stride,
                              size_t y_stride, void* stream);
int vvhip_fir_filtfilt_host(vvhip_fir* f, const float* x, float* y, size_t n);
size_t vvhip_fir_block_size(vvhip_fir* f, size_t n);

/* ---- Hilbert analytic signal (hilbert.c:14-75) ---- */
int vvhip_hilbert_host(const float* x, size_t n, float* z_out);
int vvhip_hilbert_device(const float* d_x, size_t n, size_t batch, float* d_z, void* stream);
/* Instantaneous phase / frequency (hilbert.c:77-113) of `batch` contiguous rows
 * of n samples: z complex[batch][n] -> unwrapped phase real[batch][n];
 * phase -> frequency in Hz (freq[row][0] = 0), fs the sample rate. */
int vvhip_inst_phase_host(const float* z, size_t n, float* phase);
int vvhip_inst_phase_device(const float* d_z, size_t n, size_t batch, float* d_phase, void* stream);
int vvhip_inst_freq_host(const float* phase, size_t n, double fs, float* freq);
int vvhip_inst_freq_device(const float* d_phase, size_t n, size_t batch, double fs, float* d_freq, void* stream);

/* ---- Chirp-z transform (src/spectral/czt.c:58-178) ----
 * X[k] = sum_{n<N} x[n] A^-n W^(nk), k < M (scipy.signal.czt convention).  A plan
 * holds the chirps and the chirp's spectrum for P = next_pow2(N + M - 1) <= 2^24.
 * Device: `batch` contiguous rows, x complex[batch][N] (real_in 0) or
 * real[batch][N] (real_in 1) -> X complex[batch][M]. */
int vvhip_czt_create(size_t n, size_t m, float w_re, float w_im, float a_re, float a_im, vvhip_czt** out);
void vvhip_czt_destroy(vvhip_czt* h);
int vvhip_czt_exec_device(const vvhip_czt* h, const void* d_x, int real_in, size_t batch, void* d_X,
                          void* stream);
int vvhip_czt_exec_host(const void* x, int real_in, size_t n, size_t m, float w_re, float w_im, float a_re,
                        float a_im, void* X);

/* ---- Cepstrum / minimum phase (src/envelope/cepstrum.c:7-78, minphase.c:7-31) ----
 * `batch` contiguous rows of n: real cepstrum Re IFFT(log(|FFT x| + 1e-12));
 * Re IFFT(exp(Re FFT(fold c))) and the spectrum exp(Re FFT(fold c)) (complex,
 * imaginary parts 0), fold c = (c0, 2 c1 .. 2 c(n/2-1), 0 ..). */
int vvhip_cepstrum_device(const float* d_x, size_t n, size_t batch, float* d_c, void* stream);
int vvhip_icepstrum_minphase_device(const float* d_c, size_t n, size_t batch, float* d_x, void* stream);
int vvhip_minphase_from_cepstrum_device(const float* d_c, size_t n, size_t batch, float* d_spec, void* stream);
int vvhip_cepstrum_host(const float* x, size_t n, float* c);
int vvhip_icepstrum_minphase_host(const float* c, size_t n, float* x);
int vvhip_minphase_from_cepstrum_host(const float* c, size_t n, float* spec);

/* ---- Spectral utilities (src/spectral/utils.c:5-73) ----
 * `batch` contiguous rows of n: fftshift (inverse 0) / ifftshift (inverse 1) of
 * float (cpx 0) or complex (cpx 1) rows, a permutation (in place allowed);
 * phase wrap of `count` floats into (-pi, pi]; phase unwrap of each row. */
int vvhip_fftshift_device(const void* d_in, void* d_out, size_t n, size_t batch, int cpx, int inverse,
                          void* stream);
int vvhip_phase_wrap_device(const float* d_in, float* d_out, size_t count, void* stream);
int vvhip_phase_unwrap_device(const float* d_in, float* d_out, size_t n, size_t batch, void* stream);
int vvhip_fftshift_host(const void* in, void* out, size_t n, int cpx, int inverse);
int vvhip_phase_wrap_host(const float* in, float* out, size_t n);
int vvhip_phase_unwrap_host(const float* in, float* out, size_t n);

/* ---- DCT (dct.c:86-136); nan_policy as core/nan_policy.h (0..3) ---- */
int vvhip_dct_host(const float* in, float* out, size_t n, int type, int dir, int nan_policy);
int vvhip_dct_device(const float* d_in, float* d_out, size_t n, size_t batch, int type, int dir,
                     int nan_policy, void* stream);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif
