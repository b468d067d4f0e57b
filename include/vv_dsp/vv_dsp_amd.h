/* vv_dsp_amd.h -- ADDITIVE batched / device-pointer entry points of the MI355X
 * backend.  The reference API (fft.h, stft.h, ...) is host-pointer and one
 * transform per call, which pays PCIe per call; these entry points take
 * device (HBM) pointers and whole batches and run asynchronously on a HIP
 * stream passed as void* (NULL = default stream).  Nothing here changes the
 * reference's C99 ABI. */
#ifndef VV_DSP_AMD_H
#define VV_DSP_AMD_H
#include "vv_dsp/vv_dsp_types.h"
#include "vv_dsp/spectral/fft.h"
#include "vv_dsp/spectral/stft.h"
#include "vv_dsp/spectral/dct.h"
#include "vv_dsp/filter/fir.h"
#include "vv_dsp/features/mel.h"
#include "vv_dsp/spectral/czt.h"
#include "vv_dsp/envelope/cepstrum.h"
#include "vv_dsp/envelope/minphase.h"

#ifdef __cplusplus
extern "C" {
#endif

/* number of usable HIP devices */
int vv_dsp_amd_device_count(void);
const char* vv_dsp_amd_last_error(void);
/* The calling thread's device for the device-pointer calls below (hipSetDevice):
 * one process per GPU sets it once; one process driving several GPUs switches it
 * per shard.  OUT_OF_RANGE for a bad index, UNSUPPORTED with no device. */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_amd_set_device(int device);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_amd_get_device(int* device);

/* FFT: `batch` contiguous transforms per execute (host or device pointers). */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_fft_make_plan_many(size_t n, vv_dsp_fft_type type, vv_dsp_fft_dir dir,
                                                         size_t batch, vv_dsp_fft_plan** out_plan);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_fft_execute_device(const vv_dsp_fft_plan* plan, const void* d_in,
                                                         void* d_out, void* stream);

/* STFT over nch channels (ch_stride floats apart) into [ch][frame][fft_size]
 * rows (out_ch_stride floats apart): magnitudes (_spectrogram_) or complex
 * spectra (_spectrum_). */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_spectrogram_device(vv_dsp_stft* h, const vv_dsp_real* d_signal,
                                                              size_t n, size_t nch, size_t ch_stride,
                                                              vv_dsp_real* d_out_mag, size_t out_ch_stride,
                                                              void* stream, size_t* out_frames);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_spectrum_device(vv_dsp_stft* h, const vv_dsp_real* d_signal,
                                                           size_t n, size_t nch, size_t ch_stride,
                                                           vv_dsp_cpx* d_out, size_t out_ch_stride,
                                                           void* stream, size_t* out_frames);
/* power spectrogram [ch][frame][fft_size/2+1] = re^2 + im^2 of bins 0..fft_size/2
 * (the input of vv_dsp_compute_log_mel_spectrogram / vv_dsp_mfcc_process) */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_power_device(vv_dsp_stft* h, const vv_dsp_real* d_signal,
                                                        size_t n, size_t nch, size_t ch_stride,
                                                        vv_dsp_real* d_out_power, size_t out_ch_stride,
                                                        void* stream, size_t* out_frames);
/* The same power rows placed row_pitch floats apart (row_pitch >= fft_size/2+1;
 * the pad floats past bin fft_size/2 are not written; out_ch_stride >= frames x
 * row_pitch).  A pitch of a whole number of 128 B lines -- 544 for fft_size
 * 1024: 17 lines -- starts every row on a line, so the rows leave as whole-line
 * stores; the values equal vv_dsp_stft_power_device's bit for bit.  The
 * reference's packed layout (mel.h:156-161) is row_pitch = fft_size/2+1. */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_power_pitched_device(vv_dsp_stft* h, const vv_dsp_real* d_signal,
                                                                size_t n, size_t nch, size_t ch_stride,
                                                                vv_dsp_real* d_out_power, size_t out_ch_stride,
                                                                size_t row_pitch, void* stream, size_t* out_frames);
/* One shard of a long signal's frames: rows of frames [frame0, frame0 + nframes)
 * of the same spectrogram, row of frame f at d_out + (f - frame0) * row.
 * out_kind 0: magnitudes [fft_size] floats, 1: complex spectrum [fft_size]
 * vv_dsp_cpx, 2: power [fft_size/2+1] floats.  Even frame0 gives rows
 * bit-identical to the whole-signal call.  VV_DSP_ERROR_OUT_OF_RANGE when the
 * range passes the last frame (stft.c:119 frame count). */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_frames_range_device(vv_dsp_stft* h, const vv_dsp_real* d_signal,
                                                               size_t n, size_t nch, size_t ch_stride,
                                                               size_t frame0, size_t nframes, void* d_out,
                                                               size_t out_ch_stride, int out_kind, void* stream);
/* the handle's fft_size and hop_size (either pointer may be NULL) */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_get_sizes(const vv_dsp_stft* h, size_t* fft_size, size_t* hop_size);
/* ---- Multi-GPU layout of config 5: channels shard with no
 * exchange; the only collective is the caller's gather of the rows. ----
 * The contiguous block split rank `rank` of `world` owns: channels
 * [*first, *first + *count), rank order = channel order, sizes differ by at most
 * one (the same split as vv-dsp_amd/vvdsp_dist.py channel_shard).  The RCCL
 * shard + gather entry points are in vv_dsp/vv_dsp_dist.h. */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_shard_range(size_t total, size_t world, size_t rank, size_t* first,
                                                  size_t* count);
/* One rank's share of a multi-channel spectrogram on `device`: the rows of
 * channels [first, first + count) of a [total][n] job (d_signal points at the
 * shard's first channel, on that device) into d_out [count][frames][row].
 * out_kind as vv_dsp_stft_frames_range_device (0 magnitude, 1 complex, 2 power
 * n/2+1).  The handle may be shared by all devices: its window is copied to
 * each device once.  The thread's current device is restored on return. */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_channel_shard_device(vv_dsp_stft* h, int device,
                                                                const vv_dsp_real* d_signal, size_t n, size_t count,
                                                                size_t ch_stride, int out_kind, void* d_out,
                                                                size_t out_ch_stride, void* stream, size_t* out_frames);
/* Half-spectrum rows for the gather: magnitude (or power) rows of real frames
 * are mirror-symmetric, |X[n-k]| = |X[k]|, so a rank can send bins 0..n/2 only
 * (half the xGMI bytes of config 5's gather) and the root expands them.
 * pack: [rows][fft_size] -> [rows][fft_size/2+1]; unpack: the reverse, bin k
 * above fft_size/2 taken from bin fft_size-k.  For rows of the fused STFT
 * kernels (power-of-two fft_size <= 8192, 7-smooth <= 4096) the mirror bins
 * are computed from the same conjugate pair, so unpack(pack(rows)) == rows bit
 * for bit. */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_spectrogram_pack_half_device(const vv_dsp_real* d_rows, size_t rows,
                                                                   size_t fft_size, vv_dsp_real* d_half, void* stream);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_spectrogram_unpack_half_device(const vv_dsp_real* d_half, size_t rows,
                                                                     size_t fft_size, vv_dsp_real* d_rows,
                                                                     void* stream);
/* Batched framing (vv_dsp_fetch_frame / vv_dsp_overlap_add, framing.c:71-146):
 * frames [frame0, frame0 + count) into d_frames[count][frame_len]; and count
 * frames added into d_out[output_len] at (frame0 + f) * hop_len, every output
 * sample summed in frame order (bit-identical to the per-frame loop). */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_fetch_frames_device(const vv_dsp_real* d_signal, size_t signal_len,
                                                          vv_dsp_real* d_frames, size_t frame_len, size_t hop_len,
                                                          size_t frame0, size_t count, int center,
                                                          const vv_dsp_real* d_window, void* stream);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_overlap_add_device(const vv_dsp_real* d_frames, size_t count,
                                                         vv_dsp_real* d_out, size_t output_len, size_t frame_len,
                                                         size_t hop_len, size_t frame0, void* stream);
/* count frames real[count][fft_size] -> cpx[count][fft_size] (vv_dsp_stft_process batched) */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_process_device(vv_dsp_stft* h, const vv_dsp_real* d_frames,
                                                          size_t count, vv_dsp_cpx* d_spec, void* stream);
/* count spectra overlap-added at the handle's hop (vv_dsp_stft_reconstruct batched) */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_reconstruct_device(vv_dsp_stft* h, const vv_dsp_cpx* d_spec,
                                                              size_t count, vv_dsp_real* d_out_add,
                                                              vv_dsp_real* d_norm_add, void* stream);

/* FIR plan: coefficients resident on the device; overlap-save for fir_apply_fft
 * semantics, direct form (bit-identical to vv_dsp_fir_apply) on request. */
typedef struct vv_dsp_fir_plan vv_dsp_fir_plan;
VV_DSP_NODISCARD vv_dsp_status vv_dsp_fir_plan_create(const vv_dsp_real* coeffs, size_t num_taps,
                                                      vv_dsp_fir_plan** out);
vv_dsp_status vv_dsp_fir_plan_destroy(vv_dsp_fir_plan* p);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_fir_apply_fft_device(vv_dsp_fir_plan* p, const vv_dsp_real* d_x,
                                                           vv_dsp_real* d_y, size_t n, size_t nch,
                                                           size_t x_stride, size_t y_stride, void* stream);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_fir_apply_direct_device(vv_dsp_fir_plan* p, const vv_dsp_real* d_x,
                                                              vv_dsp_real* d_y, size_t n, size_t nch,
                                                              size_t x_stride, size_t y_stride, void* stream);
/* vv_dsp_filtfilt_fir over nch rows (filter/common.c:23-80), bit-identical */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_filtfilt_fir_device(vv_dsp_fir_plan* p, const vv_dsp_real* d_x,
                                                          vv_dsp_real* d_y, size_t n, size_t nch, size_t x_stride,
                                                          size_t y_stride, void* stream);

/* Hilbert analytic signal of `batch` contiguous real[N] rows -> cpx[batch][N] */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_hilbert_analytic_device(const vv_dsp_real* d_x, size_t N, size_t batch,
                                                              vv_dsp_cpx* d_z, void* stream);
/* Instantaneous phase (unwrapped, radians) of `batch` contiguous analytic rows
 * cpx[batch][N] -> real[batch][N]; instantaneous frequency (Hz) of phase rows
 * real[batch][N] -> real[batch][N], element 0 of each row = 0 (hilbert.c:77-113). */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_instantaneous_phase_device(const vv_dsp_cpx* d_analytic, size_t N,
                                                                 size_t batch, vv_dsp_real* d_phase, void* stream);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_instantaneous_frequency_device(const vv_dsp_real* d_phase, size_t N,
                                                                     size_t batch, double sample_rate,
                                                                     vv_dsp_real* d_freq, void* stream);
/* DCT of `batch` contiguous rows with the plan's type/direction */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_dct_execute_device(const vv_dsp_dct_plan* plan, const vv_dsp_real* d_in,
                                                         vv_dsp_real* d_out, size_t batch, void* stream);

/* MFCC plan (vv_dsp_mfcc_init) on device rows: power [frames][n_fft/2+1]
 * (e.g. vv_dsp_stft_power_device) -> MFCC [frames][num_mfcc_coeffs], or ->
 * log-mel [frames][n_mels]; one fused kernel, the spectrogram read once. */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_mfcc_process_device(const vv_dsp_mfcc_plan* plan, const vv_dsp_real* d_power,
                                                          size_t num_frames, vv_dsp_real* d_out_mfcc, void* stream);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_log_mel_device(const vv_dsp_mfcc_plan* plan, const vv_dsp_real* d_power,
                                                     size_t num_frames, vv_dsp_real* d_out_log_mel, void* stream);
/* the same on power rows row_pitch >= n_fft/2+1 floats apart (e.g.
 * vv_dsp_stft_power_pitched_device's); the values do not depend on the pitch */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_mfcc_process_pitched_device(const vv_dsp_mfcc_plan* plan,
                                                                  const vv_dsp_real* d_power, size_t num_frames,
                                                                  size_t row_pitch, vv_dsp_real* d_out_mfcc,
                                                                  void* stream);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_log_mel_pitched_device(const vv_dsp_mfcc_plan* plan, const vv_dsp_real* d_power,
                                                             size_t num_frames, size_t row_pitch,
                                                             vv_dsp_real* d_out_log_mel, void* stream);
/* Signal -> log-mel / MFCC rows without the power spectrogram in HBM:
 * d_signal [nch][n] (ch_stride floats apart) -> d_out [nch][frames][n_mels]
 * (log-mel) or [nch][frames][num_mfcc_coeffs] (MFCC), out_ch_stride floats
 * apart.  The values are those of vv_dsp_stft_power_device followed by
 * vv_dsp_log_mel_device / vv_dsp_mfcc_process_device (the stft's window,
 * nfft and hop; the plan's filterbank, log epsilon, DCT and lifter), bit for
 * bit.  One kernel computes them with the power rows kept in LDS when
 * nfft = 1024, hop <= 256 and a multiple of 4, the signal 16-B aligned with
 * ch_stride a multiple of 4, n_mels <= 128 (log-mel) or n_mels <= 60 and
 * num_mfcc_coeffs <= 64 (MFCC: the log-mel rows stay in the exchange buffer's
 * spare tail); any other shape runs the two steps through a scratch buffer
 * (vvhip_debug_get("STAT_MEL_FUSED") / ("STAT_MEL_SPLIT") count which ran).
 * The plan's n_fft must equal the stft's nfft (VV_DSP_ERROR_INVALID_SIZE). */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_log_mel_device(vv_dsp_stft* h, const vv_dsp_mfcc_plan* plan,
                                                          const vv_dsp_real* d_signal, size_t n, size_t nch,
                                                          size_t ch_stride, vv_dsp_real* d_out, size_t out_ch_stride,
                                                          void* stream, size_t* out_frames);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_stft_mfcc_device(vv_dsp_stft* h, const vv_dsp_mfcc_plan* plan,
                                                       const vv_dsp_real* d_signal, size_t n, size_t nch,
                                                       size_t ch_stride, vv_dsp_real* d_out, size_t out_ch_stride,
                                                       void* stream, size_t* out_frames);

/* Chirp-z plan (vv_dsp_czt_exec_cpx / _real semantics, czt.c:44-178): chirps and
 * the chirp's spectrum resident on the device; `batch` contiguous rows
 * complex[batch][N] (real_input 0) or real[batch][N] (real_input 1) ->
 * complex[batch][M].  N + M - 1 <= 2^24. */
typedef struct vv_dsp_czt_plan vv_dsp_czt_plan;
VV_DSP_NODISCARD vv_dsp_status vv_dsp_czt_plan_create(size_t N, size_t M, vv_dsp_real W_real, vv_dsp_real W_imag,
                                                      vv_dsp_real A_real, vv_dsp_real A_imag, vv_dsp_czt_plan** out);
vv_dsp_status vv_dsp_czt_plan_destroy(vv_dsp_czt_plan* p);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_czt_execute_device(const vv_dsp_czt_plan* p, const void* d_in, int real_input,
                                                         size_t batch, vv_dsp_cpx* d_out, void* stream);
/* Cepstrum family on `batch` contiguous rows of n (cepstrum.c:7-78, minphase.c:7-31) */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_cepstrum_real_device(const vv_dsp_real* d_x, size_t n, size_t batch,
                                                           vv_dsp_real* d_cep, void* stream);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_icepstrum_minphase_device(const vv_dsp_real* d_c, size_t n, size_t batch,
                                                                vv_dsp_real* d_x, void* stream);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_minphase_from_cepstrum_device(const vv_dsp_real* d_c, size_t n, size_t batch,
                                                                    vv_dsp_cpx* d_spec, void* stream);
/* Spectral utilities on `batch` contiguous rows of n (utils.c:5-73): fftshift
 * (inverse 0) / ifftshift (inverse 1) of float or complex rows (in place
 * allowed); phase wrap of `count` floats; phase unwrap of each row. */
VV_DSP_NODISCARD vv_dsp_status vv_dsp_fftshift_device(const void* d_in, void* d_out, size_t n, size_t batch,
                                                      int is_complex, int inverse, void* stream);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_phase_wrap_device(const vv_dsp_real* d_in, vv_dsp_real* d_out, size_t count,
                                                        void* stream);
VV_DSP_NODISCARD vv_dsp_status vv_dsp_phase_unwrap_device(const vv_dsp_real* d_in, vv_dsp_real* d_out, size_t n,
                                                          size_t batch, void* stream);

#ifdef __cplusplus
}
#endif
#endif
