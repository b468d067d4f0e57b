// vvhip_internal.hpp -- launchers shared between the kernel translation units
// and the extern "C" shim (shim.hip).  Not part of the public C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace vvh {

// ---- A/B switches and path counters (debug.hip) ---------------------------
// Knob values come from vvhip_debug_set (or, with VVHIP_AB=1, from the
// environment read once per process); knob(k, dflt) returns dflt when unset.
enum Knob : int {
    KNOB_STFT_CPS, KNOB_STFT_RUN, KNOB_STFT_DBS, KNOB_POW_OLD, KNOB_STFT_RING, KNOB_STFT_DYN,
    KNOB_FS_VAR, KNOB_FS_CHUNK_MB, KNOB_FS_OLD, KNOB_BLUE_UNFUSED, KNOB_C2C_MAX, KNOB_STFT_SQ, KNOB_MIX_VAR,
    KNOB_MIX_CHUNK_MB, KNOB_MIX_R2C_FULL, KNOB_FIR_OLD, KNOB_FIR_DYN, KNOB_FIR_DIRECT_LDS, KNOB_FIR_BLOCK,
    KNOB_HOST_CHUNK_MB, KNOB_NO_MIXED, KNOB_REAL_PROMOTE, KNOB_ISTFT_OLD, KNOB_MEL_FUSED, KNOB_CZT_UNFUSED,
    KNOB_CEPS_UNFUSED, KNOB_FIR_R32, KNOB_DIST_SLAB_KB, KNOB_POW_R32, KNOB_MAG_R32, KNOB_MEL_R32,
    KNOB_C2C_TPW, KNOB_C2C_ONE, KNOB_REAL_TPW, KNOB_ANA_TPW, KNOB_MIX_TPW, KNOB_C2C_SMALL, KNOB_DCT_SMALL, KNOB_HIL_SMALL, KNOB_REAL_SMALL, KNOB_R2C_SMALL, KNOB_STFT_STAGE, KNOB_STFT_ONE, KNOB_MFCC_WIN, KNOB_COUNT
};
long long knob(Knob k, long long dflt);
// launches of the paths the tests must see taken (vvhip_debug_get("STAT_..."))
enum Stat : int { STAT_STFT_DYN, STAT_FIR_DYN, STAT_FIR_STATIC, STAT_MEL_FUSED, STAT_MEL_SPLIT, STAT_FIR_R32, STAT_POW_R32, STAT_MAG_R32, STAT_MEL_R32, STAT_COUNT };
void stat_inc(Stat s);

// Device-resident W_N^k = exp(-2*pi*i*k/N) table, k < N, f32 rounded from double.
// Cached per N for the process lifetime (per device).
const float2* twiddle_table(int n);
const double2* twiddle_table_d(long long n);
// Pass-major inter-pass twiddles of the length-n Stockham FFT (fft_core.hpp TwTab).
const float2* pass_twiddles(int n);

// Two-level table for large n (large_fft.hip): lo[2^lo_bits] ++ hi[n >> lo_bits].
const float2* twiddle_split(long long n, int* lo_bits);

// ---- large power-of-two C2C (large_fft.hip): four-step over the fused kernels
bool c2c_large_supported(long long n);     // pow2, 8192 .. 2^24
hipError_t launch_c2c_large(long long n, int fwd, const float2* in, float2* out, long long batch,
                            hipStream_t s);
// Bluestein (chirp-z) for any n with pow2(2n-1) <= 2^24; same contract as
// launch_dft_naive (real_in promotes real input; nout bins written).
constexpr long long BLUESTEIN_MIN = 1025;   // below: the f64 O(n^2) DFT (exact-angle, faster at small n)
bool bluestein_supported(long long n);
hipError_t launch_bluestein(long long n, int fwd, const void* in, int real_in, float2* out, long long nout,
                            long long batch, long long in_dist, long long out_dist, float scale, hipStream_t s);
// Mixed-radix Stockham FFT (mixed_fft.hip) for 7-smooth non-power-of-two n
// <= 4096; same contract as launch_dft_naive, and in == out is allowed.
bool mixed_supported(long long n);
bool stft_mixed_supported(long long n);
hipError_t launch_fft_mixed(long long n, int fwd, const void* in, int real_in, float2* out, long long nout,
                            long long batch, long long in_dist, long long out_dist, float scale, hipStream_t s);
// STFT rows through the mixed-radix kernel (frames gathered and windowed on
// load, |X| / complex / power bins 0..n/2 on store): kind as launch_stft.
hipError_t launch_stft_mixed(long long nfft, long long hop, int kind, const float* sig, long long n, long long nch,
                             long long ch_stride, long long frames, const float* win, void* out,
                             long long out_ch_stride, hipStream_t s);
// Real pow2 n = 2M above the fused kernels: split steps around an M-point C2C
// (fft_kernels.hip).  fwd: Z [batch][M] -> X [batch][M+1]; inv: X -> V [batch][M].
hipError_t launch_real_split_fwd(const float2* Z, float2* X, long long M, long long batch, hipStream_t s);
hipError_t launch_real_split_inv(const float2* X, float2* V, long long M, long long batch, hipStream_t s);
// real[batch][n] -> complex[batch][n] (imaginary 0)
hipError_t launch_promote_real(const float* in, float2* out, long long count, hipStream_t s);

// ---- mel / MFCC (mel_kernels.hip) ---------------------------------------
// mode 0: power rows [frames][nbins] -> log-mel [frames][n_mels]
//      1: power rows -> MFCC [frames][n_coeffs];  2: log-mel rows -> MFCC
// in_pitch (modes 0 / 1): floats from one power row's start to the next (0: nbins)
hipError_t launch_mel_grp(int mode, const float* in, long long frames, int nbins, int n_mels, int n_coeffs,
                          const float* W, int nnz, const int* chunks, int nc, const int* cbeg, const float* D,
                          const float* lift, float eps, float* out, hipStream_t s, int in_pitch = 0);
// host: chunk schedule of the filters' non-zero ranges {lo, len, off}[n_mels] for
// launch_mel_grp (chunks {lo, len, off}, cbeg[n_mels+1]); returns the chunk length
int mel_chunk_schedule(const int* meta, int n_mels, std::vector<int>* chunks, std::vector<int>* cbeg);

// Write sink (SINK_FLOATS floats): destination of lanes that must issue a store
// with nothing to write, in kernels that hand-count their memory operations.
constexpr size_t SINK_FLOATS = 1u << 18;   // 1 MiB = 4096 waves x 64 lanes
float* store_sink();
// zeroed work counters of the dynamic walks (32 counter streams x 32 words) for a
// launch on stream s (tables.hip: per-(device, stream) pool blocks; a private,
// memset-on-replay block under graph capture); nullptr: take the static walk
constexpr size_t STFT_CTR_WORDS = 32 * 32;
unsigned* stream_counters(hipStream_t s);
// ---- batched framing (framing_kernels.hip), framing.c:58-146 semantics
long long reflect_sample(long long idx, long long n);   // framing.c:21-56, host side (span bounds)
hipError_t launch_fetch_frames(const float* sig, long long base, long long n, float* out, long long len,
                               long long hop, long long frame0, long long count, int center, const float* win,
                               hipStream_t s);
hipError_t launch_overlap_add(const float* frames, long long count, float* out, long long out_len, long long len,
                              long long hop, long long frame0, hipStream_t s);

// Persistent-grid sizing: resident blocks for `kernel` x CUs, capped by work.
// CUs x resident workgroups of `kernel` (capped at max_per_cu when > 0), at most work_blocks
int persistent_grid(const void* kernel, int block, size_t dyn_lds, long long work_blocks, int max_per_cu = 0);
// persistent_grid computed once per call site (a launcher's static cache);
// concurrent first calls compute the same value, the atomic keeps that race-free
inline int cached_grid(std::atomic<int>& cache, const void* kernel, int block, size_t dyn_lds, long long work_blocks,
                       int max_per_cu = 0) {
    int g = cache.load(std::memory_order_relaxed);
    if (g == 0) {
        g = persistent_grid(kernel, block, dyn_lds, work_blocks, max_per_cu);
        cache.store(g, std::memory_order_relaxed);
    }
    return g;
}

// ---- pow2 register/LDS FFTs (fft_kernels.hip) -----------------------------
bool c2c_supported(long long n);           // pow2, 2..4096
// batch transforms of length n; element e of transform f at in[f*in_dist + e]
hipError_t launch_c2c(long long n, int fwd, const float2* in, float2* out, long long batch,
                      long long in_dist, long long out_dist, float scale, hipStream_t s);
bool r2c_supported(long long n);           // pow2 real length, 32..8192
hipError_t launch_r2c(long long n, const float* in, float2* out, long long batch,
                      long long in_dist, long long out_dist, hipStream_t s);
hipError_t launch_c2r(long long n, const float2* in, float* out, long long batch,
                      long long in_dist, long long out_dist, hipStream_t s);
// Any n: O(n^2) DFT with f64 accumulation (the reference's non-pow2 path,
// fft_kiss.c:76-92).  real_in: input is real[n] (R2C promotion); nout bins written.
hipError_t launch_dft_naive(long long n, int fwd, const void* in, int real_in, float2* out,
                            long long nout, long long batch, long long in_dist,
                            long long out_dist, float scale, hipStream_t s);
// Hermitian expansion used by C2R/Hilbert for non-pow2 n: half[n/2+1] -> full[n]
hipError_t launch_hermitian_expand(long long n, const float2* half, float2* full, long long batch,
                                   long long half_dist, int zero_dc_nyq_imag, hipStream_t s);
hipError_t launch_take_real(const float2* in, float* out, long long count, hipStream_t s);
hipError_t launch_zero_nyquist_imag(float2* out, long long n, long long batch, long long dist,
                                    hipStream_t s);

// ---- STFT (stft_kernels.hip) -------------------------------------------
// mode 0: magnitude rows [frames][nfft]; 1: complex rows [frames][nfft];
// 2: power rows [frames][nfft/2+1], row_pitch floats apart (0: packed, nfft/2+1)
bool stft_fused_supported(long long nfft);
hipError_t launch_stft(long long nfft, long long hop, int mode, const float* sig, long long n,
                       long long nch, long long ch_stride, long long frames, const float* win,
                       void* out, long long out_ch_stride, hipStream_t s, long long row_pitch = 0);
// Mel filterbank / log / DCT tables of an MFCC plan (vvhip_mel, device
// pointers) for the fused signal -> log-mel / MFCC launch
struct MelArgs {
    const float* W = nullptr;      // non-zero filter weights, packed (nnz)
    const int* chunks = nullptr;   // {lo, len, off} per chunk (mel_chunk_schedule)
    const int* cbeg = nullptr;     // first chunk of each filter [M + 1]
    const float* D = nullptr;      // DCT-II rows [C][M]
    const float* lift = nullptr;   // lifter factors [C]
    int nnz = 0, nc = 0, M = 0, C = 0;
    // The layout the kernel reads: cw = 3 -- W packed with the chunk table above;
    // cw = 0 -- each chunk's window of lc bins as a row of lcs = window_stride(lc) floats in W,
    // [c lcs + j] the weight of bin lo_c + j (zero outside the chunk), [c lcs + lc]
    // lo_c's bits, the window inside the row (lo_c + lc <= n/2 + 1), lc % 4 == 0, no
    // chunk table.  The plan passes the packed layout plus the windows (Ww, lcw);
    // launch_stft_mel gives log-mel the windows and MFCC the packed layout.
    int lc = 0, lcs = 0, cw = 3;
    // row stride of the chunk windows for lc bins (lc % 4 == 0): the first multiple
    // of 4 above lc whose quarter is odd, so 16 lanes' 16 B weight reads (rows
    // lcs floats apart) cover 16 distinct 4-bank blocks
    static constexpr int window_stride(int lc) { return (lc / 4) % 2 == 0 ? lc + 4 : lc + 8; }
#ifndef VVH_MEL_W2
#define VVH_MEL_W2 1
#endif
    // VVH_MEL_W2: the chunk windows are 4 bins longer than the chunk schedule's
    // lc and start on even bins, so the kernel reads their power pairs two bins
    // per ds_read_b128 (half the read instructions; the 4 extra bins weigh 0)
    static constexpr bool W2 = VVH_MEL_W2;
    const float* Ww = nullptr;
    int lcw = 0;
    float eps = 0.0f;
};
// Log-mel (kind 0) or MFCC (kind 1) rows [ch][frame][M or C] straight from the
// signal: the power rows of launch_stft mode 2 feed k_mel_grp's arithmetic in
// the same kernel, never written to HBM (bit-identical to the two launches).
// hipErrorNotSupported when the fused kernel does not take this shape
// (nfft != 1024, hop / alignment, M > 128, C > 64): the caller runs the two launches.
hipError_t launch_stft_mel(int kind, long long nfft, long long hop, const float* sig, long long n, long long nch,
                           long long ch_stride, long long frames, const float* win, const MelArgs& mel, float* out,
                           long long out_ch_stride, hipStream_t s);
// Frames given explicitly (stft_process batch): in real[count][nfft] -> cpx[count][nfft]
hipError_t launch_stft_frames(long long nfft, const float* frames_in, const float* win,
                              float2* out, long long count, hipStream_t s);
// Generic gather (any nfft): windowed complex frames for the generic FFT path
hipError_t launch_frame_gather(long long nfft, long long hop, const float* sig, long long n,
                               long long nch, long long ch_stride, long long frames,
                               const float* win, float2* out, hipStream_t s);
hipError_t launch_magnitude(const float2* in, float* out, long long count, hipStream_t s);
hipError_t launch_rows_half(const float* in, float* out, long long rows, long long n, int unpack, hipStream_t s);
hipError_t launch_power_half(const float2* in, float* out, long long nfft, long long rows, hipStream_t s);
// ISTFT accumulate (stft_reconstruct batch): out_add[i] += Re(t[f][i])*w[i] for frames at hop
hipError_t launch_ola(long long nfft, long long hop, const float2* time_frames, long long count,
                      const float* win, float* out_add, float* norm_add, hipStream_t s);
// the same from the spectra in one kernel (inverse FFT + window + overlap-add): nfft 1024, hop | nfft, hop >= 256
bool istft_fused_supported(long long nfft, long long hop);
hipError_t launch_istft_fused(long long nfft, long long hop, const float2* spec, long long count,
                              const float* win, float* out_add, float* norm_add, hipStream_t s);

// ---- FIR overlap-save (fir_kernels.hip) ---------------------------------
bool fir_ols_supported(long long nfft);
// H: nfft complex bins of FFT(h zero-padded)/nfft.  prefix: [nch][taps-1] chronological or null.
hipError_t launch_fir_ols(long long nfft, long long taps, const float2* H, const float* x,
                          float* y, long long n, long long nch, long long x_stride,
                          long long y_stride, const float* prefix, hipStream_t s);
hipError_t launch_fir_direct(const float* h, long long taps, const float* x, float* y, long long n,
                             long long nch, long long x_stride, long long y_stride,
                             const float* prefix, hipStream_t s);
// vv_dsp_filtfilt_fir over nch rows (common.c:23-80); tmp: nch * (n + taps - 1) floats
hipError_t launch_filtfilt(const float* h, long long taps, const float* x, float* y, long long n, long long nch,
                           long long x_stride, long long y_stride, float* tmp, hipStream_t s);
// overlap-save glue for filters beyond the fused kernels (N > 8192, four-step FFTs):
// rows q < rows of pair p0 + q over (channel, pair) items, ppc pairs per channel,
// row = z[e] = (x[2j*lout - le + e], x[(2j+1)*lout - le + e]) zero outside [0, n)
hipError_t launch_fir_long_gather(const float* x, long long n, long long x_stride, long long nfft, long long le,
                                  long long lout, long long ppc, long long p0, long long rows, float2* z,
                                  hipStream_t s);
hipError_t launch_fir_long_mul(float2* Z, const float2* H, long long nfft, long long rows, hipStream_t s);
hipError_t launch_fir_long_scatter(const float2* z, float* y, long long n, long long y_stride, long long nfft,
                                   long long le, long long lout, long long ppc, long long p0, long long rows,
                                   hipStream_t s);
hipError_t launch_scale_real(float* p, long long count, float s, hipStream_t st);
hipError_t launch_scale_cpx(float2* p, long long count, float s, hipStream_t st);

// ---- DCT / Hilbert helpers (spectral_kernels.hip) ----------------------
// single-pass analytic signal / DCT-II (analytic_kernels.hip): rows [batch][n]
bool hilbert_fused_supported(long long n);
hipError_t launch_hilbert_fused(long long n, const float* x, float2* z, long long batch, hipStream_t s);
// instantaneous phase / frequency rows (phase_kernels.hip, hilbert.c:77-113)
hipError_t launch_inst_phase(const float2* z, long long n, long long batch, float* phase, hipStream_t s);
hipError_t launch_phase_unwrap(const float* p, long long n, long long batch, float* out, hipStream_t s);
// spectral_utils_kernels.hip (src/spectral/utils.c)
hipError_t launch_fftshift(const void* in, void* out, long long n, long long batch, int cpx, int inverse,
                           hipStream_t s);
hipError_t launch_phase_wrap(const float* in, float* out, long long count, hipStream_t s);
hipError_t launch_inst_freq(const float* phase, long long n, long long batch, double scale, float* freq,
                            hipStream_t s);
bool dct2_fused_supported(long long n);
hipError_t launch_dct2_fused(long long n, const float* x, float* X, long long batch, int policy, hipStream_t s);
hipError_t launch_hilbert_mask(long long n, const float2* half, float2* full, long long batch,
                               long long half_dist, hipStream_t s);
hipError_t launch_dct2_pre(long long n, const float* x, float* v, long long batch, hipStream_t s);
hipError_t launch_dct2_post(long long n, const float2* V, float* X, long long batch,
                            const float2* tw4n, hipStream_t s);
hipError_t launch_dct3_pre(long long n, const float* X, float2* V, long long batch,
                           const float2* tw4n, hipStream_t s);
hipError_t launch_dct3_post(long long n, const float* v, float* x, long long batch, float scale,
                            hipStream_t s);
hipError_t launch_dct_naive(long long n, int type, int dir, const float* in, float* out,
                            long long batch, hipStream_t s);
hipError_t launch_nan_policy(float* p, long long count, int policy, int* flag, hipStream_t s);
// czt_kernels.hip: chirp-z stages (czt.c:58-178) and the cepstrum family (cepstrum.c, minphase.c)
hipError_t launch_czt_pre(const void* x, int real_in, long long n, long long p, long long rows, long long in_dist,
                          const float2* g, float2* a, hipStream_t s);
hipError_t launch_cmul_rows(float2* a, const float2* B, long long p, long long rows, hipStream_t s);
hipError_t launch_czt_post(const float2* a, long long n, long long p, long long m, long long rows, const float2* post,
                           float2* X, long long out_dist, hipStream_t s);
hipError_t launch_log_magnitude(float2* Y, long long count, hipStream_t s);
hipError_t launch_cepstrum_fold(const float* c, long long n, long long rows, float2* C, hipStream_t s);
hipError_t launch_exp_real(float2* H, long long count, int dbl, hipStream_t s);
// the whole chirp-z chain in one kernel for P <= 4096 (Bs = FFT_P(b) / P)
bool czt_fused_supported(long long p);
// the cepstrum family in one pass per row for pow2 n <= 4096 (kind 0 cepstrum,
// 1 icepstrum_minphase, 2 minphase_from_cepstrum with complex output rows)
bool ceps_fused_supported(long long n);
hipError_t launch_ceps_fused(int kind, long long n, const float* x, long long rows, float* y, hipStream_t s);
hipError_t launch_czt_fused(long long p, const void* x, int real_in, long long n, long long m, long long rows,
                            const float2* g, const float2* Bs, const float2* post, float2* X, hipStream_t s);

}  // namespace vvh
