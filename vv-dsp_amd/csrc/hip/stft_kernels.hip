// stft_kernels.hip -- fused STFT analysis for gfx950.
//
// One persistent kernel per power-of-two nfft (= 2M): for every (channel,
// frame) it gathers the frame (zero past the end of the signal, as
// stft.c:124-130), applies the window (vectorized_math_fallback.c:13-29), runs
// the real FFT as an M-point complex Stockham FFT in VGPRs/LDS plus the split
// step, and writes either magnitudes sqrtf(re^2+im^2) for all nfft bins
// (stft.c:133-139) or the full complex spectrum (stft_process semantics,
// stft.c:74-92) using X[nfft-k] = conj(X[k]).
//
// Memory behaviour: the next frame's samples are prefetched into registers
// while the current frame is transformed; window and twiddles live in LDS, so
// the only VMEM traffic is the streamed signal (re-reads of the nfft-hop
// overlap hit L2) and the output rows.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

#include <cstdint>

namespace vvh {

template <int M>
__device__ __forceinline__ void stft_load(float2* nx, const float* s, long long start, long long n, int t) {
    using G = Geo<M>;
    constexpr int NR = 2 * M;
    const float* base = s + start;
    if (start + NR <= n && ((reinterpret_cast<uintptr_t>(base) & 7) == 0)) {
        const float2* b2 = reinterpret_cast<const float2*>(base);
#pragma unroll
        for (int r = 0; r < G::P; ++r) nx[r] = b2[t + r * G::T];
    } else {
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            const long long e = 2 * (t + r * G::T);
            nx[r] = make_float2((start + e < n) ? base[e] : 0.0f, (start + e + 1 < n) ? base[e + 1] : 0.0f);
        }
    }
}

// MODE 0: out = float mags [ch][frame][2M]; MODE 1: out = float2 spectrum [ch][frame][2M]
template <int M, int MODE>
__global__ void __launch_bounds__(Wg<M>::value)
k_stft(const float* sig, long long n, long long nch, long long ch_stride, long long frames,
       long long hop, const float* win, void* out, long long out_ch_stride, const float2* gtabM,
       const float2* gtab2M) {
    using G = Geo<M>;
    constexpr int WG = Wg<M>::value, F = Wg<M>::F;
    constexpr int NR = 2 * M;
    __shared__ float2 lds[F * G::LDS];
    __shared__ float2 ltab[TwLayout<M>::ENTRIES];
    __shared__ float2 lpost[PostLayout<M>::ENTRIES];
    __shared__ float2 lwin[M];
    stage_twiddles<M, WG>(ltab, gtabM);
    stage_post<M, WG>(lpost, gtab2M);
    for (int i = threadIdx.x; i < M; i += WG) lwin[i] = make_float2(win[2 * i], win[2 * i + 1]);
    __syncthreads();
    const auto tw = twiddles_from<M>(ltab);
    const auto pw = post_from<M>(lpost);
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T;
    float2* my = lds + slot * G::LDS;
    const long long items = nch * frames;
    const long long stride = (long long)gridDim.x * F;
    long long it = (long long)blockIdx.x * F + slot;
    float2 nx[G::P];
    if (it < items) {
        const long long c = it / frames, fr = it - c * frames;
        stft_load<M>(nx, sig + c * ch_stride, fr * hop, n, t);
    }
    for (; it < items; it += stride) {
        const long long c = it / frames, fr = it - c * frames;
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            const float2 w = lwin[t + r * G::T];
            v[r] = make_float2(nx[r].x * w.x, nx[r].y * w.y);
        }
        const long long in_ = it + stride;
        if (in_ < items) {
            const long long c2 = in_ / frames, fr2 = in_ - c2 * frames;
            stft_load<M>(nx, sig + c2 * ch_stride, fr2 * hop, n, t);
        }
        fft_regs<M, true>(v, t, my, tw);
#pragma unroll
        for (int q = 0; q < G::P; ++q) my[G::pad(out_pos<M>(t, q))] = v[q];
        xsync<G::T>();
        const long long row = c * out_ch_stride + fr * (long long)NR;
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const int k = t + G::T * q;
            const float2 A = my[G::pad(k)];
            if (MODE == 0) {
                float* o = reinterpret_cast<float*>(out) + row;
                if (k == 0) {
                    const float x0 = A.x + A.y, xm = A.x - A.y;
                    __builtin_nontemporal_store(sqrtf(x0 * x0), o);
                    __builtin_nontemporal_store(sqrtf(xm * xm), o + M);
                } else {
                    const float2 X = split_fwd(A, cconj(my[G::pad(M - k)]), pw(k));
                    const float mag = sqrtf(X.x * X.x + X.y * X.y);
                    __builtin_nontemporal_store(mag, o + k);
                    __builtin_nontemporal_store(mag, o + (NR - k));
                }
            } else {
                float2* o = reinterpret_cast<float2*>(out) + row;
                if (k == 0) {
                    st_nt(make_float2(A.x + A.y, 0.0f), o);
                    st_nt(make_float2(A.x - A.y, 0.0f), o + M);
                } else {
                    const float2 X = split_fwd(A, cconj(my[G::pad(M - k)]), pw(k));
                    st_nt(X, o + k);
                    st_nt(cconj(X), o + (NR - k));
                }
            }
        }
        xsync<G::T>();
    }
}

template <int M, int MODE>
static hipError_t run_stft(const float* sig, long long n, long long nch, long long ch_stride,
                           long long frames, long long hop, const float* win, void* out,
                           long long out_ch_stride, hipStream_t s) {
    const float2* tM = twiddle_table(M);
    const float2* t2M = twiddle_table(2 * M);
    if (!tM || !t2M) return hipErrorOutOfMemory;
    constexpr int WG = Wg<M>::value, F = Wg<M>::F;
    static int cap = 0;
    if (!cap) cap = persistent_grid((const void*)k_stft<M, MODE>, WG, 0, 1LL << 40);
    const long long need = (nch * frames + F - 1) / F;
    const int grid = (int)(need < cap ? need : cap);
    if (grid < 1) return hipSuccess;
    hipLaunchKernelGGL((k_stft<M, MODE>), dim3(grid), dim3(WG), 0, s, sig, n, nch, ch_stride, frames,
                       hop, win, out, out_ch_stride, tM, t2M);
    return hipGetLastError();
}

bool stft_fused_supported(long long nfft) {
    return nfft >= 4 && nfft <= 8192 && (nfft & (nfft - 1)) == 0;
}

hipError_t launch_stft(long long nfft, long long hop, int mode, const float* sig, long long n,
                       long long nch, long long ch_stride, long long frames, const float* win,
                       void* out, long long out_ch_stride, hipStream_t s) {
#define CALL(MM)                                                                                   \
    (mode == 0 ? run_stft<MM, 0>(sig, n, nch, ch_stride, frames, hop, win, out, out_ch_stride, s)   \
               : run_stft<MM, 1>(sig, n, nch, ch_stride, frames, hop, win, out, out_ch_stride, s))
    switch (nfft / 2) {
        case 2: return CALL(2); case 4: return CALL(4); case 8: return CALL(8);
        case 16: return CALL(16); case 32: return CALL(32); case 64: return CALL(64);
        case 128: return CALL(128); case 256: return CALL(256); case 512: return CALL(512);
        case 1024: return CALL(1024); case 2048: return CALL(2048); case 4096: return CALL(4096);
        default: return hipErrorInvalidValue;
    }
#undef CALL
}

// stft_process over explicit frames [count][nfft] (no overlap): same kernel, hop = nfft.
hipError_t launch_stft_frames(long long nfft, const float* frames_in, const float* win, float2* out,
                              long long count, hipStream_t s) {
    return launch_stft(nfft, nfft, 1, frames_in, nfft * count, 1, 0, count, win, out, 0, s);
}

// ---- generic path (any nfft): gather windowed complex frames, then a batched
// C2C plan, then magnitudes.
__global__ void k_frame_gather(long long nfft, long long hop, const float* sig, long long n,
                               long long nch, long long ch_stride, long long frames,
                               const float* win, float2* out) {
    const long long total = nch * frames * nfft;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long e = i % nfft, fr = (i / nfft) % frames, c = i / (nfft * frames);
        const long long idx = fr * hop + e;
        const float v = (idx < n) ? sig[c * ch_stride + idx] : 0.0f;
        out[i] = make_float2(v * win[e], 0.0f);
    }
}

hipError_t launch_frame_gather(long long nfft, long long hop, const float* sig, long long n,
                               long long nch, long long ch_stride, long long frames, const float* win,
                               float2* out, hipStream_t s) {
    const long long total = nch * frames * nfft;
    if (total <= 0) return hipSuccess;
    long long blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_frame_gather, dim3((unsigned)blocks), dim3(256), 0, s, nfft, hop, sig, n, nch,
                       ch_stride, frames, win, out);
    return hipGetLastError();
}

__global__ void k_magnitude(const float2* in, float* out, long long count) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < count;
         i += (long long)gridDim.x * blockDim.x) {
        const float2 v = in[i];
        out[i] = sqrtf(v.x * v.x + v.y * v.y);
    }
}

hipError_t launch_magnitude(const float2* in, float* out, long long count, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    long long blocks = (count + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_magnitude, dim3((unsigned)blocks), dim3(256), 0, s, in, out, count);
    return hipGetLastError();
}

// ISTFT accumulate for `count` frames placed at multiples of hop (stft.c:95-110
// applied frame after frame).  One thread per output sample sums its frames in
// frame order, so the f32 rounding matches sequential accumulation.
__global__ void k_ola(long long nfft, long long hop, const float2* tf, long long count,
                      const float* win, float* out_add, float* norm_add, long long len) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < len;
         i += (long long)gridDim.x * blockDim.x) {
        long long f_hi = i / hop;
        if (f_hi > count - 1) f_hi = count - 1;
        long long f_lo = (i - nfft + 1 + hop - 1) / hop;
        if (i - nfft + 1 <= 0) f_lo = 0;
        float acc = out_add[i];
        float nacc = norm_add ? norm_add[i] : 0.0f;
        for (long long f = f_lo; f <= f_hi; ++f) {
            const long long e = i - f * hop;
            if (e < 0 || e >= nfft) continue;
            const float w = win[e];
            acc += tf[f * nfft + e].x * w;
            nacc += w * w;
        }
        out_add[i] = acc;
        if (norm_add) norm_add[i] = nacc;
    }
}

hipError_t launch_ola(long long nfft, long long hop, const float2* time_frames, long long count,
                      const float* win, float* out_add, float* norm_add, hipStream_t s) {
    const long long len = (count - 1) * hop + nfft;
    if (count <= 0) return hipSuccess;
    long long blocks = (len + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_ola, dim3((unsigned)blocks), dim3(256), 0, s, nfft, hop, time_frames, count, win,
                       out_add, norm_add, len);
    return hipGetLastError();
}

}  // namespace vvh
