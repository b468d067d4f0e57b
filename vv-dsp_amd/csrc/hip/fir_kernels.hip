// fir_kernels.hip -- FFT-domain FIR (overlap-save) for gfx950.
//
// vv_dsp_fir_apply_fft (src/filter/fir.c:75-135) is "the first n samples of the
// linear convolution with zero initial state"; vv_dsp_fir_apply (:160-196) is
// the same convolution continued from a (taps-1)-sample history.  Both are
// computed here as overlap-save with a fixed block of NR = 2M real samples:
//
//   block j of channel c covers input samples [j*Lout - (L-1), j*Lout + Lout)
//   (Lout = NR - (L-1)); samples before 0 come from `prefix` (history) or are 0.
//
// One workgroup-resident pass per block: R2C as an M-point complex FFT +
// split step (LDS), multiply by the precomputed H (already scaled by 1/M),
// inverse split step fused into the same loop (each thread owns bins k and
// M-k), M-point inverse FFT, and the last Lout samples are written.  The
// signal is read once from HBM (the L-1 overlap comes from L2) and the output
// written once: 8 B per sample of HBM traffic.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

#include <cstdint>

namespace vvh {

template <int M>
__device__ __forceinline__ void ols_load(float2* nx, const float* xs, const float* pre, long long seg0,
                                         long long n, long long lm1, int t) {
    using G = Geo<M>;
    constexpr long long NR = 2 * M;
    if (seg0 >= 0 && seg0 + NR <= n && (seg0 & 1) == 0) {
        const float2* src = reinterpret_cast<const float2*>(xs + seg0);
#pragma unroll
        for (int r = 0; r < G::P; ++r) nx[r] = ld_nt(src + t + r * G::T);
    } else {
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            const long long i0 = seg0 + 2 * (t + r * G::T);
            float a, b;
            if (i0 < 0) a = pre ? pre[lm1 + i0] : 0.0f; else a = (i0 < n) ? xs[i0] : 0.0f;
            if (i0 + 1 < 0) b = pre ? pre[lm1 + i0 + 1] : 0.0f; else b = (i0 + 1 < n) ? xs[i0 + 1] : 0.0f;
            nx[r] = make_float2(a, b);
        }
    }
}

// LDS: exchange buffer + twiddles + split twiddles + H (M+1 complex).  The next
// block's input is prefetched into registers during the current block.  With a
// mirror-paired forward FFT (M where Geo<M>::CAN_PAIR) each thread holds Z[k]
// and Z[M-k], forms Y = X*H for both bins and the inverse split step in
// registers, and one LDS scatter/gather re-orders Zi for the inverse FFT.
template <int M>
__global__ void __launch_bounds__(Wg<M>::value)
k_fir_ols(long long taps, const float2* Hg, const float* x, float* y, long long n, long long nch,
          long long x_stride, long long y_stride, const float* prefix, long long nblk,
          const float2* gpass, const float2* gtabM, const float2* gtab2M) {
    using G = Geo<M>;
    constexpr bool PAIR = G::CAN_PAIR;
    constexpr int WG = Wg<M>::value, F = Wg<M>::F;
    constexpr long long NR = 2 * M;
    __shared__ float2 lds[F * G::LDS];
    __shared__ float2 ltab[TwLayout<M>::ENTRIES];
    __shared__ float2 lpost[PostLayout<M>::ENTRIES];
    __shared__ float2 lH[M + 1];
    stage_twiddles<M, WG>(ltab, gpass, gtabM);
    stage_post<M, WG>(lpost, gtab2M);
    for (int i = threadIdx.x; i <= M; i += WG) lH[i] = Hg[i];
    __syncthreads();
    const TwTab<M> tw{ltab};
    const PostTab<M> pw{lpost};
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T;
    float2* my = lds + slot * G::LDS;
    const long long lm1 = taps - 1, lout = NR - lm1;
    const long long items = nch * nblk;
    const long long stride = (long long)gridDim.x * F;
    long long it = uni<G::T>((long long)blockIdx.x * F + slot);
    float2 nx[G::P];
    if (it < items) {
        const long long c = it / nblk, j = it - c * nblk;
        ols_load<M>(nx, x + c * x_stride, prefix ? prefix + c * lm1 : nullptr, j * lout - lm1, n, lm1, t);
    }
    for (; it < items; it += stride) {
        const long long c = it / nblk, j = it - c * nblk;
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = nx[r];
        const long long in_ = it + stride;
        if (in_ < items) {
            const long long c2 = in_ / nblk, j2 = in_ - c2 * nblk;
            ols_load<M>(nx, x + c2 * x_stride, prefix ? prefix + c2 * lm1 : nullptr, j2 * lout - lm1, n, lm1, t);
        }
        fft_regs<M, true, PAIR>(v, t, my, tw);
        if constexpr (PAIR) {
            float2 zi[G::P];
#pragma unroll
            for (int q = 0; q < G::P; ++q) {
                const int k = out_pos<M, true>(t, q);
                const float2 A = v[q];
                if (k == 0) {
                    const float y0 = (A.x + A.y) * lH[0].x;
                    const float ym = (A.x - A.y) * lH[M].x;
                    zi[q] = make_float2((y0 + ym) * 0.5f, (y0 - ym) * 0.5f);
                } else {
                    const float2 Bz = mirror_of<M, true>(v, t, q);
                    const float2 W = pw(k);
                    const float2 Wm = make_float2(-W.x, W.y);       // W^(M-k) = -conj(W^k)
                    const float2 Yk = cmul(split_fwd(A, cconj(Bz), W), lH[k]);
                    const float2 Ym = cmul(split_fwd(Bz, cconj(A), Wm), lH[M - k]);
                    zi[q] = split_inv(Yk, Ym, W);
                }
            }
#pragma unroll
            for (int q = 0; q < G::P; ++q) my[G::pad(out_pos<M, true>(t, q))] = zi[q];
            xsync<G::T>();
#pragma unroll
            for (int r = 0; r < G::P; ++r) v[r] = my[G::pad(t + r * G::T)];
            xsync<G::T>();
        } else {
#pragma unroll
            for (int q = 0; q < G::P; ++q) my[G::pad(out_pos<M>(t, q))] = v[q];
            xsync<G::T>();
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                const int k = t + r * G::T;
                const float2 A = my[G::pad(k)];
                if (k == 0) {
                    const float y0 = (A.x + A.y) * lH[0].x;
                    const float ym = (A.x - A.y) * lH[M].x;
                    v[r] = make_float2((y0 + ym) * 0.5f, (y0 - ym) * 0.5f);
                } else {
                    const float2 Bz = my[G::pad(M - k)];
                    const float2 W = pw(k);
                    const float2 Wm = make_float2(-W.x, W.y);
                    const float2 Yk = cmul(split_fwd(A, cconj(Bz), W), lH[k]);
                    const float2 Ym = cmul(split_fwd(Bz, cconj(A), Wm), lH[M - k]);
                    v[r] = split_inv(Yk, Ym, W);
                }
            }
            xsync<G::T>();
        }
        fft_regs<M, false>(v, t, my, tw);
        float* ys = y + c * y_stride;
        const long long ob = j * lout;
        if ((lm1 & 1) == 0 && ((reinterpret_cast<uintptr_t>(ys + ob) & 7) == 0)) {
#pragma unroll
            for (int q = 0; q < G::P; ++q) {
                const long long o0 = 2LL * out_pos<M>(t, q) - lm1;
                const long long g = ob + o0;
                if (o0 >= 0 && g + 1 < n) *(reinterpret_cast<float2*>(ys + g)) = v[q];
                else if (o0 >= 0 && g < n) *(ys + g) = v[q].x;
            }
        } else {
#pragma unroll
            for (int q = 0; q < G::P; ++q) {
                const long long o0 = 2LL * out_pos<M>(t, q) - lm1;
                const long long g = ob + o0;
                if (o0 >= 0 && g < n) *(ys + g) = v[q].x;
                if (o0 + 1 >= 0 && g + 1 < n) *(ys + g + 1) = v[q].y;
            }
        }
        xsync<G::T>();
    }
}

template <int M>
static hipError_t run_fir(long long taps, const float2* H, const float* x, float* y, long long n,
                          long long nch, long long x_stride, long long y_stride, const float* prefix,
                          hipStream_t s) {
    const long long lout = 2LL * M - (taps - 1);
    if (lout <= 0) return hipErrorInvalidValue;
    const long long nblk = (n + lout - 1) / lout;
    const float2* tM = twiddle_table(M);
    const float2* pM = pass_twiddles(M);
    const float2* t2M = twiddle_table(2 * M);
    if (!tM || !t2M || !pM) return hipErrorOutOfMemory;
    constexpr int WG = Wg<M>::value, F = Wg<M>::F;
    static int cap = 0;
    if (!cap) cap = persistent_grid((const void*)k_fir_ols<M>, WG, 0, 1LL << 40);
    const long long need = (nch * nblk + F - 1) / F;
    const int grid = (int)(need < cap ? need : cap);
    if (grid < 1) return hipSuccess;
    hipLaunchKernelGGL(k_fir_ols<M>, dim3(grid), dim3(WG), 0, s, taps, H, x, y, n, nch, x_stride, y_stride,
                       prefix, nblk, pM, tM, t2M);
    return hipGetLastError();
}

bool fir_ols_supported(long long nfft) { return nfft >= 32 && nfft <= 8192 && (nfft & (nfft - 1)) == 0; }

hipError_t launch_fir_ols(long long nfft, long long taps, const float2* H, const float* x, float* y,
                          long long n, long long nch, long long x_stride, long long y_stride,
                          const float* prefix, hipStream_t s) {
#define CALL(MM) run_fir<MM>(taps, H, x, y, n, nch, x_stride, y_stride, prefix, s)
    switch (nfft / 2) {
        case 16: return CALL(16); case 32: return CALL(32); case 64: return CALL(64);
        case 128: return CALL(128); case 256: return CALL(256); case 512: return CALL(512);
        case 1024: return CALL(1024); case 2048: return CALL(2048); case 4096: return CALL(4096);
        default: return hipErrorInvalidValue;
    }
#undef CALL
}

// ------------------------------------------------------------------------
// Direct form, bit-identical to vv_dsp_fir_apply (fir.c:170-186):
//   acc = 0; acc += h[0]*x[i]; acc += h[t]*x[i-t] for t = 1..L-1 (newest first)
// with every product and sum rounded separately (no FMA contraction), so the
// f32 result equals the reference's.  Samples before x[0] come from `prefix`.
// A block stages its input window (DIRECT_TILE + L - 1 samples) and h in LDS.
// ------------------------------------------------------------------------
constexpr int DIRECT_TILE = 1024;

__global__ void __launch_bounds__(256)
k_fir_direct(const float* __restrict__ h, long long taps, const float* __restrict__ x,
             float* __restrict__ y, long long n, long long x_stride, long long y_stride,
             const float* __restrict__ prefix, long long tiles_per_ch) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* hs = smem;                          // taps
    float* xs = smem + ((taps + 3) & ~3LL);    // DIRECT_TILE + taps - 1
    const long long c = blockIdx.x / tiles_per_ch;
    const long long i0 = (blockIdx.x % tiles_per_ch) * DIRECT_TILE;
    const long long lm1 = taps - 1;
    const float* xc = x + c * x_stride;
    const float* pc = prefix ? prefix + c * lm1 : nullptr;
    for (long long t = threadIdx.x; t < taps; t += blockDim.x) hs[t] = h[t];
    for (long long e = threadIdx.x; e < DIRECT_TILE + lm1; e += blockDim.x) {
        const long long idx = i0 - lm1 + e;
        float v;
        if (idx < 0) v = pc ? pc[lm1 + idx] : 0.0f;
        else v = (idx < n) ? xc[idx] : 0.0f;
        xs[e] = v;
    }
    __syncthreads();
    float* yc = y + c * y_stride;
    for (int o = threadIdx.x; o < DIRECT_TILE; o += blockDim.x) {
        const long long i = i0 + o;
        if (i >= n) break;
        const float* xi = xs + lm1 + o;        // xi[-t] = x[i - t]
        // hipcc contracts a*b+c into v_fma regardless of pragmas; an empty asm on
        // the product keeps the multiply and the add separately rounded.
        float acc = 0.0f;
        float p0 = hs[0] * xi[0];
        asm volatile("" : "+v"(p0));
        acc = acc + p0;
        for (long long t = 1; t < taps; ++t) {
            float pt = hs[t] * xi[-t];
            asm volatile("" : "+v"(pt));
            acc = acc + pt;
        }
        yc[i] = acc;
    }
}

hipError_t launch_fir_direct(const float* h, long long taps, const float* x, float* y, long long n,
                             long long nch, long long x_stride, long long y_stride,
                             const float* prefix, hipStream_t s) {
    const long long tiles = (n + DIRECT_TILE - 1) / DIRECT_TILE;
    if (tiles * nch <= 0) return hipSuccess;
    const size_t lds = sizeof(float) * (((taps + 3) & ~3LL) + DIRECT_TILE + taps - 1);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_fir_direct, dim3((unsigned)(tiles * nch)), dim3(256), lds, s, h, taps, x, y, n,
                       x_stride, y_stride, prefix, tiles);
    return hipGetLastError();
}

}  // namespace vvh
