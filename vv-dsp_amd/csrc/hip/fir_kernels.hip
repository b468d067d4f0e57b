// fir_kernels.hip -- FFT-domain FIR (overlap-save) for gfx950.
//
// vv_dsp_fir_apply_fft (src/filter/fir.c:75-135) is "the first n samples of the
// linear convolution with zero initial state"; vv_dsp_fir_apply (:160-196) is
// the same convolution continued from a (taps-1)-sample history.  Both are
// computed here as overlap-save with blocks of N real samples:
//
//   block j of channel c covers input samples [j*Lout - (L-1), j*Lout + Lout)
//   (Lout = N - (L-1)); samples before 0 come from `prefix` (history) or are 0;
//   outputs j*Lout + [0, Lout) are the block's circular-convolution samples
//   L-1 .. N-1.
//
// Two real blocks per complex FFT: z = a + i b (blocks j and j+1), then
// Y = FFT(z) * H with H = FFT(h)/N over all N bins, and y = IFFT(Y) holds
// a*h in its real part and b*h in its imaginary part (h is real, so the
// product keeps the two convolutions separate -- no split step at all).
// Per pair: forward N-pt FFT in registers/LDS, multiply by H (staged in LDS),
// one LDS re-order into natural order, inverse N-pt FFT, lane-contiguous
// stores.  The signal is read once from HBM (the L-1 overlap comes from L2)
// and the output written once: 8 B per sample.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

#include <cstdint>

namespace vvh {

// samples s0 + t + r*T of one block (prefix before 0, zero past n)
template <int N>
__device__ __forceinline__ void fir_blk_load(float* xr, const float* xs, const float* pre, long long s0,
                                             long long n, long long lm1, int t) {
    using G = Geo<N>;
    if (s0 >= 0 && s0 + N <= n) {
        const float* b = xs + s0;
#pragma unroll
        for (int r = 0; r < G::P; ++r) xr[r] = b[t + r * G::T];
    } else {
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            const long long i = s0 + t + r * G::T;
            float v = 0.0f;
            if (i < 0) {
                if (pre) v = pre[lm1 + i];
            } else if (i < n) {
                v = xs[i];
            }
            xr[r] = v;
        }
    }
}

template <int N>
__global__ void __launch_bounds__(Wg<N>::value)
k_fir_pair(long long taps, const float2* Hg, const float* x, float* y, long long n, long long nch,
           long long x_stride, long long y_stride, const float* prefix, long long nblk, const float2* gpass,
           const float2* gtab) {
    using G = Geo<N>;
    constexpr int WG = Wg<N>::value, F = Wg<N>::F;
    __shared__ float2 lds[F * G::LDS];
    __shared__ float2 ltab[TwLayout<N>::ENTRIES];
    __shared__ float2 lH[N];
    stage_twiddles<N, WG>(ltab, gpass, gtab);
    for (int i = threadIdx.x; i < N; i += WG) lH[i] = Hg[i];
    __syncthreads();
    const TwTab<N> tw{ltab};
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T;
    float2* my = lds + slot * G::LDS;
    const long long lm1 = taps - 1, lout = N - lm1;
    const long long ppc = (nblk + 1) / 2;   // block pairs per channel
    long long p, p_end;
    chunk_of(nch * ppc, (long long)blockIdx.x * F + slot, (long long)gridDim.x * F, &p, &p_end);
    p = uni<G::T>(p);
    p_end = uni<G::T>(p_end);
    if (p >= p_end) return;   // uniform per transform (F == 1 whenever T > 64)
    long long c = p / ppc, j = 2 * (p - c * ppc);
    float xa[G::P], xb[G::P];
    auto load_pair = [&](long long cc, long long jj) {
        const float* xs = x + cc * x_stride;
        const float* pre = prefix ? prefix + cc * lm1 : nullptr;
        fir_blk_load<N>(xa, xs, pre, jj * lout - lm1, n, lm1, t);
        fir_blk_load<N>(xb, xs, pre, (jj + 1) * lout - lm1, n, lm1, t);
    };
    load_pair(c, j);
    for (; p < p_end; ++p) {
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = make_float2(xa[r], xb[r]);
        long long cn = c, jn = j + 2;
        if (jn >= 2 * ppc) {
            jn = 0;
            ++cn;
        }
        if (p + 1 < p_end) load_pair(cn, jn);
        fft_regs<N, true>(v, t, my, tw);
        // Y = Z * H, re-ordered to natural order for the inverse transform
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const int k = out_pos<N>(t, q);
            my[G::pad(k)] = cmul(v[q], lH[k]);
        }
        xsync<G::T>();
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = my[G::pad(t + r * G::T)];
        xsync<G::T>();
        fft_regs<N, false>(v, t, my, tw);
        // circular samples e >= L-1 are outputs: Re -> block j, Im -> block j+1
        float* ys = y + c * y_stride;
        const long long oa0 = j * lout - lm1;
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const long long e = out_pos<N>(t, q);
            if (e >= lm1) {
                const long long oa = oa0 + e, ob = oa + lout;
                if (oa < n) ys[oa] = v[q].x;
                if (ob < n) ys[ob] = v[q].y;
            }
        }
        c = cn;
        j = jn;
    }
}

template <int N>
static hipError_t run_fir(long long taps, const float2* H, const float* x, float* y, long long n,
                          long long nch, long long x_stride, long long y_stride, const float* prefix,
                          hipStream_t s) {
    const long long lout = (long long)N - (taps - 1);
    if (lout <= 0) return hipErrorInvalidValue;
    const long long nblk = (n + lout - 1) / lout;
    const float2* tN = twiddle_table(N);
    const float2* pN = pass_twiddles(N);
    if (!tN || !pN) return hipErrorOutOfMemory;
    constexpr int WG = Wg<N>::value, F = Wg<N>::F;
    static int cap = 0;
    if (!cap) cap = persistent_grid((const void*)k_fir_pair<N>, WG, 0, 1LL << 40);
    const long long need = (nch * ((nblk + 1) / 2) + F - 1) / F;
    const int grid = (int)(need < cap ? need : cap);
    if (grid < 1) return hipSuccess;
    hipLaunchKernelGGL(k_fir_pair<N>, dim3(grid), dim3(WG), 0, s, taps, H, x, y, n, nch, x_stride, y_stride,
                       prefix, nblk, pN, tN);
    return hipGetLastError();
}

bool fir_ols_supported(long long nfft) { return nfft >= 64 && nfft <= 8192 && (nfft & (nfft - 1)) == 0; }

// H: N complex bins of FFT(h zero-padded to N) / N
hipError_t launch_fir_ols(long long nfft, long long taps, const float2* H, const float* x, float* y,
                          long long n, long long nch, long long x_stride, long long y_stride,
                          const float* prefix, hipStream_t s) {
#define CALL(NN) run_fir<NN>(taps, H, x, y, n, nch, x_stride, y_stride, prefix, s)
    switch (nfft) {
        case 64: return CALL(64); case 128: return CALL(128); case 256: return CALL(256);
        case 512: return CALL(512); case 1024: return CALL(1024); case 2048: return CALL(2048);
        case 4096: return CALL(4096); case 8192: return CALL(8192);
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
