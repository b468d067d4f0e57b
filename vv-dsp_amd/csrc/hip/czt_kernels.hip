// czt_kernels.hip -- element-wise stages of the chirp-z transform and of the
// real cepstrum / minimum-phase family for gfx950.  The transforms between them
// are the library's own FFT launches (fft_run in shim.hip).
//
// CZT (src/spectral/czt.c:58-178), X[k] = sum_n x[n] A^-n W^(nk), k < M, as
// Bluestein's convolution with P = next_pow2(N + M - 1):
//   a[i] = x[i] g[i] (i < N, else 0),  g[n] = A^-n W^(n^2/2)      k_czt_pre
//   a <- IFFT(FFT(a) * B),  B = FFT(b), b[i] = W^(-(i-N+1)^2/2)    k_cmul_rows
//   X[k] = a[N-1+k] W^(k^2/2)                                      k_czt_post
// The chirps g, W^(k^2/2) and b are tabulated once per plan on the host in
// extended precision (the reference rounds n^2/2 and its angle to float, which
// loses the phase for N beyond a few hundred).
//
// Cepstrum (src/envelope/cepstrum.c:7-41): c = Re IFFT(log(|FFT(x)| + 1e-12)),
// computed as R2C -> log-magnitude of the n/2+1 bins -> C2R (the log-magnitude
// spectrum of a real signal is real and even, so C2R gives its real inverse).
// Minimum phase (cepstrum.c:43-78, minphase.c:7-31): the causal fold of a
// cepstrum (c0, 2c1 .. 2c(n/2-1), 0 ..), a C2C FFT, then exp of the real part.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

namespace vvh {

static inline unsigned czt_blocks(long long count) {
    long long b = (count + 255) / 256;
    if (b > 65536) b = 65536;
    if (b < 1) b = 1;
    return (unsigned)b;
}

#define CZT_GRID_STRIDE(i, count) \
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < (count); i += (long long)gridDim.x * blockDim.x)

// a[r][i] = x[r][i] * g[i] for i < n, 0 for n <= i < p; real_in: x is float[r][n]
__global__ void k_czt_pre(const void* __restrict__ x, int real_in, long long n, long long p, long long rows,
                          long long in_dist, const float2* __restrict__ g, float2* __restrict__ a) {
    CZT_GRID_STRIDE(i, p * rows) {
        const long long r = i / p, j = i - r * p;
        float2 v = make_float2(0.0f, 0.0f);
        if (j < n) {
            const float2 xv = real_in ? make_float2(static_cast<const float*>(x)[r * in_dist + j], 0.0f)
                                      : static_cast<const float2*>(x)[r * in_dist + j];
            v = cmul(xv, g[j]);
        }
        a[i] = v;
    }
}

hipError_t launch_czt_pre(const void* x, int real_in, long long n, long long p, long long rows, long long in_dist,
                          const float2* g, float2* a, hipStream_t s) {
    hipLaunchKernelGGL(k_czt_pre, dim3(czt_blocks(p * rows)), dim3(256), 0, s, x, real_in, n, p, rows, in_dist, g, a);
    return hipGetLastError();
}

// a[r][i] *= B[i] (the chirp's spectrum, shared by every row)
__global__ void k_cmul_rows(float2* __restrict__ a, const float2* __restrict__ B, long long p, long long rows) {
    CZT_GRID_STRIDE(i, p * rows) {
        const long long j = i % p;
        a[i] = cmul(a[i], B[j]);
    }
}

hipError_t launch_cmul_rows(float2* a, const float2* B, long long p, long long rows, hipStream_t s) {
    hipLaunchKernelGGL(k_cmul_rows, dim3(czt_blocks(p * rows)), dim3(256), 0, s, a, B, p, rows);
    return hipGetLastError();
}

// X[r][k] = a[r][n - 1 + k] * post[k], k < m
__global__ void k_czt_post(const float2* __restrict__ a, long long n, long long p, long long m, long long rows,
                           const float2* __restrict__ post, float2* __restrict__ X, long long out_dist) {
    CZT_GRID_STRIDE(i, m * rows) {
        const long long r = i / m, k = i - r * m;
        X[r * out_dist + k] = cmul(a[r * p + (n - 1) + k], post[k]);
    }
}

hipError_t launch_czt_post(const float2* a, long long n, long long p, long long m, long long rows, const float2* post,
                           float2* X, long long out_dist, hipStream_t s) {
    hipLaunchKernelGGL(k_czt_post, dim3(czt_blocks(m * rows)), dim3(256), 0, s, a, n, p, m, rows, post, X, out_dist);
    return hipGetLastError();
}

// Y[i] = (logf(sqrtf(re^2 + im^2) + 1e-12f), 0)  (cepstrum.c:26-32, float build)
__global__ void k_log_magnitude(float2* Y, long long count) {
    CZT_GRID_STRIDE(i, count) {
        const float2 v = Y[i];
        Y[i] = make_float2(logf(sqrtf(v.x * v.x + v.y * v.y) + 1e-12f), 0.0f);
    }
}

hipError_t launch_log_magnitude(float2* Y, long long count, hipStream_t s) {
    hipLaunchKernelGGL(k_log_magnitude, dim3(czt_blocks(count)), dim3(256), 0, s, Y, count);
    return hipGetLastError();
}

// C[r][i] = (c0, 0), (2 c[i], 0) for 1 <= i < n/2, else 0  (cepstrum.c:50-55, minphase.c:15-19)
__global__ void k_cepstrum_fold(const float* __restrict__ c, long long n, long long rows, float2* __restrict__ C) {
    const long long nh = n / 2;
    CZT_GRID_STRIDE(i, n * rows) {
        const long long j = i % n;
        float v = 0.0f;
        if (j == 0) v = c[i];
        else if (j < nh) v = 2.0f * c[i];
        C[i] = make_float2(v, 0.0f);
    }
}

hipError_t launch_cepstrum_fold(const float* c, long long n, long long rows, float2* C, hipStream_t s) {
    hipLaunchKernelGGL(k_cepstrum_fold, dim3(czt_blocks(n * rows)), dim3(256), 0, s, c, n, rows, C);
    return hipGetLastError();
}

// H[i] = (exp(Re H[i]), 0): dbl = 0 expf (cepstrum.c:64-69), 1 (float)exp((double)..) (minphase.c:24)
__global__ void k_exp_real(float2* H, long long count, int dbl) {
    CZT_GRID_STRIDE(i, count) {
        const float re = H[i].x;
        H[i] = make_float2(dbl ? (float)exp((double)re) : expf(re), 0.0f);
    }
}

hipError_t launch_exp_real(float2* H, long long count, int dbl, hipStream_t s) {
    hipLaunchKernelGGL(k_exp_real, dim3(czt_blocks(count)), dim3(256), 0, s, H, count, dbl);
    return hipGetLastError();
}

}  // namespace vvh

namespace vvh {

// ------------------------------------------------------------------------
// k_czt_fused<P>: the whole chirp-z chain for P = next_pow2(N + M - 1) <= 4096
// in one pass per row: x * g on load, the P-point forward FFT in registers,
// the product with B / P re-indexed in registers (after the forward Stockham
// passes register q holds bin t + T*m, exactly the inverse transform's input
// set, as in the FIR overlap-save kernel), the inverse FFT, and W^(k^2/2) on
// the M outputs at positions N-1+k.  HBM traffic: the row in and the M outputs
// (plus the L2-resident g, B, post tables) instead of ~4 x 16 P bytes.
// Rows are walked grid-stride by a persistent grid, the next row's samples
// prefetched into registers during the current row's transforms.
// ------------------------------------------------------------------------
template <int P, bool REAL>
__global__ void __launch_bounds__(Wg<P>::value)
k_czt_fused(const void* __restrict__ x, long long n, long long m, long long rows, const float2* __restrict__ g,
            const float2* __restrict__ Bs, const float2* __restrict__ post, float2* __restrict__ X,
            const float2* gpass, const float2* gtab) {
    using G = Geo<P>;
    constexpr int WG = Wg<P>::value, F = Wg<P>::F;
    constexpr int LDSN = G::NPASS > 1 ? F * G::LDS : 1;
    __shared__ float2 lds[LDSN];
    __shared__ float2 ltab[TwLayout<P>::ENTRIES];
    stage_twiddles<P, WG>(ltab, gpass, gtab);
    __syncthreads();
    const TwTab<P> tw{ltab};
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T;
    float2* my = lds + (G::NPASS > 1 ? slot * G::LDS : 0);
    const long long stride = (long long)gridDim.x * F;
    long long f = uni<G::T>((long long)blockIdx.x * F + slot);
    float2 nx[G::P];
    auto load = [&](long long row) {
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            const long long e = t + r * G::T;
            float2 v = make_float2(0.0f, 0.0f);
            if (e < n) {
                if constexpr (REAL) v = make_float2(static_cast<const float*>(x)[row * n + e], 0.0f);
                else v = static_cast<const float2*>(x)[row * n + e];
            }
            nx[r] = v;
        }
    };
    if (f < rows) load(f);
    for (; f < rows; f += stride) {
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            const long long e = t + r * G::T;
            v[r] = e < n ? cmul(nx[r], g[e]) : make_float2(0.0f, 0.0f);
        }
        if (f + stride < rows) load(f + stride);
        fft_regs<P, true>(v, t, my, tw);
        float2 u[G::P];
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const int mm = q / G::RL + G::NPT * (q % G::RL);   // out_pos<P>(t, q) = t + T*mm
            u[mm] = cmul(v[q], Bs[t + G::T * mm]);
        }
        fft_regs<P, false>(u, t, my, tw);
        float2* dst = X + f * m;
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const long long k = (long long)out_pos<P>(t, q) - (n - 1);
            if (k >= 0 && k < m) dst[k] = cmul(u[q], post[k]);
        }
    }
}

template <int P>
static hipError_t run_czt_fused(const void* x, int real_in, long long n, long long m, long long rows,
                                const float2* g, const float2* Bs, const float2* post, float2* X, hipStream_t s) {
    const float2* tab = twiddle_table(P);
    const float2* pas = pass_twiddles(P);
    if (!tab || !pas) return hipErrorOutOfMemory;
    constexpr int WG = Wg<P>::value, F = Wg<P>::F;
    static std::atomic<int> capc[2];
    auto go = [&](auto kern, int ri) {
        const int cap = cached_grid(capc[ri], (const void*)kern, WG, 0, 1LL << 40);
        const long long need = (rows + F - 1) / F;
        const int grid = (int)(need < cap ? need : cap);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(WG), 0, s, x, n, m, rows, g, Bs, post, X, pas, tab);
    };
    if (real_in) go(k_czt_fused<P, true>, 1);
    else go(k_czt_fused<P, false>, 0);
    return hipGetLastError();
}

bool czt_fused_supported(long long p) { return p >= 2 && p <= 4096 && (p & (p - 1)) == 0; }

// Bs = B / P (the inverse transform's scale folded into the chirp spectrum)
hipError_t launch_czt_fused(long long p, const void* x, int real_in, long long n, long long m, long long rows,
                            const float2* g, const float2* Bs, const float2* post, float2* X, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
#define VVH_CZT(PP) \
    case PP: return run_czt_fused<PP>(x, real_in, n, m, rows, g, Bs, post, X, s);
    switch (p) {
        VVH_CZT(2) VVH_CZT(4) VVH_CZT(8) VVH_CZT(16) VVH_CZT(32) VVH_CZT(64) VVH_CZT(128) VVH_CZT(256)
        VVH_CZT(512) VVH_CZT(1024) VVH_CZT(2048) VVH_CZT(4096)
        default: return hipErrorInvalidValue;
    }
#undef VVH_CZT
}

}  // namespace vvh

namespace vvh {

// ------------------------------------------------------------------------
// k_ceps_fused<N, KIND>: one row of the cepstrum family per N-point complex
// transform pair, N <= 4096, the row read once and written once:
//   KIND 0  cepstrum       x -> FFT(x + 0i) -> (log(|X| + 1e-12), 0) -> IFFT -> Re
//   KIND 1  icepstrum      c -> fold -> FFT -> (expf(Re H), 0)        -> IFFT -> Re
//   KIND 2  minphase spec  c -> fold -> FFT -> ((float)exp((double)Re H), 0)   (no inverse)
// (cepstrum.c:7-78, minphase.c:7-31, the reference's own C2C formulation).
// The element-wise step is done in the forward transform's output layout, which
// is the inverse transform's input layout after the register re-index (as in
// the FIR and CZT kernels); the 1/N of the inverse is applied at the store.
// ------------------------------------------------------------------------
template <int N, int KIND>
__global__ void __launch_bounds__(Wg<N>::value)
k_ceps_fused(const float* __restrict__ x, long long rows, float* __restrict__ y, const float2* gpass,
             const float2* gtab) {
    using G = Geo<N>;
    constexpr int WG = Wg<N>::value, F = Wg<N>::F;
    constexpr int LDSN = G::NPASS > 1 ? F * G::LDS : 1;
    __shared__ float2 lds[LDSN];
    __shared__ float2 ltab[TwLayout<N>::ENTRIES];
    stage_twiddles<N, WG>(ltab, gpass, gtab);
    __syncthreads();
    const TwTab<N> tw{ltab};
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T;
    float2* my = lds + (G::NPASS > 1 ? slot * G::LDS : 0);
    const long long stride = (long long)gridDim.x * F;
    long long f = uni<G::T>((long long)blockIdx.x * F + slot);
    float nx[G::P];
    auto load = [&](long long row) {
#pragma unroll
        for (int r = 0; r < G::P; ++r) nx[r] = x[row * N + t + r * G::T];
    };
    if (f < rows) load(f);
    for (; f < rows; f += stride) {
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            float a = nx[r];
            if constexpr (KIND != 0) {   // causal fold: c0, 2 c[i] for 1 <= i < N/2, 0 beyond
                const int e = t + r * G::T;
                a = e == 0 ? a : (e < N / 2 ? 2.0f * a : 0.0f);
            }
            v[r] = make_float2(a, 0.0f);
        }
        if (f + stride < rows) load(f + stride);
        fft_regs<N, true>(v, t, my, tw);
        if constexpr (KIND == 2) {
            float2* dst = reinterpret_cast<float2*>(y) + f * N;
#pragma unroll
            for (int q = 0; q < G::P; ++q) dst[out_pos<N>(t, q)] = make_float2((float)exp((double)v[q].x), 0.0f);
        } else {
            float2 u[G::P];
#pragma unroll
            for (int q = 0; q < G::P; ++q) {
                const int mm = q / G::RL + G::NPT * (q % G::RL);   // out_pos<N>(t, q) = t + T*mm
                const float2 z = v[q];
                const float e = KIND == 0 ? logf(sqrtf(z.x * z.x + z.y * z.y) + 1e-12f) : expf(z.x);
                u[mm] = make_float2(e, 0.0f);
            }
            fft_regs<N, false>(u, t, my, tw);
            float* dst = y + f * N;
#pragma unroll
            for (int q = 0; q < G::P; ++q) dst[out_pos<N>(t, q)] = u[q].x * (1.0f / (float)N);
        }
    }
}

bool ceps_fused_supported(long long n) { return n >= 2 && n <= 4096 && (n & (n - 1)) == 0; }

template <int N>
static hipError_t run_ceps_fused(int kind, const float* x, long long rows, float* y, hipStream_t s) {
    const float2* tab = twiddle_table(N);
    const float2* pas = pass_twiddles(N);
    if (!tab || !pas) return hipErrorOutOfMemory;
    constexpr int WG = Wg<N>::value, F = Wg<N>::F;
    static std::atomic<int> capc[3];
    auto go = [&](auto kern, int k) {
        const int cap = cached_grid(capc[k], (const void*)kern, WG, 0, 1LL << 40);
        const long long need = (rows + F - 1) / F;
        const int grid = (int)(need < cap ? need : cap);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(WG), 0, s, x, rows, y, pas, tab);
    };
    if (kind == 0) go(k_ceps_fused<N, 0>, 0);
    else if (kind == 1) go(k_ceps_fused<N, 1>, 1);
    else go(k_ceps_fused<N, 2>, 2);
    return hipGetLastError();
}

// kind 0 cepstrum, 1 icepstrum_minphase, 2 minphase_from_cepstrum (y complex[rows][n])
hipError_t launch_ceps_fused(int kind, long long n, const float* x, long long rows, float* y, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
#define VVH_CEPS(NN) \
    case NN: return run_ceps_fused<NN>(kind, x, rows, y, s);
    switch (n) {
        VVH_CEPS(2) VVH_CEPS(4) VVH_CEPS(8) VVH_CEPS(16) VVH_CEPS(32) VVH_CEPS(64) VVH_CEPS(128) VVH_CEPS(256)
        VVH_CEPS(512) VVH_CEPS(1024) VVH_CEPS(2048) VVH_CEPS(4096)
        default: return hipErrorInvalidValue;
    }
#undef VVH_CEPS
}

}  // namespace vvh
