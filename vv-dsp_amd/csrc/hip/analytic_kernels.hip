// analytic_kernels.hip -- single-pass Hilbert analytic signal and DCT-II for
// gfx950: one HBM read of the input rows and one write of the output rows,
// two rows per complex FFT, everything else in registers/LDS.
//
// Hilbert (src/spectral/hilbert.c:14-75): z = IFFT(m . FFT(x)) with the
// one-sided mask m = 1 at DC and N/2, 2 on 1..N/2-1, 0 above, and the
// backward transform scaled by 1/N (fft_kiss.c:45,70-73).  Two real rows a, b
// share one forward FFT of a + i b; since the mask is linear,
//   w = IFFT(m . FFT(a + i b)) = za + i zb,  za = a + i ha,  zb = b + i hb,
// so  Re w = a - hb  and  Im w = ha + b:  the two analytic signals are
//   za = (a, Im w - b),  zb = (b, a - Re w)
// with a and b kept in registers.  After the forward Stockham FFT thread t
// holds Z[t + T m], exactly the input set of the inverse FFT (register
// re-index, no LDS re-order), and after the inverse it holds w[t + T m], the
// same index set as its a[m], b[m].  Replaces R2C + mask + C2C (36 B/point of
// HBM traffic) with 12 B/point.
//
// DCT-II (src/spectral/dct.c:21-30, X[k] = sum x[n] cos(pi (n+1/2) k / N)) by
// Makhoul's permutation v[j] = x[2j] (j < N/2), v[N-1-j] = x[2j+1], an N-point
// FFT and X[k] = Re(W_4N^k V[k]).  Two rows per complex FFT with the
// mirror-paired last pass: Va[k] = (Z[k] + conj Z[N-k])/2,
// Vb[k] = (Z[k] - conj Z[N-k])/2i straight from registers.  The NaN policy
// (src/core/nan_policy.c) is applied as the input is read and as the output is
// written, like dct.c:98,130 (propagate, zero, clamp; the error policy keeps
// the multi-pass path, which must scan first).
// Replaces copy + policy + permute + R2C + post (≈40 B/point) with 8 B/point.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

namespace vvh {

template <int N>
__global__ void __launch_bounds__(Wg<N>::value)
k_hilbert_pair(const float* __restrict__ x, float2* __restrict__ z, long long batch, long long x_dist,
               long long z_dist, const float2* gpass, const float2* gtab) {
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
    const long long pairs = (batch + 1) / 2;
    const float inv = 1.0f / (float)N;
    for (long long p = uni<G::T>((long long)blockIdx.x * F + slot); p < pairs; p += (long long)gridDim.x * F) {
        const long long ra = 2 * p;
        const bool hb = ra + 1 < batch;
        const float* xa = x + ra * x_dist;
        const float* xb = hb ? xa + x_dist : xa;   // unconditional loads (no exec-masked branch)
        float a[G::P], b[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            a[r] = xa[t + r * G::T];
            b[r] = xb[t + r * G::T];
        }
#pragma unroll
        for (int r = 0; r < G::P; ++r) b[r] = hb ? b[r] : 0.0f;
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = make_float2(a[r], b[r]);
        fft_regs<N, true>(v, t, my, tw);
        float2 u[G::P];
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const int m = q / G::RL + G::NPT * (q % G::RL);   // out_pos<N>(t, q) = t + T*m
            const int k = t + G::T * m;
            const float s = (k == 0 || 2 * k == N) ? 1.0f : (2 * k < N ? 2.0f : 0.0f);
            u[m] = cscale(v[q], s);
        }
        fft_regs<N, false>(u, t, my, tw);
        float2* za = z + ra * z_dist;
        float2* zb = za + z_dist;
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const int m = q / G::RL + G::NPT * (q % G::RL);
            const int k = t + G::T * m;
            const float2 w = cscale(u[q], inv);
            st_nt(make_float2(a[m], w.y - b[m]), za + k);
            if (hb) st_nt(make_float2(b[m], a[m] - w.x), zb + k);
        }
    }
}

// Small N (16..128) with dense rows: k_hilbert_pair's arithmetic with each wave's
// 2 x 64 / T input rows (2048 floats) loaded as 16 B per lane and re-laid through
// LDS, and its complex outputs staged the same way (even rows, then odd rows) --
// lane-strided 4 / 8 B accesses touched 16..64 lines per instruction; a
// wave-uniform loop.
template <int N>
__global__ void __launch_bounds__(256, N >= 32 ? 3 : 4)
k_hilbert_small(const float* __restrict__ x, float2* __restrict__ z, long long batch, const float2* gpass,
                const float2* gtab) {
    using G = Geo<N>;
    static_assert(G::P == 16 && G::T <= 8, "16..128 points");
    constexpr int F = 256 / G::T, WS = 64 / G::T, WF = 2048 + 128;   // floats per wave area
    constexpr int LDSN = (F * G::LDS > 4 * WF / 2) ? F * G::LDS : 4 * WF / 2;
    __shared__ __attribute__((aligned(16))) float2 lds[LDSN];
    __shared__ float2 ltab[TwLayout<N>::ENTRIES];
    stage_twiddles<N, 256>(ltab, gpass, gtab);
    __syncthreads();
    const TwTab<N> tw{ltab};
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T, wv = lt >> 6, lane = lt & 63, sl = slot - wv * WS;
    float2* my = lds + (G::NPASS > 1 ? slot * G::LDS : 0);
    float* wa = reinterpret_cast<float*>(lds) + wv * WF;
    auto padf = [](int e) { return e + (e >> 4); };
    const long long pairs = (batch + 1) / 2;
    const float inv = 1.0f / (float)N;
    for (long long pw = (long long)blockIdx.x * F + (long long)wv * WS; pw < pairs; pw += (long long)gridDim.x * F) {
        const long long r0 = 2 * pw;
        const long long nr = batch - r0 < 2 * WS ? batch - r0 : 2 * WS;
        const int nval = (int)nr * N;
        {
            vf4_t blk[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int e = i * 256 + 4 * lane;
                blk[i] = e < nval ? __builtin_nontemporal_load(reinterpret_cast<const vf4_t*>(x + r0 * N + e))
                                  : vf4_t{0.0f, 0.0f, 0.0f, 0.0f};
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int e = i * 256 + 4 * lane;
#pragma unroll
                for (int k = 0; k < 4; ++k) wa[padf(e + k)] = blk[i][k];
            }
        }
        xsync<64>();
        float a[G::P], b[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            a[r] = wa[padf(2 * sl * N + t + r * G::T)];
            b[r] = wa[padf((2 * sl + 1) * N + t + r * G::T)];
        }
        xsync<64>();
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = make_float2(a[r], b[r]);
        fft_regs<N, true>(v, t, my, tw);
        float2 u[G::P];
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const int m = q / G::RL + G::NPT * (q % G::RL);   // out_pos<N>(t, q) = t + T*m
            const int k = t + G::T * m;
            const float sc = (k == 0 || 2 * k == N) ? 1.0f : (2 * k < N ? 2.0f : 0.0f);
            u[m] = cscale(v[q], sc);
        }
        fft_regs<N, false>(u, t, my, tw);
        // outputs as k_hilbert_pair (row 2 sl: (a, w.y - b), row 2 sl + 1: (b, a - w.x)),
        // staged in two passes -- the wave's even rows, then its odd rows (WS rows x N
        // complex, padded 1 per 16 in the area) -- and stored as 16 B per lane, row
        // segments of N complex
        float2* wc = reinterpret_cast<float2*>(wa);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            xsync<64>();
#pragma unroll
            for (int q = 0; q < G::P; ++q) {
                const int m = q / G::RL + G::NPT * (q % G::RL);
                const int k = t + G::T * m;
                const float2 w = cscale(u[q], inv);
                wc[G::pad(sl * N + k)] = h == 0 ? make_float2(a[m], w.y - b[m]) : make_float2(b[m], a[m] - w.x);
            }
            xsync<64>();
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int e = i * 128 + 2 * lane;        // complex index among the WS rows
                const int row = e / N, col = e - row * N;   // N >= 16: e, e + 1 in one row
                const long long gr = r0 + 2 * row + h;      // its row of the batch
                if (gr < batch) {
                    const float2 c0 = wc[G::pad(e)], c1 = wc[G::pad(e + 1)];
                    __builtin_nontemporal_store(vf4_t{c0.x, c0.y, c1.x, c1.y},
                                                reinterpret_cast<vf4_t*>(z + gr * N + col));
                }
            }
        }
        xsync<64>();
    }
}

bool hilbert_fused_supported(long long n) { return n >= 2 && n <= 8192 && (n & (n - 1)) == 0; }

hipError_t launch_hilbert_fused(long long n, const float* x, float2* z, long long batch, hipStream_t s) {
    if (batch <= 0) return hipSuccess;
    // 16..128 points: the staged kernel (knob HIL_SMALL = 0 keeps k_hilbert_pair, A/B)
    if (n >= 16 && n <= 128 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)z & 15) == 0 && knob(KNOB_HIL_SMALL, 1) == 1) {
#define VVH_HILS(NN)                                                                                          \
        case NN: {                                                                                            \
            const float2* tab = twiddle_table(NN);                                                            \
            const float2* pas = pass_twiddles(NN);                                                            \
            if (!tab || !pas) return hipErrorOutOfMemory;                                                     \
            constexpr int F = 256 / Geo<NN>::T;                                                               \
            const long long need = ((batch + 1) / 2 + F - 1) / F;                                             \
            const int grid = (int)(need < (1LL << 30) ? need : (1LL << 30));                                  \
            hipLaunchKernelGGL((k_hilbert_small<NN>), dim3(grid), dim3(256), 0, s, x, z, batch, pas, tab);    \
            return hipGetLastError();                                                                         \
        }
        switch (n) {
            VVH_HILS(16) VVH_HILS(32) VVH_HILS(64) VVH_HILS(128)
            default: break;
        }
#undef VVH_HILS
    }
#define VVH_HIL(NN)                                                                                         \
    case NN: {                                                                                              \
        const float2* tab = twiddle_table(NN);                                                              \
        const float2* pas = pass_twiddles(NN);                                                              \
        if (!tab || !pas) return hipErrorOutOfMemory;                                                       \
        constexpr int WG = Wg<NN>::value, F = Wg<NN>::F;                                                    \
        static std::atomic<int> capc;                                                                                 \
        const int cap0 = cached_grid(capc, (const void*)k_hilbert_pair<NN>, WG, 0, 1LL << 40);                \
        /* knob ANA_TPW = 1: not persistent (A/B; Hilbert 1024 / 4096 +6 %, r05_ab2_analytic_mixed_grid) */ \
        const long long cap = knob(KNOB_ANA_TPW, 0) == 1 ? (1LL << 30) : cap0;                              \
        const long long need = ((batch + 1) / 2 + F - 1) / F;                                               \
        const int grid = (int)(need < cap ? need : cap);                                                    \
        hipLaunchKernelGGL(k_hilbert_pair<NN>, dim3(grid), dim3(WG), 0, s, x, z, batch, n, n, pas, tab);    \
        return hipGetLastError();                                                                           \
    }
    switch (n) {
        VVH_HIL(2) VVH_HIL(4) VVH_HIL(8) VVH_HIL(16) VVH_HIL(32) VVH_HIL(64) VVH_HIL(128) VVH_HIL(256)
        VVH_HIL(512) VVH_HIL(1024) VVH_HIL(2048) VVH_HIL(4096) VVH_HIL(8192)
        default: return hipErrorInvalidValue;
    }
#undef VVH_HIL
}

// NaN policy (src/core/nan_policy.c): 0 propagate, 1 zero, 3 clamp
template <int POL>
__device__ __forceinline__ float nan_fix(float v) {
    if constexpr (POL == 0) return v;
    else if constexpr (POL == 1) return isfinite(v) ? v : 0.0f;
    else return isfinite(v) ? v : (isnan(v) ? 0.0f : (v > 0 ? 3.402823466e+38f : -3.402823466e+38f));
}

template <int N, int POL>
__global__ void __launch_bounds__(Wg<N>::value)
k_dct2_pair(const float* __restrict__ x, float* __restrict__ X, long long batch, long long dist,
            const float2* gpass, const float2* gtab, const float2* __restrict__ tw4n) {
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
    // W_4N^k for this thread's output bins (loop invariant).  PAIRV: bins k =
    // out_pos(t, q) of the mirror-paired last pass; otherwise (N = 256: one last-pass
    // butterfly per thread) bins k = t + T r, whose mirrors N - k are read back
    // through LDS
    constexpr bool PAIRV = G::CAN_PAIR;
    float2 wk[G::P];
    int kq[G::P];
#pragma unroll
    for (int q = 0; q < G::P; ++q) {
        kq[q] = PAIRV ? out_pos<N, true>(t, q) : t + G::T * q;
        wk[q] = tw4n[kq[q]];
    }
    const long long pairs = (batch + 1) / 2;
    for (long long p = uni<G::T>((long long)blockIdx.x * F + slot); p < pairs; p += (long long)gridDim.x * F) {
        const long long ra = 2 * p;
        const bool hb = ra + 1 < batch;
        const float* xa = x + ra * dist;
        const float* xb = hb ? xa + dist : xa;   // unconditional loads; b zeroed below when absent
        float2 v[G::P];
        if constexpr (G::T == 1) {   // one thread owns the row pair: permute in registers
#pragma unroll
            for (int j = 0; j < G::P; ++j) {
                const int src = j < N / 2 ? 2 * j : 2 * N - 2 * j - 1;
                const float bv = xb[src];
                v[j] = make_float2(nan_fix<POL>(xa[src]), hb ? nan_fix<POL>(bv) : 0.0f);
            }
        } else {   // coalesced loads, Makhoul permutation through LDS
            float a[G::P], b[G::P];
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                a[r] = xa[t + r * G::T];
                b[r] = xb[t + r * G::T];
            }
#pragma unroll
            for (int r = 0; r < G::P; ++r)
                my[G::pad(t + r * G::T)] = make_float2(nan_fix<POL>(a[r]), hb ? nan_fix<POL>(b[r]) : 0.0f);
            xsync<G::T>();
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                const int j = t + r * G::T;
                v[r] = my[G::pad(j < N / 2 ? 2 * j : 2 * N - 2 * j - 1)];
            }
            xsync<G::T>();   // the FFT's first exchange overwrites `my`
        }
        float* oa = X + ra * dist;
        float* ob = oa + dist;
        if constexpr (!PAIRV) {
            // natural last-pass layout, then (Z[k], Z[N - k]) from LDS for k = t + T r:
            // lane-contiguous bins, stored straight out
            fft_regs<N, true, false>(v, t, my, tw);
#pragma unroll
            for (int q = 0; q < G::P; ++q) my[G::pad(out_pos<N>(t, q))] = v[q];
            xsync<G::T>();
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                const int k = kq[r];
                const float2 Z = my[G::pad(k)], Zm = my[G::pad((N - k) & (N - 1))];
                const float2 Va = make_float2(0.5f * (Z.x + Zm.x), 0.5f * (Z.y - Zm.y));
                const float2 Vb = make_float2(0.5f * (Z.y + Zm.y), -0.5f * (Z.x - Zm.x));
                const float2 W = wk[r];
                __builtin_nontemporal_store(nan_fix<POL>(W.x * Va.x - W.y * Va.y), oa + k);
                if (hb) __builtin_nontemporal_store(nan_fix<POL>(W.x * Vb.x - W.y * Vb.y), ob + k);
            }
            xsync<G::T>();   // the next row pair's permutation overwrites `my`
            continue;
        } else {
            fft_regs<N, true, true>(v, t, my, tw);
        }
        float2 o[G::P];   // (Xa[k], Xb[k]) at k = kq[q]
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const float2 Z = v[q], Zm = mirror_of<N, true>(v, t, q);
            const float2 Va = make_float2(0.5f * (Z.x + Zm.x), 0.5f * (Z.y - Zm.y));
            const float2 Vb = make_float2(0.5f * (Z.y + Zm.y), -0.5f * (Z.x - Zm.x));
            const float2 W = wk[q];
            // policy on the output too (dct.c:130)
            o[q] = make_float2(nan_fix<POL>(W.x * Va.x - W.y * Va.y), nan_fix<POL>(W.x * Vb.x - W.y * Vb.y));
        }
        if constexpr (G::T == 1) {
#pragma unroll
            for (int q = 0; q < G::P; ++q) {
                oa[kq[q]] = o[q].x;
                if (hb) ob[kq[q]] = o[q].y;
            }
        } else {   // back to natural order through LDS: lane-contiguous, full-line stores
#pragma unroll
            for (int q = 0; q < G::P; ++q) my[G::pad(kq[q])] = o[q];
            xsync<G::T>();
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                const int k = t + r * G::T;
                const float2 x2 = my[G::pad(k)];
                __builtin_nontemporal_store(x2.x, oa + k);
                if (hb) __builtin_nontemporal_store(x2.y, ob + k);
            }
            xsync<G::T>();
        }
    }
}

// Small N (16..128, several row pairs per wave) with dense rows: the same
// transform as k_dct2_pair, but a wave's 2 * 64 / T rows (2048 consecutive
// floats) are loaded as 16 B per lane and re-laid through LDS (padded 1 per 16
// floats), and its outputs leave the same way -- lane-strided 4 B accesses
// touched 16 lines per instruction (0.10 of the roofline at 64 points).  The
// loop is wave-uniform; slots past the batch compute on zeros and store nothing.
template <int N, int POL>
__global__ void __launch_bounds__(256, N >= 32 ? 3 : 4)
k_dct2_small(const float* __restrict__ x, float* __restrict__ X, long long batch, const float2* gpass,
             const float2* gtab, const float2* __restrict__ tw4n) {
    using G = Geo<N>;
    static_assert(G::P == 16 && G::T <= 8 && G::CAN_PAIR, "16..128 points");
    constexpr int F = 256 / G::T, WS = 64 / G::T, WF = 2048 + 128;   // floats per wave area
    constexpr int LDSN = (F * G::LDS > 4 * WF / 2) ? F * G::LDS : 4 * WF / 2;
    __shared__ __attribute__((aligned(16))) float2 lds[LDSN];
    __shared__ float2 ltab[TwLayout<N>::ENTRIES];
    __shared__ float2 lw4[N];   // W_4N^k, k < N (read per output bin: no registers held)
    stage_twiddles<N, 256>(ltab, gpass, gtab);
    for (int i = threadIdx.x; i < N; i += 256) lw4[i] = tw4n[i];
    __syncthreads();
    const TwTab<N> tw{ltab};
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T, wv = lt >> 6, lane = lt & 63, sl = slot - wv * WS;
    float2* my = lds + (G::NPASS > 1 ? slot * G::LDS : 0);
    float* wa = reinterpret_cast<float*>(lds) + wv * WF;   // the wave's staging area (its slots' buffers)
    auto padf = [](int e) { return e + (e >> 4); };
    const long long pairs = (batch + 1) / 2;
    for (long long pw = (long long)blockIdx.x * F + (long long)wv * WS; pw < pairs; pw += (long long)gridDim.x * F) {
        const long long r0 = 2 * pw;                       // the wave's first row
        const long long nr = batch - r0 < 2 * WS ? batch - r0 : 2 * WS;
        const int nval = (int)nr * N;                      // valid floats of the block
        {
            vf4_t blk[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int e = i * 256 + 4 * lane;
                blk[i] = e < nval ? __builtin_nontemporal_load(reinterpret_cast<const vf4_t*>(x + r0 * N + e))
                                  : vf4_t{0.0f, 0.0f, 0.0f, 0.0f};
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int e = i * 256 + 4 * lane;
#pragma unroll
                for (int k = 0; k < 4; ++k) wa[padf(e + k)] = blk[i][k];
            }
        }
        xsync<64>();
        float a[G::P], b[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            a[r] = wa[padf(2 * sl * N + t + r * G::T)];
            b[r] = wa[padf((2 * sl + 1) * N + t + r * G::T)];
        }
        xsync<64>();   // the permutation below and the FFT reuse the area
        float2 v[G::P];
        if constexpr (G::T == 1) {
#pragma unroll
            for (int j = 0; j < G::P; ++j) {
                const int src = j < N / 2 ? 2 * j : 2 * N - 2 * j - 1;
                v[j] = make_float2(nan_fix<POL>(a[src]), nan_fix<POL>(b[src]));
            }
        } else {
#pragma unroll
            for (int r = 0; r < G::P; ++r) my[G::pad(t + r * G::T)] = make_float2(nan_fix<POL>(a[r]), nan_fix<POL>(b[r]));
            xsync<64>();
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                const int j = t + r * G::T;
                v[r] = my[G::pad(j < N / 2 ? 2 * j : 2 * N - 2 * j - 1)];
            }
            xsync<64>();
        }
        fft_regs<N, true, true>(v, t, my, tw);
        // (the wave's LDS accesses run in program order: its FFT's last reads
        // precede these writes into the same area)
        xsync<64>();
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const float2 Z = v[q], Zm = mirror_of<N, true>(v, t, q);
            const float2 Va = make_float2(0.5f * (Z.x + Zm.x), 0.5f * (Z.y - Zm.y));
            const float2 Vb = make_float2(0.5f * (Z.y + Zm.y), -0.5f * (Z.x - Zm.x));
            const int k = out_pos<N, true>(t, q);
            const float2 W = lw4[k];
            wa[padf(2 * sl * N + k)] = nan_fix<POL>(W.x * Va.x - W.y * Va.y);
            wa[padf((2 * sl + 1) * N + k)] = nan_fix<POL>(W.x * Vb.x - W.y * Vb.y);
        }
        xsync<64>();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int e = i * 256 + 4 * lane;
            if (e < nval) {
                vf4_t w4;
#pragma unroll
                for (int k = 0; k < 4; ++k) w4[k] = wa[padf(e + k)];
                __builtin_nontemporal_store(w4, reinterpret_cast<vf4_t*>(X + r0 * N + e));
            }
        }
        xsync<64>();   // the next block's loads overwrite the area
    }
}

bool dct2_fused_supported(long long n) {
    // 256, 4096, 8192 (one last-pass butterfly per thread) read their mirror bins
    // through LDS; 4096 / 8192 run one transform per workgroup (T = 256 / 512)
    return n >= 2 && n <= 8192 && (n & (n - 1)) == 0;
}

hipError_t launch_dct2_fused(long long n, const float* x, float* X, long long batch, int policy, hipStream_t s) {
    if (batch <= 0) return hipSuccess;
    const float2* tw4n = twiddle_table((int)(4 * n));
    if (!tw4n) return hipErrorOutOfMemory;
    // 16..128 points: the staged kernel, one wave block per 2 x 64 / T rows (not
    // persistent); knob DCT_SMALL = 0 keeps k_dct2_pair (A/B)
    if (n >= 16 && n <= 128 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)X & 15) == 0 && knob(KNOB_DCT_SMALL, 1) == 1) {
#define VVH_DCTS(NN)                                                                                          \
        case NN: {                                                                                            \
            const float2* tab = twiddle_table(NN);                                                            \
            const float2* pas = pass_twiddles(NN);                                                            \
            if (!tab || !pas) return hipErrorOutOfMemory;                                                     \
            constexpr int F = 256 / Geo<NN>::T;                                                               \
            const long long need = ((batch + 1) / 2 + F - 1) / F;                                             \
            const int grid = (int)(need < (1LL << 30) ? need : (1LL << 30));                                  \
            if (policy == 1)                                                                                  \
                hipLaunchKernelGGL((k_dct2_small<NN, 1>), dim3(grid), dim3(256), 0, s, x, X, batch, pas, tab, tw4n); \
            else if (policy == 3)                                                                             \
                hipLaunchKernelGGL((k_dct2_small<NN, 3>), dim3(grid), dim3(256), 0, s, x, X, batch, pas, tab, tw4n); \
            else                                                                                              \
                hipLaunchKernelGGL((k_dct2_small<NN, 0>), dim3(grid), dim3(256), 0, s, x, X, batch, pas, tab, tw4n); \
            return hipGetLastError();                                                                         \
        }
        switch (n) {
            VVH_DCTS(16) VVH_DCTS(32) VVH_DCTS(64) VVH_DCTS(128)
            default: break;
        }
#undef VVH_DCTS
    }
#define VVH_DCT(NN)                                                                                          \
    case NN: {                                                                                               \
        const float2* tab = twiddle_table(NN);                                                               \
        const float2* pas = pass_twiddles(NN);                                                               \
        if (!tab || !pas) return hipErrorOutOfMemory;                                                        \
        constexpr int WG = Wg<NN>::value, F = Wg<NN>::F;                                                     \
        static std::atomic<int> capc;                                                                                  \
        const int cap0 = cached_grid(capc, (const void*)k_dct2_pair<NN, 0>, WG, 0, 1LL << 40);                 \
        /* knob ANA_TPW = 1: not persistent (A/B; DCT-II 2048 +22 %, r05_ab2_analytic_mixed_grid) */        \
        const long long cap = knob(KNOB_ANA_TPW, 0) == 1 ? (1LL << 30) : cap0;                               \
        const long long need = ((batch + 1) / 2 + F - 1) / F;                                                \
        const int grid = (int)(need < cap ? need : cap);                                                     \
        if (policy == 1)                                                                                     \
            hipLaunchKernelGGL((k_dct2_pair<NN, 1>), dim3(grid), dim3(WG), 0, s, x, X, batch, n, pas, tab, tw4n); \
        else if (policy == 3)                                                                                \
            hipLaunchKernelGGL((k_dct2_pair<NN, 3>), dim3(grid), dim3(WG), 0, s, x, X, batch, n, pas, tab, tw4n); \
        else                                                                                                 \
            hipLaunchKernelGGL((k_dct2_pair<NN, 0>), dim3(grid), dim3(WG), 0, s, x, X, batch, n, pas, tab, tw4n); \
        return hipGetLastError();                                                                            \
    }
    switch (n) {
        VVH_DCT(2) VVH_DCT(4) VVH_DCT(8) VVH_DCT(16) VVH_DCT(32) VVH_DCT(64) VVH_DCT(128) VVH_DCT(256) VVH_DCT(512)
        VVH_DCT(1024) VVH_DCT(2048) VVH_DCT(4096) VVH_DCT(8192)
        default: return hipErrorInvalidValue;
    }
#undef VVH_DCT
}

}  // namespace vvh
