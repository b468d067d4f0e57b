// fft_core.hpp -- register/LDS Stockham FFT building blocks for gfx950 (CDNA4).
//
// One power-of-two transform of length N (2..8192) is owned by T = N/P threads;
// every thread holds P points in VGPRs (P = 16 for N >= 16).  A transform runs
// as a chain of radix-16 passes (the last one radix 2/4/8 when log2 N is not a
// multiple of 4).  Each pass is a Stockham autosort step:
//
//   butterfly b = t + T*i (i < P/R), inputs  b + r*N/R            (r < R)
//   twiddle   W_{Ns*R}^{(b mod Ns)*r}                              (Ns = product of earlier radices)
//   outputs   (b div Ns)*Ns*R + (b mod Ns) + r*Ns
//
// so the FIRST pass reads x[t + r*T] (lane-contiguous -> coalesced global loads)
// and the LAST pass produces X[t + T*i + r*N/R] (lane-contiguous -> coalesced
// global stores).  Between passes the points are exchanged through LDS with one
// float2 of padding per 16 (conflict-free ds_write_b64/ds_read_b64 for the
// strides that occur).  The in-register radix-R DFTs use exact constant
// twiddles; the inter-pass twiddles come from a W_N^k table rounded from double
// on the host and staged in LDS (see TwDirect / TwSplit).
//
// Semantics match the reference (src/spectral/fft_kiss.c:27-74): forward is
// exp(-2*pi*i*k*n/N) unscaled; backward is exp(+...) and the caller applies 1/N.
#pragma once
#include <hip/hip_runtime.h>

namespace vvh {

__host__ __device__ constexpr int ilog2(int n) { return n <= 1 ? 0 : 1 + ilog2(n >> 1); }

// cos(2*pi*m/16), m = 0..15 (exact decimal expansions rounded to float by the compiler)
__device__ __forceinline__ constexpr float cos16(int m) {
    constexpr float c1 = 0.92387953251128675613f, c2 = 0.70710678118654752440f,
                    c3 = 0.38268343236508977173f;
    switch (m & 15) {
        case 0: return 1.0f;   case 1: return c1;     case 2: return c2;     case 3: return c3;
        case 4: return 0.0f;   case 5: return -c3;    case 6: return -c2;    case 7: return -c1;
        case 8: return -1.0f;  case 9: return -c1;    case 10: return -c2;   case 11: return -c3;
        case 12: return 0.0f;  case 13: return c3;    case 14: return c2;    default: return c1;
    }
}

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 w) {
    return make_float2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }

// Streaming (non-temporal) global accesses: data touched exactly once.
typedef float vf2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2 ld_nt(const float2* p) {
    const vf2_t v = __builtin_nontemporal_load(reinterpret_cast<const vf2_t*>(p));
    return make_float2(v.x, v.y);
}
__device__ __forceinline__ void st_nt(float2 a, float2* p) {
    vf2_t v;
    v.x = a.x;
    v.y = a.y;
    __builtin_nontemporal_store(v, reinterpret_cast<vf2_t*>(p));
}

// v * W_R^k with W_R = exp(-2*pi*i/R) (forward) or its conjugate (backward).
// k and R are compile-time after unrolling; trivial twiddles are exact swaps.
template <int R, bool FWD>
__device__ __forceinline__ float2 twc(float2 v, int k) {
    const int m = ((k * (16 / R)) & 15);   // angle in units of 2*pi/16
    if (m == 0) return v;
    if (m == 8) return make_float2(-v.x, -v.y);
    if (m == 4) return FWD ? make_float2(v.y, -v.x) : make_float2(-v.y, v.x);
    if (m == 12) return FWD ? make_float2(-v.y, v.x) : make_float2(v.y, -v.x);
    const float c = cos16(m);
    const float s = FWD ? -cos16(m + 12) : cos16(m + 12);   // sin(2*pi*m/16) = cos16(m-4)
    return make_float2(v.x * c - v.y * s, v.x * s + v.y * c);
}

// In-register DFT of length R (1,2,4,8,16), natural order in and out.
template <int R, bool FWD>
struct Dft {
    __device__ __forceinline__ static void run(float2* v) {
        float2 e[R / 2], o[R / 2];
#pragma unroll
        for (int i = 0; i < R / 2; ++i) { e[i] = v[2 * i]; o[i] = v[2 * i + 1]; }
        Dft<R / 2, FWD>::run(e);
        Dft<R / 2, FWD>::run(o);
#pragma unroll
        for (int k = 0; k < R / 2; ++k) {
            const float2 t = twc<R, FWD>(o[k], k);
            v[k] = cadd(e[k], t);
            v[k + R / 2] = csub(e[k], t);
        }
    }
};
template <bool FWD>
struct Dft<1, FWD> {
    __device__ __forceinline__ static void run(float2*) {}
};
template <bool FWD>
struct Dft<2, FWD> {
    __device__ __forceinline__ static void run(float2* v) {
        const float2 a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    }
};
template <bool FWD>
struct Dft<4, FWD> {
    __device__ __forceinline__ static void run(float2* v) {
        const float2 s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
        const float2 s13 = cadd(v[1], v[3]), d13 = csub(v[1], v[3]);
        // d13 * W_4^1: forward -i, backward +i
        const float2 r = FWD ? make_float2(d13.y, -d13.x) : make_float2(-d13.y, d13.x);
        v[0] = cadd(s02, s13);
        v[2] = csub(s02, s13);
        v[1] = cadd(d02, r);
        v[3] = csub(d02, r);
    }
};

// Compile-time geometry of a length-N transform.
template <int N>
struct Geo {
    static_assert(N >= 2 && (N & (N - 1)) == 0, "power of two");
    static constexpr int LOG = ilog2(N);
    static constexpr int P = N >= 16 ? 16 : N;          // points per thread
    static constexpr int T = N / P;                     // threads per transform
    static constexpr int NPASS = N >= 16 ? (LOG + 3) / 4 : 1;
    static constexpr int LDS = N + (N >> 4);            // padded LDS floats2 per transform
    __host__ __device__ static constexpr int radix(int p) {
        return N < 16 ? N : ((LOG - 4 * p) >= 4 ? 16 : (1 << (LOG - 4 * p)));
    }
    __host__ __device__ static constexpr int ns(int p) {
        int s = 1;
        for (int q = 0; q < p; ++q) s *= radix(q);
        return s;
    }
    __host__ __device__ static constexpr int pad(int e) { return e + (e >> 4); }
};

// Barrier between LDS writes and reads of one transform.  A transform owned by
// threads of a single wave needs no s_barrier: LDS ops of a wave execute in
// order; only the compiler must not move them (wave_barrier + fence).
template <int T>
__device__ __forceinline__ void xsync() {
    if constexpr (T > 64) {
        __syncthreads();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// ---- inter-pass twiddle sources -------------------------------------------
// Streaming kernels keep every table in LDS so that VMEM carries only the
// streamed data (loads of the NEXT transform are prefetched; a table load at
// use would sit behind them in the in-order vmcnt queue).  Tables are staged
// from the host-computed W_N^k (f32 rounded from double) at kernel start.
//   TwDirect : W_N^k = tab[k]                          (N <= 2048: <= 16 KB)
//   TwSplit  : W_N^k = lo[k & 63] * hi[k >> 6]          (N  > 2048: 64 + N/64 entries)
struct TwDirect {
    const float2* tab;
    __device__ __forceinline__ float2 operator()(int k) const { return tab[k]; }
};
struct TwSplit {
    const float2* lo;   // W_N^j, j < 64
    const float2* hi;   // W_N^(64 i), i < N/64
    __device__ __forceinline__ float2 operator()(int k) const { return cmul(lo[k & 63], hi[k >> 6]); }
};

// LDS footprint (float2 entries) of the twiddle source for a length-N transform.
template <int N>
struct TwLayout {
    static constexpr bool SPLIT = N > 2048;
    static constexpr int ENTRIES = SPLIT ? 64 + N / 64 : N;
};

// Cooperative copy of the W_N table into LDS (all threads of the block), then
// returns the accessor.  `gtab` is the global W_N^k table (N entries).
template <int N, int NTHREADS>
__device__ __forceinline__ void stage_twiddles(float2* lds_tab, const float2* gtab) {
    if constexpr (TwLayout<N>::SPLIT) {
        for (int i = threadIdx.x; i < 64; i += NTHREADS) lds_tab[i] = gtab[i];
        for (int i = threadIdx.x; i < N / 64; i += NTHREADS) lds_tab[64 + i] = gtab[64 * i];
    } else {
        for (int i = threadIdx.x; i < N; i += NTHREADS) lds_tab[i] = gtab[i];
    }
}

template <int N>
__device__ __forceinline__ auto twiddles_from(const float2* lds_tab) {
    if constexpr (TwLayout<N>::SPLIT) return TwSplit{lds_tab, lds_tab + 64};
    else return TwDirect{lds_tab};
}

// One Stockham pass p on the registers (twiddle + radix-R DFT), in place.
// Twiddle W_{Ns*R}^{j*r} = W_N^{j*r*N/(Ns*R)}; a backward pass conjugates.
template <int N, bool FWD, int p, class TW>
__device__ __forceinline__ void pass_compute(float2* v, int t, const TW& tw) {
    using G = Geo<N>;
    constexpr int R = G::radix(p);
    constexpr int Ns = G::ns(p);
#pragma unroll
    for (int i = 0; i < G::P / R; ++i) {
        if constexpr (p > 0) {
            const int j = (t + G::T * i) % Ns;
#pragma unroll
            for (int r = 1; r < R; ++r) {
                const float2 w = tw(j * r * (N / (Ns * R)));
                v[i * R + r] = cmul(v[i * R + r], FWD ? w : cconj(w));
            }
        }
        Dft<R, FWD>::run(v + i * R);
    }
}

// Exchange after pass p: scatter outputs of pass p, gather inputs of pass p+1.
template <int N, int p>
__device__ __forceinline__ void pass_exchange(float2* v, int t, float2* lds) {
    using G = Geo<N>;
    constexpr int R = G::radix(p), Ns = G::ns(p), R2 = G::radix(p + 1);
#pragma unroll
    for (int i = 0; i < G::P / R; ++i) {
        const int b = t + G::T * i;
        const int base = (b / Ns) * Ns * R + (b % Ns);
#pragma unroll
        for (int r = 0; r < R; ++r) lds[G::pad(base + r * Ns)] = v[i * R + r];
    }
    xsync<G::T>();
#pragma unroll
    for (int i = 0; i < G::P / R2; ++i) {
        const int b = t + G::T * i;
#pragma unroll
        for (int r = 0; r < R2; ++r) v[i * R2 + r] = lds[G::pad(b + r * (N / R2))];
    }
    if constexpr (G::T > 64) __syncthreads();   // next pass' writes must not race these reads
}

template <int N, bool FWD, int p, class TW>
struct PassChain {
    __device__ __forceinline__ static void run(float2* v, int t, float2* lds, const TW& tw) {
        pass_compute<N, FWD, p>(v, t, tw);
        if constexpr (p + 1 < Geo<N>::NPASS) {
            pass_exchange<N, p>(v, t, lds);
            PassChain<N, FWD, p + 1, TW>::run(v, t, lds, tw);
        }
    }
};

// Full transform.  On entry v[r] = x[t + r*T] (r < P).  On exit, with R the
// last radix, v[i*R + r] = X[t + T*i + r*(N/R)].
template <int N, bool FWD, class TW>
__device__ __forceinline__ void fft_regs(float2* v, int t, float2* lds, const TW& tw) {
    PassChain<N, FWD, 0, TW>::run(v, t, lds, tw);
}

// Output position of register q after fft_regs (last-pass layout).
template <int N>
__device__ __forceinline__ constexpr int out_pos(int t, int q) {
    using G = Geo<N>;
    constexpr int R = G::radix(G::NPASS - 1);
    return t + G::T * (q / R) + (q % R) * (N / R);
}

// ---- shared pieces of the persistent streaming kernels ---------------------
// Workgroup geometry: 256 threads (several transforms per block) unless one
// transform needs more threads.
template <int N>
struct Wg {
    static constexpr int value = Geo<N>::T > 256 ? Geo<N>::T : 256;
    static constexpr int F = value / Geo<N>::T;   // transforms per workgroup
};

// Real-FFT split step: X[k] from A = Z[k], B = conj(Z[M-k]): Fe + W_{2M}^k (-i Fo)
__device__ __forceinline__ float2 split_fwd(float2 A, float2 B, float2 W) {
    const float2 fe = cscale(cadd(A, B), 0.5f);
    const float2 fo = cscale(csub(A, B), 0.5f);
    return cadd(fe, cmul(make_float2(fo.y, -fo.x), W));
}

// Inverse split step: Zi[k] = E + iO, E = (A + conj(B))/2, O = (A - conj(B)) conj(W_{2M}^k)/2
// with A = X[k], B = X[M-k].
__device__ __forceinline__ float2 split_inv(float2 A, float2 B, float2 W) {
    const float2 Bc = cconj(B);
    const float2 E = cscale(cadd(A, Bc), 0.5f);
    const float2 O = cmul(cscale(csub(A, Bc), 0.5f), cconj(W));
    return make_float2(E.x - O.y, E.y + O.x);
}

// W_{2M}^k for k < M (split-step twiddles), staged in LDS like TwLayout.
template <int M>
struct PostLayout {
    static constexpr bool SPLIT = 2 * M > 2048;
    static constexpr int ENTRIES = SPLIT ? 64 + M / 64 : M;
};

template <int M, int NTHREADS>
__device__ __forceinline__ void stage_post(float2* lds_tab, const float2* g2M) {
    if constexpr (PostLayout<M>::SPLIT) {
        for (int i = threadIdx.x; i < 64; i += NTHREADS) lds_tab[i] = g2M[i];
        for (int i = threadIdx.x; i < M / 64; i += NTHREADS) lds_tab[64 + i] = g2M[64 * i];
    } else {
        for (int i = threadIdx.x; i < M; i += NTHREADS) lds_tab[i] = g2M[i];
    }
}

template <int M>
__device__ __forceinline__ auto post_from(const float2* lds_tab) {
    if constexpr (PostLayout<M>::SPLIT) return TwSplit{lds_tab, lds_tab + 64};
    else return TwDirect{lds_tab};
}

}  // namespace vvh
