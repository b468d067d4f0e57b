// fft_core.hpp -- register/LDS Stockham FFT building blocks for gfx950 (CDNA4).
//
// One power-of-two transform of length N (2..8192) is owned by T = N/P threads;
// every thread holds P points in VGPRs (P = 16 for N >= 16).  A transform runs
// as a chain of radix-16 passes (the last one radix 2/4/8 when log2 N is not a
// multiple of 4).  Each pass is a Stockham autosort step:
//
//   butterfly b (thread t owns P/R of them), inputs  b + r*N/R        (r < R)
//   twiddle   W_{Ns*R}^{(b mod Ns)*r}                 (Ns = product of earlier radices)
//   outputs   (b div Ns)*Ns*R + (b mod Ns) + r*Ns
//
// With the standard ownership b = t + T*i the FIRST pass reads x[t + r*T]
// (lane-contiguous, coalesced loads) and the LAST pass produces
// X[t + T*i + r*N/R] (lane-contiguous stores).  Between passes the points go
// through LDS with one float2 of padding per 16 (conflict-free b64 accesses).
//
// "Mirror-paired" last pass (PAIRED = true): the thread owns butterfly pairs
// {b, NB - b} of the last pass (NB = N/R butterflies), so it ends holding both
// X[k] and X[N-k] in registers.  Every real-signal split step (R2C, STFT of two
// frames packed in one complex FFT, FIR spectrum multiply) then needs no LDS
// round trip.  Available when the last pass leaves >= 2 butterflies per thread.
//
// Twiddles: in-register radix-R DFTs use exact constants; inter-pass twiddles
// come from tables rounded from double on the host and staged in LDS.  For
// N <= 2048 the table is pass-major (entry (r-1)*Ns + j of pass p holds
// W_{Ns R}^{j r}) so that lanes with consecutive j read consecutive LDS words
// (no bank conflicts); larger N use a two-level table W_N^k = lo[k%64]*hi[k/64].
//
// Semantics match the reference (src/spectral/fft_kiss.c:27-74): forward is
// exp(-2*pi*i*k*n/N) unscaled; backward is exp(+...) and the caller applies 1/N.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

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

// Complex arithmetic as packed-f32 vector ops (v_pk_add/mul/fma_f32 with
// op_sel swizzles and neg modifiers): one instruction per complex add and two
// per complex multiply, instead of letting the SLP vectorizer pair unrelated
// scalars (which costs a v_mov per operand).
typedef float vf2_t __attribute__((ext_vector_type(2)));
typedef float vf4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ vf2_t pk(float2 a) { return vf2_t{a.x, a.y}; }
__device__ __forceinline__ float2 upk(vf2_t v) { return make_float2(v.x, v.y); }
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return upk(pk(a) + pk(b)); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return upk(pk(a) - pk(b)); }
// a*w = a.xx * w + a.yy * (-w.y, w.x): t = a.yy * (-w.y, w.x) as one v_pk_mul_f32
// with op_sel swizzles and a neg modifier, then one v_pk_fma_f32 -- two
// instructions (left to itself the compiler spends a third, multiplying w by
// (-1, 1) first).  Same roundings: (fma(a.x, w.x, -a.y w.y), fma(a.x, w.y, a.y w.x)).
__device__ __forceinline__ float2 cmul(float2 a, float2 w) {
    const vf2_t A = pk(a), W = pk(w);
    vf2_t t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(t) : "v"(A), "v"(W));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r) : "v"(A), "v"(W), "v"(t));
    return upk(r);
}
// e + i*o (PLUS_I) or e - i*o as one v_pk_add_f32 with swizzle and negation
// modifiers: the quarter-turn rotations of the radix-4/8/16 butterflies cost no
// multiply (exact, as the multiply by +-1 it replaces)
template <bool PLUS_I>
__device__ __forceinline__ float2 cadd_i(float2 e, float2 o) {
    vf2_t r;
    if constexpr (PLUS_I)   // (e.x - o.y, e.y + o.x)
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(pk(e)), "v"(pk(o)));
    else                    // (e.x + o.y, e.y - o.x)
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(pk(e)), "v"(pk(o)));
    return upk(r);
}
__device__ __forceinline__ float2 cconj(float2 a) { return upk(pk(a) * vf2_t{1.0f, -1.0f}); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return upk(pk(a) * s); }
// -i*a (forward quarter turn) and +i*a
__device__ __forceinline__ float2 cmul_mi(float2 a) { return upk(pk(a).yx * vf2_t{1.0f, -1.0f}); }
__device__ __forceinline__ float2 cmul_pi(float2 a) { return upk(pk(a).yx * vf2_t{-1.0f, 1.0f}); }

// x * (w.lo, w.lo) (HI = 0) or x * (w.hi, w.hi) (HI = 1) as one v_pk_mul_f32
// with op_sel: a packed pair of per-register constants (two window values)
// then costs one VGPR each.  Written out because the SLP vectorizer otherwise
// materialises (w, w) duplicates -- 16 extra VGPRs for a 16-point window.
template <int HI>
__device__ __forceinline__ vf2_t pk_mul_bcast(vf2_t x, vf2_t w) {
    vf2_t r;
    if constexpr (HI) asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(x), "v"(w));
    else asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(x), "v"(w));
    return r;
}

// Streaming (non-temporal) global accesses: data touched exactly once.
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
    if (m == 8) return upk(-pk(v));
    if (m == 4) return FWD ? cmul_mi(v) : cmul_pi(v);
    if (m == 12) return FWD ? cmul_pi(v) : cmul_mi(v);
    const float c = cos16(m);
    const float s = FWD ? -cos16(m + 12) : cos16(m + 12);   // sin(2*pi*m/16) = cos16(m-4)
    const vf2_t V = pk(v);
    return upk(V.xx * vf2_t{c, s} + V.yy * vf2_t{-s, c});
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
            const int m = (k * (16 / R)) & 15;
            if (m == 4 || m == 12) {   // o * (-+i): folded into the adds
                const bool plus_i = (m == 12) == FWD;
                v[k] = plus_i ? cadd_i<true>(e[k], o[k]) : cadd_i<false>(e[k], o[k]);
                v[k + R / 2] = plus_i ? cadd_i<false>(e[k], o[k]) : cadd_i<true>(e[k], o[k]);
            } else {
                const float2 t = twc<R, FWD>(o[k], k);
                v[k] = cadd(e[k], t);
                v[k + R / 2] = csub(e[k], t);
            }
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
        // d13 * W_4^1: forward -i, backward +i (folded into the adds)
        v[0] = cadd(s02, s13);
        v[2] = csub(s02, s13);
        v[1] = FWD ? cadd_i<false>(d02, d13) : cadd_i<true>(d02, d13);
        v[3] = FWD ? cadd_i<true>(d02, d13) : cadd_i<false>(d02, d13);
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
    static constexpr int LDS = N + (N >> 4);            // padded LDS float2 per transform
    __host__ __device__ static constexpr int radix(int p) {
        return N < 16 ? N : ((LOG - 4 * p) >= 4 ? 16 : (1 << (LOG - 4 * p)));
    }
    __host__ __device__ static constexpr int ns(int p) {
        int s = 1;
        for (int q = 0; q < p; ++q) s *= radix(q);
        return s;
    }
    __host__ __device__ static constexpr int pad(int e) { return e + (e >> 4); }
    static constexpr int RL = radix(NPASS - 1);         // last radix
    static constexpr int NB = N / RL;                   // butterflies in the last pass
    static constexpr int NPT = P / RL;                  // last-pass butterflies per thread
    // mirror pairing possible: single-thread transforms, or >= 2 last-pass butterflies per thread
    static constexpr bool CAN_PAIR = (T == 1) || (NPT >= 2);
    // pass-major twiddle table: offset of pass p, total entries
    __host__ __device__ static constexpr int tw_off(int p) {
        int o = 0;
        for (int q = 1; q < p; ++q) o += (radix(q) - 1) * ns(q);
        return o;
    }
    static constexpr int TW_PASS_ENTRIES = tw_off(NPASS) > 0 ? tw_off(NPASS) : 1;
};

// Butterfly owned by thread t in slot i of pass p.
template <int N, int p, bool PAIRED>
__device__ __forceinline__ int bfly(int t, int i) {
    using G = Geo<N>;
    if constexpr (PAIRED && G::T > 1 && p == G::NPASS - 1) {
        const int b0 = t + G::T * (i >> 1);
        if ((i & 1) == 0) return b0;
        return b0 == 0 ? G::NB / 2 : G::NB - b0;
    } else {
        return t + G::T * i;
    }
}

// Output position of register q after fft_regs (last-pass layout).
template <int N, bool PAIRED = false>
__device__ __forceinline__ int out_pos(int t, int q) {
    using G = Geo<N>;
    constexpr int R = G::RL;
    return bfly<N, G::NPASS - 1, PAIRED>(t, q / R) + (q % R) * (N / R);
}

// In a PAIRED layout: register holding X[N - out_pos(t, q)].  Two candidates
// (compile-time indices) selected by whether this is thread 0's self-mirrored
// slots 0/1; callers pick with `t == 0 && q < 2R ? special : normal`.
template <int N>
struct Mirror {
    using G = Geo<N>;
    static constexpr int R = G::RL;
    __host__ __device__ static constexpr int normal(int q) {
        if (G::T == 1) return (N - q) % N;
        const int i = q / R, r = q % R;
        return (i ^ 1) * R + (R - 1 - r);
    }
    __host__ __device__ static constexpr int special(int q) {   // thread 0, slots 0 and 1
        if (G::T == 1) return (N - q) % N;
        const int i = q / R, r = q % R;
        return i == 0 ? (R - r) % R : R + (R - 1 - r);
    }
};

// Bitwise select between two register values.  A plain `c ? v[i] : v[j]` is
// folded by LLVM into `v[c ? i : j]` -- a dynamic index that sends the whole
// register array to scratch; masking the bits keeps both indices static.
__device__ __forceinline__ float2 select2(bool c, float2 a, float2 b) {
    const unsigned m = c ? 0xffffffffu : 0u;
    return make_float2(__uint_as_float((__float_as_uint(a.x) & m) | (__float_as_uint(b.x) & ~m)),
                       __uint_as_float((__float_as_uint(a.y) & m) | (__float_as_uint(b.y) & ~m)));
}

template <int N, bool PAIRED>
__device__ __forceinline__ float2 mirror_of(const float2* v, int t, int q) {
    using M = Mirror<N>;
    if constexpr (Geo<N>::T == 1) {
        return v[M::normal(q)];
    } else {
        if (q < 2 * M::R) return select2(t == 0, v[M::special(q)], v[M::normal(q)]);
        return v[M::normal(q)];
    }
}

// ---- inter-pass twiddle sources --------------------------------------------
// Streaming kernels keep every table in LDS so that VMEM carries only the
// streamed data (loads of the NEXT transform are prefetched; a table load at
// use would sit behind them in the in-order vmcnt queue).
template <int N>
struct TwLayout {
    static constexpr bool SPLIT = N > 2048;
    static constexpr int ENTRIES = SPLIT ? 64 + N / 64 : Geo<N>::TW_PASS_ENTRIES;
};

template <int N>
struct TwTab {
    const float2* tab;   // LDS: pass-major table, or lo[64] ++ hi[N/64] when SPLIT
    template <int p>
    __device__ __forceinline__ float2 at(int j, int r, int /*i*/ = 0) const {
        using G = Geo<N>;
        if constexpr (TwLayout<N>::SPLIT) {
            const int k = j * r * (N / (G::ns(p) * G::radix(p)));
            return cmul(tab[k & 63], tab[64 + (k >> 6)]);
        } else {
            return tab[G::tw_off(p) + (r - 1) * G::ns(p) + j];
        }
    }
};

// Timing probe only (wrong twiddles): TwTab's LDS reads from a 128-entry table.
template <int N>
struct TwMask {
    const float2* tab;
    template <int p>
    __device__ __forceinline__ float2 at(int j, int r, int /*i*/ = 0) const {
        using G = Geo<N>;
        return tab[(G::tw_off(p) + (r - 1) * G::ns(p) + j) & 127];
    }
};

// Twiddle source for one-wave transforms (T = N/16) that streams many
// transforms through one kernel: the passes before the last read the LDS
// pass-major table (only tw_off(LAST) entries are staged); the last pass'
// twiddles are derived in registers -- a thread's last-pass butterflies are the
// same for every transform (j = t + T*i), W_N^{j r} = W_N^{t r} * W_16^{i r},
// and W_16^{i r} is an exact in-register rotation.  Saves the largest part of
// the table in LDS (6 KB of 8 KB for N = 1024).
template <int N>
struct TwLastReg {
    using G = Geo<N>;
    static constexpr int LAST = G::NPASS - 1, RL = G::RL, NS = G::ns(LAST);
    static_assert(G::T * (G::P / RL) == NS && G::T == N / 16, "j = t + T*i < NS, and W_N^T = W_16");
    const float2* tab;   // LDS: pass-major entries of passes < LAST
    float2 w[RL - 1];    // W_N^{r t}, r = 1..RL-1
    // last pass: j = t + T*i (< NS), twiddle W_N^{j r} = W_N^{t r} * W_N^{T i r}; with
    // T = N/16 the second factor is W_16^{i r}, an exact in-register rotation
    template <int p>
    __device__ __forceinline__ float2 at(int j, int r, int i) const {
        if constexpr (p == LAST) return twc<16, true>(w[r - 1], i * r);
        else return tab[G::tw_off(p) + (r - 1) * G::ns(p) + j];
    }
    __device__ __forceinline__ void load(const float2* gpass, int t) {
#pragma unroll
        for (int r = 1; r < RL; ++r) w[r - 1] = gpass[G::tw_off(LAST) + (r - 1) * NS + t];
        // consume the loads here, so that the compiler's vmcnt wait for them
        // sits before the streaming loop (it does not count the loop's asm ops)
        opaque();
    }
    // Called before each transform: the derived twiddles then cannot be hoisted
    // out of the pair loop (LICM would keep all (RL-1)*P/RL of them, and their
    // conjugates, live across it -- 48 VGPRs and scratch spills).
    __device__ __forceinline__ void opaque() {
#pragma unroll
        for (int r = 0; r < RL - 1; ++r) asm volatile("" : "+v"(w[r].x), "+v"(w[r].y));
    }
};

// The same for a MIRROR-PAIRED last pass with two butterflies per thread
// (NPT = 2, e.g. N = 2048: T = 128, last radix 8): a thread's last-pass
// butterflies are j0 = t (< NS/2) and j1 = NS - t (NS / 2 for t = 0, so in
// [NS/2, NS)), the same for every transform.  Butterfly j0's RL - 1 twiddles
// are loaded once into registers; butterfly j1's are read per transform from
// the upper half of the last pass' table staged in LDS (`hi`: [r-1][j - NS/2]).
// Either way the table's own values -- bit-identical to TwTab -- with half the
// last pass' entries in LDS and RL - 1 twiddles in VGPRs.
template <int N>
struct TwLastRegP {
    using G = Geo<N>;
    static constexpr int LAST = G::NPASS - 1, RL = G::RL, NS = G::ns(LAST);
    static constexpr int HI_ENTRIES = (RL - 1) * (NS / 2);
    static_assert(G::NPT == 2 && G::NB == NS && G::T == NS / 2, "two mirror-paired last-pass butterflies per thread");
    const float2* tab;   // LDS: pass-major entries of passes < LAST
    const float2* hi;    // LDS: [r-1][j - NS/2], the last pass for j in [NS/2, NS)
    float2 w[RL - 1];    // W^{t r} of the last pass, r = 1..RL-1
    template <int p>
    __device__ __forceinline__ float2 at(int j, int r, int i) const {
        if constexpr (p == LAST) return (i & 1) ? hi[(r - 1) * (NS / 2) + (j - NS / 2)] : w[r - 1];
        else return tab[G::tw_off(p) + (r - 1) * G::ns(p) + j];
    }
    __device__ __forceinline__ void load(const float2* gpass, int t) {
#pragma unroll
        for (int r = 1; r < RL; ++r) w[r - 1] = gpass[G::tw_off(LAST) + (r - 1) * NS + t];
        opaque();
    }
    // stage the table entries of the passes < LAST and the last pass' upper half
    template <int NTHREADS>
    __device__ __forceinline__ static void stage(float2* lds_tab, float2* lds_hi, const float2* gpass) {
        for (int i = threadIdx.x; i < G::tw_off(LAST); i += NTHREADS) lds_tab[i] = gpass[i];
        for (int i = threadIdx.x; i < HI_ENTRIES; i += NTHREADS)
            lds_hi[i] = gpass[G::tw_off(LAST) + (i / (NS / 2)) * NS + NS / 2 + i % (NS / 2)];
    }
    __device__ __forceinline__ void opaque() {
#pragma unroll
        for (int r = 0; r < RL - 1; ++r) asm volatile("" : "+v"(w[r].x), "+v"(w[r].y));
    }
};

// The same for every last-pass butterfly of a thread held in registers (any
// NPT, e.g. N = 1024 mirror-paired: T = 64, last radix 4, four butterflies
// t, NB - t, t + 64, NB - 64 - t): NPT (RL - 1) twiddles in VGPRs (24 at 1024),
// loaded once per workgroup from the global pass-major table -- the table's own
// values, so bit-identical to TwTab -- and only the passes before the last in
// LDS (240 of 1008 entries at 1024: 6 KB of LDS and 12 LDS reads per
// transform saved).
template <int N, bool PAIRED>
struct TwLastRegA {
    using G = Geo<N>;
    static constexpr int LAST = G::NPASS - 1, RL = G::RL, NS = G::ns(LAST), NPT = G::NPT;
    static_assert(G::NB == NS, "the last pass' butterfly index is its twiddle index");
    const float2* tab;            // LDS: pass-major entries of passes < LAST
    float2 w[NPT * (RL - 1)];     // [i][r - 1]: W^{j_i r} of the thread's last-pass butterfly i
    template <int p>
    __device__ __forceinline__ float2 at(int j, int r, int i) const {
        if constexpr (p == LAST) return w[i * (RL - 1) + r - 1];
        else return tab[G::tw_off(p) + (r - 1) * G::ns(p) + j];
    }
    __device__ __forceinline__ void load(const float2* gpass, int t) {
#pragma unroll
        for (int i = 0; i < NPT; ++i) {
            const int j = bfly<N, LAST, PAIRED>(t, i);
#pragma unroll
            for (int r = 1; r < RL; ++r) w[i * (RL - 1) + r - 1] = gpass[G::tw_off(LAST) + (r - 1) * NS + j];
        }
        opaque();
    }
    template <int NTHREADS>
    __device__ __forceinline__ static void stage(float2* lds_tab, const float2* gpass) {
        for (int i = threadIdx.x; i < G::tw_off(LAST); i += NTHREADS) lds_tab[i] = gpass[i];
    }
    __device__ __forceinline__ void opaque() {
#pragma unroll
        for (int r = 0; r < NPT * (RL - 1); ++r) asm volatile("" : "+v"(w[r].x), "+v"(w[r].y));
    }
};

// Stage the global table into LDS (all NTHREADS threads of the block).
//   gpass : pass-major table for N (host: pass_twiddles(N)), used when !SPLIT
//   gtab  : W_N^k, k < N (host: twiddle_table(N)), used when SPLIT
template <int N, int NTHREADS>
__device__ __forceinline__ void stage_twiddles(float2* lds_tab, const float2* gpass, const float2* gtab) {
    if constexpr (TwLayout<N>::SPLIT) {
        for (int i = threadIdx.x; i < 64; i += NTHREADS) lds_tab[i] = gtab[i];
        for (int i = threadIdx.x; i < N / 64; i += NTHREADS) lds_tab[64 + i] = gtab[64 * i];
    } else {
        for (int i = threadIdx.x; i < TwLayout<N>::ENTRIES; i += NTHREADS) lds_tab[i] = gpass[i];
    }
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// Barrier between LDS writes and reads of one transform.  A transform owned by
// threads of a single wave needs no s_barrier: LDS ops of a wave execute in
// order; only the compiler must not move them (wave_barrier + fence).
// No memory fences: a fence makes hipcc drain vmcnt (outstanding global loads
// AND stores) at every exchange, which serialises the streaming pipeline.  LDS
// ordering needs only lgkmcnt + s_barrier across waves, and nothing but a
// compiler barrier within one wave.
template <int T>
__device__ __forceinline__ void xsync() {
    if constexpr (T > 64) {
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
    }
}

// One Stockham pass p on the registers (twiddle + radix-R DFT), in place.
// TW: twiddle source with `at<p>(j, r, i)` (j = butterfly index mod Ns, i = the
// thread's butterfly slot) -- TwTab<N>, or one holding some passes in registers.
template <int N, bool FWD, int p, bool PAIRED, class TW>
__device__ __forceinline__ void pass_compute(float2* v, int t, const TW& tw) {
    using G = Geo<N>;
    constexpr int R = G::radix(p);
    constexpr int Ns = G::ns(p);
#pragma unroll
    for (int i = 0; i < G::P / R; ++i) {
        if constexpr (p > 0) {
            const int j = bfly<N, p, PAIRED>(t, i) % Ns;
#pragma unroll
            for (int r = 1; r < R; ++r) {
                const float2 w = tw.template at<p>(j, r, i);
                v[i * R + r] = cmul(v[i * R + r], FWD ? w : cconj(w));
            }
        }
        Dft<R, FWD>::run(v + i * R);
    }
}

// Exchange after pass p: scatter outputs of pass p, gather inputs of pass p+1.
// Padding of the complex (b64) exchange after pass p: Geo<N>::pad, except the
// second exchange of N = 4096 (passes 16, 16, 16), where e + (e >> 9) makes the
// reads conflict-free (Geo::pad: 128 extra LDS cycles per wave and transform;
// host model in tests/test_lds_banks.py); inside Geo<4096>::LDS float2.
template <int N, int p>
__host__ __device__ constexpr int cx_pad(int e) {
    if constexpr (N == 4096 && p == 1) return e + (e >> 9);
    else return Geo<N>::pad(e);
}
__host__ __device__ constexpr bool cx_pad_check() {
    for (int e = 1; e < 4096; ++e)
        if (cx_pad<4096, 1>(e) <= cx_pad<4096, 1>(e - 1)) return false;
    return cx_pad<4096, 1>(4095) < Geo<4096>::LDS;
}
static_assert(cx_pad_check(), "cx_pad<4096, 1>");
template <int N, int p, bool PAIRED>
__device__ __forceinline__ void pass_exchange(float2* v, int t, float2* lds) {
    using G = Geo<N>;
    constexpr int R = G::radix(p), Ns = G::ns(p), R2 = G::radix(p + 1);
#pragma unroll
    for (int i = 0; i < G::P / R; ++i) {
        const int b = bfly<N, p, PAIRED>(t, i);
        const int base = (b / Ns) * Ns * R + (b % Ns);
#pragma unroll
        for (int r = 0; r < R; ++r) lds[cx_pad<N, p>(base + r * Ns)] = v[i * R + r];
    }
    xsync<G::T>();
#pragma unroll
    for (int i = 0; i < G::P / R2; ++i) {
        const int b = bfly<N, p + 1, PAIRED>(t, i);
#pragma unroll
        for (int r = 0; r < R2; ++r) v[i * R2 + r] = lds[cx_pad<N, p>(b + r * (N / R2))];
    }
    if constexpr (G::T > 64) xsync<G::T>();   // next pass' writes must not race these reads
}

// The same exchange through a buffer of half the size (Geo<N>::LDS floats):
// real parts first, then imaginary parts.  Twice the LDS instructions (b32
// instead of b64), half the LDS footprint -- for kernels whose occupancy is
// bounded by LDS.
// Per-exchange padding of the dword layout: for N = 1024 (passes 16, 16, 4)
// these make both exchanges bank-conflict-free and keep all compile-time
// offsets additive.  After pass 0 a thread's 16 outputs are contiguous, so
// they go out as four ds_write_b128 (8-lane groups, 32 banks: the pad
// 4 (e >> 5) puts the 8 lanes' 16 B chunks on distinct banks) and are read
// back as b32 (32-lane groups, conflict-free for the same pad).  Largest index
// 1147: the buffer is ri_floats<N>() floats, 16 B aligned.
// floats of one transform's pass_exchange_ri buffer
template <int N>
__host__ __device__ constexpr int ri_floats() {
    return N == 1024 ? 1148 : Geo<N>::LDS;
}
// VVH_RI_B128 (default): pass-0 writes as four ds_write_b128 per half (pad 4
// per 32 floats).  VVH_RI_B128=0: ds_write2_b32 pairs straight from the complex
// registers (pad 1 per 32 floats: lane b's 16 floats start at 16b + (b >> 1), on
// 32 distinct banks), which saves the 16 v_mov per half that gather four real
// (or imaginary) parts into a 16 B register quad -- but measured no faster
// (c2c 1024 +3.9 %, FIR +1.4 %, STFT even; profiles/r02_ab_ri_write2.jsonl):
// the LDS instruction count, not VALU, is what these kernels wait on.
#ifndef VVH_RI_B128
#define VVH_RI_B128 1
#endif
// N = 2048 (passes 16, 16, 8; T = 128, mirror-paired last pass): e + (e >> 4)
// left a 2-way conflict in every 32-lane group of each exchange read (lane 31's
// b + (b >> 4) wraps onto lane 0's bank: 256 extra LDS cycles per frame pair,
// half the kernel's LDS-array time, SQ_LDS_BANK_CONFLICT in
// profiles/r06_pmc_stft256_2048_pow.txt); these per-pass pads are conflict-free
// for both the writes and the reads (a host model of every access,
// tests/test_lds_banks.py) and stay inside Geo<2048>::LDS floats.
template <int N, int p>
__host__ __device__ constexpr int ri_pad(int e) {
    if constexpr (N == 1024 && p == 0) return VVH_RI_B128 ? e + 4 * (e >> 5) : e + (e >> 5);
    else if constexpr (N == 1024 && p == 1) return e + 4 * (e >> 7) + 8 * (e >> 8);
    else if constexpr (N == 2048 && p == 0) return e + (e >> 5);
    else if constexpr (N == 2048 && p == 1) return e + 16 * (e >> 8);
    else return Geo<N>::pad(e);
}

// N = 1024 (passes 16, 16, 4): ri_pad<1024, p> of every exchange access as a
// lane base plus a compile-time offset, so each access is one ds_write/ds_read
// with an immediate offset off a few base registers.  (Left to itself the
// compiler keeps one padded address per access live across the loop: 16+
// VGPRs.)  Derivations (b: the butterfly, r: its register):
//   p 0 writes  16b + r             -> (16b + 4(b>>1)) + r   (16 B aligned base)
//   p 0 reads   b + 64r   (b < 64)  -> (b + 4(b>>5)) + 72r
//   p 1 writes  256(b>>4) + (b&15) + 16r -> (272(b>>4) + (b&15)) + 16r + 4[r>=8]
//   p 1 reads   b + 256r  (b < 256) -> (b + 4(b>>7)) + 272r
struct Ri1024 {
    template <int p>
    __host__ __device__ static constexpr int wbase(int b) {
        return p == 0 ? (VVH_RI_B128 ? 16 * b + 4 * (b >> 1) : 16 * b + (b >> 1)) : 272 * (b >> 4) + (b & 15);
    }
    template <int p>
    __host__ __device__ static constexpr int woff(int r) {
        return p == 0 ? r : 16 * r + (r >= 8 ? 4 : 0);
    }
    template <int p>
    __host__ __device__ static constexpr int rbase(int b) {
        return p == 0 ? (VVH_RI_B128 ? b + 4 * (b >> 5) : b + (b >> 5)) : b + 4 * (b >> 7);
    }
    template <int p>
    __host__ __device__ static constexpr int roff(int r) {
        return p == 0 ? (VVH_RI_B128 ? 72 * r : 66 * r) : 272 * r;
    }
};
__host__ __device__ constexpr bool ri1024_check() {
    for (int b = 0; b < 64; ++b)
        for (int r = 0; r < 16; ++r) {
            if (ri_pad<1024, 0>(16 * b + r) != Ri1024::wbase<0>(b) + Ri1024::woff<0>(r)) return false;
            if (ri_pad<1024, 0>(b + 64 * r) != Ri1024::rbase<0>(b) + Ri1024::roff<0>(r)) return false;
            const int e = 256 * (b >> 4) + (b & 15) + 16 * r;
            if (ri_pad<1024, 1>(e) != 272 * (b >> 4) + (b & 15) + Ri1024::woff<1>(r)) return false;
        }
    for (int b = 0; b < 256; ++b)
        for (int r = 0; r < 4; ++r)
            if (ri_pad<1024, 1>(b + 256 * r) != b + 4 * (b >> 7) + Ri1024::roff<1>(r)) return false;
    // each layout is one-to-one (strictly increasing) and fits ri_floats
    for (int e = 1; e < 1024; ++e)
        if (ri_pad<1024, 0>(e) <= ri_pad<1024, 0>(e - 1) || ri_pad<1024, 1>(e) <= ri_pad<1024, 1>(e - 1)) return false;
    return ri_pad<1024, 0>(1023) < 1148 && ri_pad<1024, 1>(1023) < 1148;
}
static_assert(ri1024_check(), "Ri1024 decomposition of ri_pad");
// the N = 2048 / 4096 paddings: strictly increasing (one-to-one) and inside the buffer
__host__ __device__ constexpr bool pads_check() {
    for (int e = 1; e < 2048; ++e)
        if (ri_pad<2048, 0>(e) <= ri_pad<2048, 0>(e - 1) || ri_pad<2048, 1>(e) <= ri_pad<2048, 1>(e - 1)) return false;
    return ri_pad<2048, 0>(2047) < ri_floats<2048>() && ri_pad<2048, 1>(2047) < ri_floats<2048>();
}
static_assert(pads_check(), "ri_pad<2048, p>");

template <int BASE, int STEP>
__device__ __forceinline__ void lds_rd32x16(const float* base, float* o);
template <int STEP>
__device__ __forceinline__ void lds_rd32x4x4(const float* b0, const float* b1, const float* b2, const float* b3,
                                             float* o);
// RIV 1 (N = 1024): the reads as single ds_read_b32 (lds_rd32x16 /
// lds_rd32x4x4) so each real part and its imaginary part land straight in one
// complex register pair (RIV 0: the compiler's ds_read2 pairs, then v_movs).
template <int N, int p, bool PAIRED, int RIV = 0>
__device__ __forceinline__ void pass_exchange_ri(float2* v, int t, float* lds) {
    using G = Geo<N>;
    if constexpr (N == 1024 && RIV == 1) {
        constexpr int R = G::radix(p), R2 = G::radix(p + 1);
        static_assert(R == 16 && G::P / R == 1, "N = 1024: one radix-16 butterfly per thread before the exchange");
        const int wb = Ri1024::wbase<p>(bfly<N, p, PAIRED>(t, 0));
        int rb[G::P / R2];
#pragma unroll
        for (int i = 0; i < G::P / R2; ++i) rb[i] = Ri1024::rbase<p>(bfly<N, p + 1, PAIRED>(t, i));
        auto write = [&](auto part) {
            constexpr int Y = decltype(part)::value;
            if constexpr (p == 0 && VVH_RI_B128) {   // 16 contiguous floats: four 16 B stores
#pragma unroll
                for (int u = 0; u < R / 4; ++u)
                    *reinterpret_cast<vf4_t*>(lds + wb + 4 * u) =
                        Y ? vf4_t{v[4 * u].y, v[4 * u + 1].y, v[4 * u + 2].y, v[4 * u + 3].y}
                          : vf4_t{v[4 * u].x, v[4 * u + 1].x, v[4 * u + 2].x, v[4 * u + 3].x};
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) lds[wb + Ri1024::woff<p>(r)] = Y ? v[r].y : v[r].x;
            }
        };
        auto read = [&](float* o) {
            if constexpr (p == 0) {
                static_assert(G::P / R2 == 1 && R2 == 16, "pass 1 reads: one radix-16 butterfly");
                lds_rd32x16<0, 4 * Ri1024::roff<0>(1)>(lds + rb[0], o);
            } else {
                static_assert(G::P / R2 == 4 && R2 == 4, "pass 2 reads: four radix-4 butterflies");
                lds_rd32x4x4<4 * Ri1024::roff<1>(1)>(lds + rb[0], lds + rb[1], lds + rb[2], lds + rb[3], o);
            }
        };
        float re[G::P], im[G::P];
        write(std::integral_constant<int, 0>{});
        xsync<G::T>();
        read(re);
        xsync<G::T>();
        write(std::integral_constant<int, 1>{});
        xsync<G::T>();
        read(im);
#pragma unroll
        for (int k = 0; k < G::P; ++k) v[k] = make_float2(re[k], im[k]);
        return;
    }
    if constexpr (N == 1024) {
        constexpr int R = G::radix(p), R2 = G::radix(p + 1);
        static_assert(R == 16 && G::P / R == 1, "N = 1024: one radix-16 butterfly per thread before the exchange");
        float nx[G::P];
        const int wb = Ri1024::wbase<p>(bfly<N, p, PAIRED>(t, 0));
        int rb[G::P / R2];
#pragma unroll
        for (int i = 0; i < G::P / R2; ++i) rb[i] = Ri1024::rbase<p>(bfly<N, p + 1, PAIRED>(t, i));
        if constexpr (p == 0 && VVH_RI_B128) {   // 16 contiguous floats: four 16 B stores
#pragma unroll
            for (int u = 0; u < R / 4; ++u)
                *reinterpret_cast<vf4_t*>(lds + wb + 4 * u) =
                    vf4_t{v[4 * u].x, v[4 * u + 1].x, v[4 * u + 2].x, v[4 * u + 3].x};
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) lds[wb + Ri1024::woff<p>(r)] = v[r].x;
        }
        xsync<G::T>();
#pragma unroll
        for (int i = 0; i < G::P / R2; ++i)
#pragma unroll
            for (int r = 0; r < R2; ++r) nx[i * R2 + r] = lds[rb[i] + Ri1024::roff<p>(r)];
        xsync<G::T>();
        if constexpr (p == 0 && VVH_RI_B128) {
#pragma unroll
            for (int u = 0; u < R / 4; ++u)
                *reinterpret_cast<vf4_t*>(lds + wb + 4 * u) =
                    vf4_t{v[4 * u].y, v[4 * u + 1].y, v[4 * u + 2].y, v[4 * u + 3].y};
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) lds[wb + Ri1024::woff<p>(r)] = v[r].y;
        }
        xsync<G::T>();
#pragma unroll
        for (int i = 0; i < G::P / R2; ++i)
#pragma unroll
            for (int r = 0; r < R2; ++r)
                v[i * R2 + r] = make_float2(nx[i * R2 + r], lds[rb[i] + Ri1024::roff<p>(r)]);
        return;
    }
    constexpr int R = G::radix(p), Ns = G::ns(p), R2 = G::radix(p + 1);
    float nx[G::P];
#pragma unroll
    for (int i = 0; i < G::P / R; ++i) {
        const int b = bfly<N, p, PAIRED>(t, i);
        const int base = (b / Ns) * Ns * R + (b % Ns);
#pragma unroll
        for (int r = 0; r < R; ++r) lds[ri_pad<N, p>(base + r * Ns)] = v[i * R + r].x;
    }
    xsync<G::T>();
#pragma unroll
    for (int i = 0; i < G::P / R2; ++i) {
        const int b = bfly<N, p + 1, PAIRED>(t, i);
#pragma unroll
        for (int r = 0; r < R2; ++r) nx[i * R2 + r] = lds[ri_pad<N, p>(b + r * (N / R2))];
    }
    xsync<G::T>();   // one wave: LDS ops execute in order; across waves: s_barrier
#pragma unroll
    for (int i = 0; i < G::P / R; ++i) {
        const int b = bfly<N, p, PAIRED>(t, i);
        const int base = (b / Ns) * Ns * R + (b % Ns);
#pragma unroll
        for (int r = 0; r < R; ++r) lds[ri_pad<N, p>(base + r * Ns)] = v[i * R + r].y;
    }
    xsync<G::T>();
#pragma unroll
    for (int i = 0; i < G::P / R2; ++i) {
        const int b = bfly<N, p + 1, PAIRED>(t, i);
#pragma unroll
        for (int r = 0; r < R2; ++r) v[i * R2 + r] = make_float2(nx[i * R2 + r], lds[ri_pad<N, p>(b + r * (N / R2))]);
    }
    if constexpr (G::T > 64) xsync<G::T>();
}

// N = 1024 (passes 16, 16, 4), one wave per transform, not PAIRED: the
// exchange of whole complex values (b64 LDS accesses, half the LDS instructions
// of pass_exchange_ri for twice the buffer) with every address a per-lane base
// plus a compile-time offset.  Layout: element e at e + (e >> 4) (Geo::pad);
//   p 0 writes  16b + r             -> 17b + r
//   p 0 reads   b + 64r   (b < 64)  -> (b + (b >> 4)) + 68r
//   p 1 writes  256(b>>4) + (b&15) + 16r -> (272(b >> 4) + (b & 15)) + 17r
//   p 1 reads   b + 256r, b = t + 64i   -> (t + (t >> 4)) + 68i + 272r
// Bit-identical to pass_exchange (a permutation through LDS either way).
__host__ __device__ constexpr bool c1024_check() {
    for (int b = 0; b < 64; ++b)
        for (int r = 0; r < 16; ++r) {
            if (Geo<1024>::pad(16 * b + r) != 17 * b + r) return false;
            if (Geo<1024>::pad(b + 64 * r) != b + (b >> 4) + 68 * r) return false;
            if (Geo<1024>::pad(256 * (b >> 4) + (b & 15) + 16 * r) != 272 * (b >> 4) + (b & 15) + 17 * r) return false;
        }
    for (int t = 0; t < 64; ++t)
        for (int i = 0; i < 4; ++i)
            for (int r = 0; r < 4; ++r)
                if (Geo<1024>::pad(t + 64 * i + 256 * r) != t + (t >> 4) + 68 * i + 272 * r) return false;
    return true;
}
static_assert(c1024_check(), "pass_exchange_c1024 offsets");

// LDS reads as single ds_read_b64.  Left to itself the compiler pairs
// neighbouring b64 reads into ds_read2_b64, which moves the same bytes at half
// the rate (8 LDS cycles for two, against 2 per ds_read_b64: MI355X_MICROARCH.md,
// LDS table).  Each helper is ONE asm statement that issues its reads and then
// waits (s_waitcnt lgkmcnt(0)): the outputs are defined only after the wait, so
// the compiler can neither use nor copy them early (a read in one asm and the
// wait in another would let it copy a not-yet-written register).  Outputs are
// early-clobber: the address register stays intact while the reads issue.
// 16 reads from the LDS address `base` at byte offsets BASE + i * STEP (i < 16)
template <int BASE, int STEP>
__device__ __forceinline__ void lds_rd64x16(const float2* base, float2* out) {
    static_assert(BASE >= 0 && BASE + 15 * STEP < 65536 && BASE + 15 * STEP >= 0, "ds offset range");
    const unsigned a = (unsigned)(uintptr_t)base;
    vf2_t o[16];
    asm volatile("ds_read_b64 %0, %16 offset:%17\n\t"
                 "ds_read_b64 %1, %16 offset:%18\n\t"
                 "ds_read_b64 %2, %16 offset:%19\n\t"
                 "ds_read_b64 %3, %16 offset:%20\n\t"
                 "ds_read_b64 %4, %16 offset:%21\n\t"
                 "ds_read_b64 %5, %16 offset:%22\n\t"
                 "ds_read_b64 %6, %16 offset:%23\n\t"
                 "ds_read_b64 %7, %16 offset:%24\n\t"
                 "ds_read_b64 %8, %16 offset:%25\n\t"
                 "ds_read_b64 %9, %16 offset:%26\n\t"
                 "ds_read_b64 %10, %16 offset:%27\n\t"
                 "ds_read_b64 %11, %16 offset:%28\n\t"
                 "ds_read_b64 %12, %16 offset:%29\n\t"
                 "ds_read_b64 %13, %16 offset:%30\n\t"
                 "ds_read_b64 %14, %16 offset:%31\n\t"
                 "ds_read_b64 %15, %16 offset:%32\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]), "=&v"(o[7]), "=&v"(o[8]), "=&v"(o[9]), "=&v"(o[10]), "=&v"(o[11]), "=&v"(o[12]), "=&v"(o[13]), "=&v"(o[14]), "=&v"(o[15])
                 : "v"(a), "n"(BASE + 0 * STEP), "n"(BASE + 1 * STEP), "n"(BASE + 2 * STEP), "n"(BASE + 3 * STEP), "n"(BASE + 4 * STEP), "n"(BASE + 5 * STEP), "n"(BASE + 6 * STEP), "n"(BASE + 7 * STEP), "n"(BASE + 8 * STEP), "n"(BASE + 9 * STEP), "n"(BASE + 10 * STEP), "n"(BASE + 11 * STEP), "n"(BASE + 12 * STEP), "n"(BASE + 13 * STEP), "n"(BASE + 14 * STEP), "n"(BASE + 15 * STEP));
#pragma unroll
    for (int i = 0; i < 16; ++i) out[i] = upk(o[i]);
}
// 16 single-dword reads (b32, never merged into ds_read2) at byte offsets
// BASE + i * STEP from `base`, then the wait -- one asm statement as above.
// The outputs are 16 independent registers, so the caller can pair each with
// another value into one complex register pair without a move (the compiler's
// ds_read2 merging fixes each destination pair, and re-pairing costs v_movs).
template <int BASE, int STEP>
__device__ __forceinline__ void lds_rd32x16(const float* base, float* o) {
    static_assert(BASE >= 0 && BASE + 15 * STEP < 65536, "ds offset range");
    const unsigned a = (unsigned)(uintptr_t)base;
    asm volatile("ds_read_b32 %0, %16 offset:%17\n\t"
                 "ds_read_b32 %1, %16 offset:%18\n\t"
                 "ds_read_b32 %2, %16 offset:%19\n\t"
                 "ds_read_b32 %3, %16 offset:%20\n\t"
                 "ds_read_b32 %4, %16 offset:%21\n\t"
                 "ds_read_b32 %5, %16 offset:%22\n\t"
                 "ds_read_b32 %6, %16 offset:%23\n\t"
                 "ds_read_b32 %7, %16 offset:%24\n\t"
                 "ds_read_b32 %8, %16 offset:%25\n\t"
                 "ds_read_b32 %9, %16 offset:%26\n\t"
                 "ds_read_b32 %10, %16 offset:%27\n\t"
                 "ds_read_b32 %11, %16 offset:%28\n\t"
                 "ds_read_b32 %12, %16 offset:%29\n\t"
                 "ds_read_b32 %13, %16 offset:%30\n\t"
                 "ds_read_b32 %14, %16 offset:%31\n\t"
                 "ds_read_b32 %15, %16 offset:%32\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]), "=&v"(o[7]), "=&v"(o[8]), "=&v"(o[9]), "=&v"(o[10]), "=&v"(o[11]), "=&v"(o[12]), "=&v"(o[13]), "=&v"(o[14]), "=&v"(o[15])
                 : "v"(a), "n"(BASE + 0 * STEP), "n"(BASE + 1 * STEP), "n"(BASE + 2 * STEP), "n"(BASE + 3 * STEP), "n"(BASE + 4 * STEP), "n"(BASE + 5 * STEP), "n"(BASE + 6 * STEP), "n"(BASE + 7 * STEP), "n"(BASE + 8 * STEP), "n"(BASE + 9 * STEP), "n"(BASE + 10 * STEP), "n"(BASE + 11 * STEP), "n"(BASE + 12 * STEP), "n"(BASE + 13 * STEP), "n"(BASE + 14 * STEP), "n"(BASE + 15 * STEP));
}
// 4 x 4 single-dword reads: o[4 i + r] from base i at byte offset r * STEP
template <int STEP>
__device__ __forceinline__ void lds_rd32x4x4(const float* b0, const float* b1, const float* b2, const float* b3,
                                             float* o) {
    static_assert(3 * STEP < 65536, "ds offset range");
    const unsigned a0 = (unsigned)(uintptr_t)b0, a1 = (unsigned)(uintptr_t)b1, a2 = (unsigned)(uintptr_t)b2,
                   a3 = (unsigned)(uintptr_t)b3;
    asm volatile("ds_read_b32 %0, %16 offset:%20\n\t"
                 "ds_read_b32 %1, %16 offset:%21\n\t"
                 "ds_read_b32 %2, %16 offset:%22\n\t"
                 "ds_read_b32 %3, %16 offset:%23\n\t"
                 "ds_read_b32 %4, %17 offset:%20\n\t"
                 "ds_read_b32 %5, %17 offset:%21\n\t"
                 "ds_read_b32 %6, %17 offset:%22\n\t"
                 "ds_read_b32 %7, %17 offset:%23\n\t"
                 "ds_read_b32 %8, %18 offset:%20\n\t"
                 "ds_read_b32 %9, %18 offset:%21\n\t"
                 "ds_read_b32 %10, %18 offset:%22\n\t"
                 "ds_read_b32 %11, %18 offset:%23\n\t"
                 "ds_read_b32 %12, %19 offset:%20\n\t"
                 "ds_read_b32 %13, %19 offset:%21\n\t"
                 "ds_read_b32 %14, %19 offset:%22\n\t"
                 "ds_read_b32 %15, %19 offset:%23\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]), "=&v"(o[7]), "=&v"(o[8]), "=&v"(o[9]), "=&v"(o[10]), "=&v"(o[11]), "=&v"(o[12]), "=&v"(o[13]), "=&v"(o[14]), "=&v"(o[15])
                 : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "n"(0 * STEP), "n"(1 * STEP), "n"(2 * STEP), "n"(3 * STEP));
}
// 32 reads of float2 from `base`: consecutive (byte offsets 8 i, i < 32), or with
// GAP one float2 skipped after the first 16 (offsets 8 (i + i / 16): the 32 x 32
// transpose's row layout, r32_transpose)
template <bool GAP = false>
__device__ __forceinline__ void lds_rd64x32(const float2* base, float2* out) {
    const unsigned a = (unsigned)(uintptr_t)base;
    vf2_t o[32];
    asm volatile("ds_read_b64 %0, %32 offset:%33\n\t"
                 "ds_read_b64 %1, %32 offset:%34\n\t"
                 "ds_read_b64 %2, %32 offset:%35\n\t"
                 "ds_read_b64 %3, %32 offset:%36\n\t"
                 "ds_read_b64 %4, %32 offset:%37\n\t"
                 "ds_read_b64 %5, %32 offset:%38\n\t"
                 "ds_read_b64 %6, %32 offset:%39\n\t"
                 "ds_read_b64 %7, %32 offset:%40\n\t"
                 "ds_read_b64 %8, %32 offset:%41\n\t"
                 "ds_read_b64 %9, %32 offset:%42\n\t"
                 "ds_read_b64 %10, %32 offset:%43\n\t"
                 "ds_read_b64 %11, %32 offset:%44\n\t"
                 "ds_read_b64 %12, %32 offset:%45\n\t"
                 "ds_read_b64 %13, %32 offset:%46\n\t"
                 "ds_read_b64 %14, %32 offset:%47\n\t"
                 "ds_read_b64 %15, %32 offset:%48\n\t"
                 "ds_read_b64 %16, %32 offset:%49\n\t"
                 "ds_read_b64 %17, %32 offset:%50\n\t"
                 "ds_read_b64 %18, %32 offset:%51\n\t"
                 "ds_read_b64 %19, %32 offset:%52\n\t"
                 "ds_read_b64 %20, %32 offset:%53\n\t"
                 "ds_read_b64 %21, %32 offset:%54\n\t"
                 "ds_read_b64 %22, %32 offset:%55\n\t"
                 "ds_read_b64 %23, %32 offset:%56\n\t"
                 "ds_read_b64 %24, %32 offset:%57\n\t"
                 "ds_read_b64 %25, %32 offset:%58\n\t"
                 "ds_read_b64 %26, %32 offset:%59\n\t"
                 "ds_read_b64 %27, %32 offset:%60\n\t"
                 "ds_read_b64 %28, %32 offset:%61\n\t"
                 "ds_read_b64 %29, %32 offset:%62\n\t"
                 "ds_read_b64 %30, %32 offset:%63\n\t"
                 "ds_read_b64 %31, %32 offset:%64\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]), "=&v"(o[7]), "=&v"(o[8]), "=&v"(o[9]), "=&v"(o[10]), "=&v"(o[11]), "=&v"(o[12]), "=&v"(o[13]), "=&v"(o[14]), "=&v"(o[15]), "=&v"(o[16]), "=&v"(o[17]), "=&v"(o[18]), "=&v"(o[19]), "=&v"(o[20]), "=&v"(o[21]), "=&v"(o[22]), "=&v"(o[23]), "=&v"(o[24]), "=&v"(o[25]), "=&v"(o[26]), "=&v"(o[27]), "=&v"(o[28]), "=&v"(o[29]), "=&v"(o[30]), "=&v"(o[31])
                 : "v"(a), "n"(8 * (0 + (GAP ? 0 / 16 : 0))), "n"(8 * (1 + (GAP ? 1 / 16 : 0))), "n"(8 * (2 + (GAP ? 2 / 16 : 0))), "n"(8 * (3 + (GAP ? 3 / 16 : 0))), "n"(8 * (4 + (GAP ? 4 / 16 : 0))), "n"(8 * (5 + (GAP ? 5 / 16 : 0))), "n"(8 * (6 + (GAP ? 6 / 16 : 0))), "n"(8 * (7 + (GAP ? 7 / 16 : 0))), "n"(8 * (8 + (GAP ? 8 / 16 : 0))), "n"(8 * (9 + (GAP ? 9 / 16 : 0))), "n"(8 * (10 + (GAP ? 10 / 16 : 0))), "n"(8 * (11 + (GAP ? 11 / 16 : 0))), "n"(8 * (12 + (GAP ? 12 / 16 : 0))), "n"(8 * (13 + (GAP ? 13 / 16 : 0))), "n"(8 * (14 + (GAP ? 14 / 16 : 0))), "n"(8 * (15 + (GAP ? 15 / 16 : 0))), "n"(8 * (16 + (GAP ? 16 / 16 : 0))), "n"(8 * (17 + (GAP ? 17 / 16 : 0))), "n"(8 * (18 + (GAP ? 18 / 16 : 0))), "n"(8 * (19 + (GAP ? 19 / 16 : 0))), "n"(8 * (20 + (GAP ? 20 / 16 : 0))), "n"(8 * (21 + (GAP ? 21 / 16 : 0))), "n"(8 * (22 + (GAP ? 22 / 16 : 0))), "n"(8 * (23 + (GAP ? 23 / 16 : 0))), "n"(8 * (24 + (GAP ? 24 / 16 : 0))), "n"(8 * (25 + (GAP ? 25 / 16 : 0))), "n"(8 * (26 + (GAP ? 26 / 16 : 0))), "n"(8 * (27 + (GAP ? 27 / 16 : 0))), "n"(8 * (28 + (GAP ? 28 / 16 : 0))), "n"(8 * (29 + (GAP ? 29 / 16 : 0))), "n"(8 * (30 + (GAP ? 30 / 16 : 0))), "n"(8 * (31 + (GAP ? 31 / 16 : 0))));
#pragma unroll
    for (int i = 0; i < 32; ++i) out[i] = upk(o[i]);
}

template <int p>
__device__ __forceinline__ void pass_exchange_c1024(float2* v, int t, float2* lds) {
    static_assert(p == 0 || p == 1, "N = 1024 has two exchanges");
    const float2* q = lds + t + (t >> 4);   // the read base
    if constexpr (p == 0) {
        float2* w = lds + 17 * t;
#pragma unroll
        for (int r = 0; r < 16; ++r) w[r] = v[r];
        xsync<64>();
        lds_rd64x16<0, 8 * 68>(q, v);
    } else {
        float2* w = lds + 272 * (t >> 4) + (t & 15);
#pragma unroll
        for (int r = 0; r < 16; ++r) w[17 * r] = v[r];
        xsync<64>();
        float2 t4[16];   // t4[4 r + i] = element b + 256 r, b = t + 64 i: offsets 8 (68 i + 272 r)
        lds_rd64x16<0, 8 * 68>(q, t4);   // 68 (4 r + i) = 68 i + 272 r
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[4 * i + r] = t4[4 * r + i];
    }
    xsync<64>();   // the next exchange's writes must not pass these reads (compiler order only)
}

// ---- 1024 = 32 x 32 transforms on half-waves (k_fir_r32, k_c2c_r32) -------
__device__ __forceinline__ constexpr float cos32(int m) {
    constexpr float c1 = 0.98078528040323044913f, c2 = 0.92387953251128675613f, c3 = 0.83146961230254523708f,
                    c4 = 0.70710678118654752440f, c5 = 0.55557023301960222474f, c6 = 0.38268343236508977173f,
                    c7 = 0.19509032201612826785f;
    switch (m & 31) {
        case 0: return 1.0f;  case 1: return c1;  case 2: return c2;  case 3: return c3;
        case 4: return c4;    case 5: return c5;  case 6: return c6;  case 7: return c7;
        case 8: return 0.0f;  case 9: return -c7; case 10: return -c6; case 11: return -c5;
        case 12: return -c4;  case 13: return -c3; case 14: return -c2; case 15: return -c1;
        case 16: return -1.0f; case 17: return -c1; case 18: return -c2; case 19: return -c3;
        case 20: return -c4;  case 21: return -c5; case 22: return -c6; case 23: return -c7;
        case 24: return 0.0f; case 25: return c7;  case 26: return c6;  case 27: return c5;
        case 28: return c4;   case 29: return c3;  case 30: return c2;  default: return c1;
    }
}

// In-register DFT of length 32 (natural order in and out) as radix 4 x 8:
// DFT_8 of each residue class x[4 m + j], twiddle W_32^(j k1), then a DFT_4
// over j -> X[k1 + 8 k2].  20 non-trivial twiddles plus 2 per DFT_8 (28
// complex multiplies; the radix-2 split takes 34), the same 160 complex adds.
// The twiddle constants are SGPR operands of the packed FMA (cmul's asm would
// copy each into VGPRs first); cmul's roundings.
template <bool FWD>
__device__ __forceinline__ float2 tw32(float2 o, int e) {
    e &= 31;
    if (e == 0) return o;
    if (e == 16) return upk(-pk(o));
    if (e == 8) return FWD ? cmul_mi(o) : cmul_pi(o);
    if (e == 24) return FWD ? cmul_pi(o) : cmul_mi(o);
    const float c = cos32(e), sn = FWD ? -cos32(e - 8) : cos32(e - 8);   // -+sin(2 pi e / 32)
    const vf2_t O = pk(o);
    return upk(__builtin_elementwise_fma(O.xx, vf2_t{c, sn}, O.yy * vf2_t{-sn, c}));
}
template <bool FWD>
__device__ __forceinline__ void dft32(float2* v) {
    float2 y[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int m = 0; m < 8; ++m) y[j][m] = v[4 * m + j];
#pragma unroll
    for (int j = 0; j < 4; ++j) Dft<8, FWD>::run(y[j]);
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) {
        const float2 a0 = y[0][k1], a1 = tw32<FWD>(y[1][k1], k1), a2 = tw32<FWD>(y[2][k1], 2 * k1),
                     a3 = tw32<FWD>(y[3][k1], 3 * k1);
        const float2 s02 = cadd(a0, a2), d02 = csub(a0, a2), s13 = cadd(a1, a3), d13 = csub(a1, a3);
        v[k1] = cadd(s02, s13);
        v[k1 + 16] = csub(s02, s13);
        // d13 * W_4^1 (forward -i, backward +i) folded into the adds, as Dft<4>
        v[k1 + 8] = FWD ? cadd_i<false>(d02, d13) : cadd_i<true>(d02, d13);
        v[k1 + 24] = FWD ? cadd_i<true>(d02, d13) : cadd_i<false>(d02, d13);
    }
}

// a * conj(w) in two packed instructions (cmul's sequence with the signs of w.y flipped)
__device__ __forceinline__ float2 cmulc(float2 a, float2 w) {
    const vf2_t A = pk(a), W = pk(w);
    vf2_t t, r;
    // t = a.yy * (w.y, w.x); r = a.xx * (w.x, -w.y) + t = (a.x w.x + a.y w.y, a.y w.x - a.x w.y)
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(t) : "v"(A), "v"(W));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_hi:[0,1,0]" : "=v"(r) : "v"(A), "v"(W), "v"(t));
    return upk(r);
}

constexpr int R32_ROW = 33;                   // padded row of the 32 x 32 transpose (float2)
constexpr int R32_BUF = 32 * R32_ROW;         // one transform's exchange buffer (float2)

// register r of every lane -> row r, column `col`; then row `row` -> registers
// (col = row = the lane's index in its half for the plain split).
// Row layout: columns 0..15 at slots 0..15, columns 16..31 at slots 17..32
// (slot = col + col / 16), rows R32_ROW = 33 apart.  Banks (MI355X_MICROARCH
// §LDS): ds_write_b64 serves 16 contiguous lanes per cycle on (a/4) mod 32,
// i.e. 16 float2 slots; the paired FIR / STFT layout writes columns 2k (lanes
// 0..15) or 2k + 1 (lanes 16..31), which the plain col + 33 r layout put on 8
// slots twice (2-way, SQ_LDS_BANK_CONFLICT 0.38 of the LDS cycles in round 4);
// the gap after column 15 spreads any 16 columns of one parity, and any 16
// consecutive columns, over 16 distinct slots.  ds_read_b64 serves 32 lanes on
// (a/4) mod 64 = 32 slots: lane rows 33 apart stay distinct for any row
// permutation of the 32 lanes.  So every write and read here is conflict-free.
__device__ __forceinline__ void r32_transpose(float2* v, float2* buf, int col, int row) {
    float2* w = buf + col + (col >> 4);
#pragma unroll
    for (int r = 0; r < 32; ++r) w[R32_ROW * r] = v[r];
    xsync<64>();
    lds_rd64x32<true>(buf + R32_ROW * row, v);
    xsync<64>();   // the next transpose's writes must stay behind these reads
}
__device__ __forceinline__ void r32_transpose(float2* v, float2* buf, int lane32) { r32_transpose(v, buf, lane32, lane32); }

// Lanes l and l + 16 of each half-wave trade a <-> b (v_permlane16_swap: rows
// 1 and 3 of `a` with rows 0 and 2 of `b`): afterwards lane l < 16 holds (its a,
// lane l+16's a) and lane l + 16 (lane l's b, its b).  Two dwords loaded as one
// 8 B pair per lane (samples 2l, 2l+1 of 64) become samples 2l, 2l + 32 in lane
// l < 16 and 2l + 1, 2l + 33 in lane l + 16: the r32 layout (one residue mod 32
// per lane) with residue 2 (l & 15) + (l >> 4).  The same swap turns two r32
// registers (rows b, b + 1 of that residue layout) back into 8 B pairs.
// Half-waves trade a <-> b (v_permlane32_swap: lanes 32..63 of `a` with lanes
// 0..31 of `b`): afterwards a = (half 0's a | half 0's b), b = (half 1's a |
// half 1's b) -- each register then holds one half's pair of values across the
// whole wave.
__device__ __forceinline__ void r32_halfswap(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
// (a.lo, b.lo) (SEL 0) or (a.hi, b.hi) (SEL 1) as one v_pk_mov_b32: two
// registers from two different pairs without a v_mov per half
template <int SEL>
__device__ __forceinline__ vf2_t pk_pair(vf2_t a, vf2_t b) {
    vf2_t r;
    if constexpr (SEL) asm("v_pk_mov_b32 %0, %1, %2 op_sel:[1,1]" : "=v"(r) : "v"(a), "v"(b));
    else asm("v_pk_mov_b32 %0, %1, %2 op_sel:[0,0]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ void r32_pairswap(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}


// v[r] *= W_1024^(m r) (FWD) or its conjugate, r = 1..31, from an LDS table
// laid out [r][m] (atw: entry [0][m]); eight ds_read_b64 at a time
template <bool FWD>
__device__ __forceinline__ void r32_twiddle(float2* v, const float2* atw) {
    float2 w[16];
    lds_rd64x16<0, 256>(atw, w);   // r = 0..15 (row 0 = W^0, unused)
#pragma unroll
    for (int r = 1; r < 16; ++r) v[r] = FWD ? cmul(v[r], w[r]) : cmulc(v[r], w[r]);
    lds_rd64x16<16 * 256, 256>(atw, w);   // r = 16..31
#pragma unroll
    for (int r = 16; r < 32; ++r) v[r] = FWD ? cmul(v[r], w[r - 16]) : cmulc(v[r], w[r - 16]);
}

// NOX: timing ablation only (scripts/membench.hip) -- the passes without their
// exchanges, i.e. a wrong transform with the FFT's arithmetic but no LDS traffic.
// C64: N = 1024 one-wave transforms exchange through pass_exchange_c1024.
template <int N, bool FWD, int p, bool PAIRED, bool RI = false, bool NOX = false, bool C64 = false, int RIV = 0>
struct PassChain {
    template <class TW>
    __device__ __forceinline__ static void run(float2* v, int t, float2* lds, const TW& tw) {
        pass_compute<N, FWD, p, PAIRED>(v, t, tw);
        if constexpr (p + 1 < Geo<N>::NPASS) {
            if constexpr (NOX) asm volatile("" ::: "memory");
            else if constexpr (C64) pass_exchange_c1024<p>(v, t, lds);
            else if constexpr (RI) pass_exchange_ri<N, p, PAIRED, RIV>(v, t, reinterpret_cast<float*>(lds));
            else pass_exchange<N, p, PAIRED>(v, t, lds);
            PassChain<N, FWD, p + 1, PAIRED, RI, NOX, C64, RIV>::run(v, t, lds, tw);
        }
    }
};

// Full transform.  On entry v[r] = x[t + r*T] (r < P).  On exit register q
// holds X[out_pos<N, PAIRED>(t, q)].  RI: `lds` needs only Geo<N>::LDS floats
// (pass_exchange_ri) instead of Geo<N>::LDS float2.  C64 (N = 1024, T = 64,
// not PAIRED): the explicit-offset complex exchange, Geo<N>::LDS float2.
template <int N, bool FWD, bool PAIRED = false, bool RI = false, class TW = TwTab<N>, bool NOX = false,
          bool C64 = false, int RIV = 0>
__device__ __forceinline__ void fft_regs(float2* v, int t, float2* lds, const TW& tw) {
    static_assert(!PAIRED || Geo<N>::CAN_PAIR, "mirror pairing needs >= 2 last-pass butterflies per thread");
    static_assert(!C64 || (N == 1024 && !PAIRED && !RI), "pass_exchange_c1024: N = 1024, one wave, not paired");
    PassChain<N, FWD, 0, PAIRED, RI, NOX, C64, RIV>::run(v, t, lds, tw);
}

// ---- shared pieces of the persistent streaming kernels ---------------------
// A transform owned by >= 64 threads has one work item per wave: make the loop
// state wave-uniform (SGPRs, scalar branches) so the compiler does not keep
// exec-masked copies of the register arrays alive across the prefetch branch.
template <int T>
__device__ __forceinline__ long long uni(long long x) {
    if constexpr (T >= 64) {
        const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(x & 0xffffffffLL));
        const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)((unsigned long long)x >> 32));
        return (long long)(((unsigned long long)hi << 32) | lo);
    } else {
        return x;
    }
}

// ---- hand-counted memory pipeline (LDS-DMA input spans) ---------------------
// hipcc does not track inline-asm memory operations, so a kernel using these
// counts them itself: the vector-memory ops of a wave retire in issue order
// (loads, stores and LDS-DMA alike), and inside such a loop the only ops are
// these (no compiler-generated global access, no scratch).
// 16 B per lane global -> LDS (dest = M0 + lane*16; M0 is written in the same
// statement that uses it, as the compiler reserves it).
__device__ __forceinline__ void glds16(const float* gsrc, float* lds_dst) {
    const unsigned l = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(l)
                 : "memory");
}
// the same with a cache-policy suffix: loads POL 1 "nt", 2 "sc1"; stores POL 1 "sc1", 2 "sc0 sc1 nt"
template <int POL>
__device__ __forceinline__ void glds16_pol(const float* gsrc, float* lds_dst) {
    const unsigned l = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(uintptr_t)lds_dst);
    unsigned keep;
    if constexpr (POL == 1)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(gsrc), "s"(l) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(gsrc), "s"(l) : "memory");
}
template <int IMM, int POL>
__device__ __forceinline__ void st4_pol_sbase(unsigned lane_off, float v, const void* base) {
    if constexpr (POL == 1)
        asm volatile("global_store_dword %0, %1, %2 offset:%3 sc1" ::"v"(lane_off), "v"(v), "s"(base), "n"(IMM) : "memory");
    else
        asm volatile("global_store_dword %0, %1, %2 offset:%3 sc0 sc1 nt" ::"v"(lane_off), "v"(v), "s"(base), "n"(IMM)
                     : "memory");
}
// The trailing s_nop covers the gfx9 hazard "VALU write of a >8-byte VMEM
// store's data VGPRs right after the store", which hipcc does not model for asm.
__device__ __forceinline__ void st16_nt_counted(vf4_t* p, vf4_t v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st4_counted(float* p, float v) {
    asm volatile("global_store_dword %0, %1, off" ::"v"(p), "v"(v) : "memory");
}
// the same store from lane 0 alone (exec narrowed inside the asm, so it is
// still exactly one counted instruction per wave and no other lane writes
// anywhere: a shared dummy target would take every wave's 63 spare lanes)
__device__ __forceinline__ void st4_lane0_counted(float* p, float v) {
    unsigned long long keep;
    asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\tglobal_store_dword %1, %2, off\n\ts_mov_b64 exec, %0"
                 : "=&s"(keep)
                 : "v"(p), "v"(v)
                 : "memory");
}
// dword streaming store at wave-uniform base (SGPR pair) + 32-bit lane offset + IMM
// (13-bit signed immediate: -4096..4095)
template <int IMM>
__device__ __forceinline__ void st4_nt_sbase(unsigned lane_off, float v, const void* base) {
    static_assert(IMM >= -4096 && IMM <= 4095, "global offset range");
    asm volatile("global_store_dword %0, %1, %2 offset:%3 nt" ::"v"(lane_off), "v"(v), "s"(base), "n"(IMM)
                 : "memory");
}
// 8 B (complex) streaming store at wave-uniform base + 32-bit lane offset + IMM
template <int IMM>
__device__ __forceinline__ void st8_nt_sbase(unsigned lane_off, float2 v, const void* base) {
    static_assert(IMM >= -4096 && IMM <= 4095, "global offset range");
    const vf2_t d = pk(v);
    asm volatile("global_store_dwordx2 %0, %1, %2 offset:%3 nt" ::"v"(lane_off), "v"(d), "s"(base), "n"(IMM)
                 : "memory");
}
// the same with a plain (write-back) store
template <int IMM>
__device__ __forceinline__ void st4_sbase(unsigned lane_off, float v, const void* base) {
    static_assert(IMM >= -4096 && IMM <= 4095, "global offset range");
    asm volatile("global_store_dword %0, %1, %2 offset:%3" ::"v"(lane_off), "v"(v), "s"(base), "n"(IMM)
                 : "memory");
}
template <int CNT>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CNT) : "memory");
}
__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void lds_barrier() { asm volatile("s_barrier" ::: "memory"); }

// Contiguous chunk [lo, hi) of `total` work items for persistent slot g of S:
// consecutive items of a slot share input lines in L1/L2 (overlapping frames,
// overlap-save halos) instead of being fetched by another XCD.
__device__ __forceinline__ void chunk_of(long long total, long long g, long long S, long long* lo,
                                         long long* hi) {
    const long long per = total / S, rem = total % S;
    *lo = g * per + (g < rem ? g : rem);
    *hi = *lo + per + (g < rem ? 1 : 0);
}

// Work sequence of persistent slot `slot` (of F per block) over items [0, total):
// the block groups blockIdx % 8 (the blocks sharing one XCD and its L2) each
// take a contiguous share, and inside a group consecutive slots take
// consecutive items, so a group sweeps its share as one front.  Items that
// share input lines (overlapping frames, overlap-save halos) are then fetched
// once into that XCD's L2, and the DRAM sees few open pages at a time.
// A slot visits first, first + step, ... < end.
__device__ __forceinline__ void xcd_walk(long long total, int F, int slot, long long* first, long long* end,
                                         long long* step) {
    const long long nb = gridDim.x, b = blockIdx.x;
    const long long ng = nb < 8 ? nb : 8;
    const long long grp = b % ng;
    const long long nbg = (nb - grp + ng - 1) / ng;   // blocks in this group
    long long lo, hi;
    chunk_of(total, grp, ng, &lo, &hi);
    *first = lo + (b / ng) * F + slot;
    *end = hi;
    *step = nbg * F;
}

// Band walk (persistent, grid a multiple of 8): each step the whole grid covers
// S = gridDim.x * F consecutive items, cut into 8 contiguous sub-bands, one per
// XCD (block b runs on XCD b % 8), so at any time the chip reads and writes one
// moving band of the data and neighbouring items share their XCD's L2.
__device__ __forceinline__ void band_walk(long long total, int F, int slot, long long* first, long long* end,
                                          long long* step) {
    const long long nb = gridDim.x, b = blockIdx.x;
    *first = (b % 8) * (nb / 8) * F + (b / 8) * F + slot;
    *step = nb * F;
    *end = total;
}

// Work sequence of transform slot `slot` (of F per block): with chunk > 0 the
// launch is not persistent -- block b owns items [b*chunk, (b+1)*chunk), its
// slots interleaved -- otherwise the persistent xcd_walk.
__device__ __forceinline__ void work_walk(long long total, int F, int slot, long long chunk, long long* first,
                                          long long* end, long long* step) {
    if (chunk > 0) {
        *first = (long long)blockIdx.x * chunk + slot;
        *step = F;
        const long long e = (long long)(blockIdx.x + 1) * chunk;
        *end = e < total ? e : total;
    } else {
        xcd_walk(total, F, slot, first, end, step);
    }
}

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

// W_{2M}^k for k < M (split-step twiddles) staged in LDS: direct or two-level.
template <int M>
struct PostLayout {
    static constexpr bool SPLIT = 2 * M > 2048;
    static constexpr int ENTRIES = SPLIT ? 64 + M / 64 : M;
};

template <int M>
struct PostTab {
    const float2* tab;
    __device__ __forceinline__ float2 operator()(int k) const {
        if constexpr (PostLayout<M>::SPLIT) return cmul(tab[k & 63], tab[64 + (k >> 6)]);
        else return tab[k];
    }
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

}  // namespace vvh
