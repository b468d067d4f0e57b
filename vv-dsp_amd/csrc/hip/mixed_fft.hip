// mixed_fft.hip -- batched mixed-radix FFT for 7-smooth lengths that are not
// powers of two (n = 2^a 3^b 5^c 7^d, 6 <= n <= 4096) on gfx950.
//
// The reference runs every non-power-of-two length through its O(n^2) DFT
// (src/spectral/fft_kiss.c:76-92, dispatched at :114-116, and for all C2R).
// The common audio lengths are 7-smooth (STFT frames of 400, 480, 960 or 2000
// samples; 44100 = 2^2 3^2 5^2 7^2), so this kernel replaces that O(n^2) work
// with a Stockham autosort FFT whose radices are read from a per-length plan:
//
//   pass p, radix R, Ns = product of the earlier radices, butterfly j < n/R:
//     inputs   j + r*n/R                        (r < R)
//     twiddle  W_{Ns*R}^{(j mod Ns)*r} = W_n^{r*(j mod Ns)*n/(Ns*R)}
//     outputs  (j div Ns)*Ns*R + (j mod Ns) + r*Ns
//
// One transform lives in LDS (n float2) and is owned by T threads, each holding
// at most 16 points per pass in VGPRs: a pass reads all of a thread's
// butterflies, synchronises, and writes them back in place.  The W_n table
// (rounded once from double on the host, tables.hip) is staged in LDS with the
// transforms.  Radix-2/4/8 butterflies are the exact in-register DFTs of
// fft_core.hpp; radix 3/5/7 use the symmetric-pair form with constants written
// to 20 digits.  The inverse is conj(FFT(conj x)), then the caller's scale.
//
// Loads and stores are lane-contiguous (coalesced); a transform is read whole
// into LDS before any of it is written, so in == out is safe.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

#include <cstdlib>

namespace vvh {

namespace {

constexpr int MIX_MAXP = 12;    // 3^7 = 2187 needs 7 passes; 4096-bounded lengths fit in 12
constexpr int MIX_MAXN = 4096;
constexpr int MIX_PTS = 16;     // points per thread per pass at most
#ifndef VVH_MIX_LB
#define VVH_MIX_LB 1
#endif
constexpr int LB = VVH_MIX_LB;

struct MixedPlan {
    int n;
    int np;
    int radix[MIX_MAXP];
    int ns[MIX_MAXP];
    int tstep[MIX_MAXP];   // n / (Ns * R): W_{Ns R}^m = W_n^(m * tstep)
    float rns[MIX_MAXP];   // 1 / Ns for the butterfly index split
};

// cos / sin(2*pi*j/R) for the odd radices, j = 1 .. (R-1)/2
template <int R>
struct OddC;
template <>
struct OddC<3> {
    __device__ static constexpr float c(int) { return -0.5f; }
    __device__ static constexpr float s(int) { return 0.86602540378443864676f; }
};
template <>
struct OddC<5> {
    __device__ static constexpr float c(int j) { return j == 1 ? 0.30901699437494742410f : -0.80901699437494742410f; }
    __device__ static constexpr float s(int j) { return j == 1 ? 0.95105651629515357212f : 0.58778525229247312917f; }
};
template <>
struct OddC<7> {
    __device__ static constexpr float c(int j) {
        return j == 1 ? 0.62348980185873353053f : j == 2 ? -0.22252093395631440429f : -0.90096886790241912624f;
    }
    __device__ static constexpr float s(int j) {
        return j == 1 ? 0.78183148246802980871f : j == 2 ? 0.97492791218182360702f : 0.43388373911755812048f;
    }
};

// forward DFT of odd length R over symmetric pairs s_m = x_m + x_{R-m},
// d_m = x_m - x_{R-m}:  X_k = x0 + sum_m cos(2 pi k m / R) s_m - i sum_m sin(2 pi k m / R) d_m,
// X_{R-k} the same with +i.
template <int R>
__device__ __forceinline__ void odd_dft(float2* v) {
    constexpr int H = (R - 1) / 2;
    float2 s[H], d[H];
#pragma unroll
    for (int m = 1; m <= H; ++m) {
        s[m - 1] = cadd(v[m], v[R - m]);
        d[m - 1] = csub(v[m], v[R - m]);
    }
    const float2 x0 = v[0];
    float2 sum = x0;
#pragma unroll
    for (int m = 0; m < H; ++m) sum = cadd(sum, s[m]);
    v[0] = sum;
#pragma unroll
    for (int k = 1; k <= H; ++k) {
        vf2_t a = pk(x0), b = vf2_t{0.0f, 0.0f};
#pragma unroll
        for (int m = 1; m <= H; ++m) {
            const int j = (k * m) % R;
            const int jj = j <= H ? j : R - j;            // cos symmetric, sin antisymmetric
            const float c = OddC<R>::c(jj);
            const float sn = j <= H ? OddC<R>::s(jj) : -OddC<R>::s(jj);
            a = a + pk(s[m - 1]) * c;
            b = b + pk(d[m - 1]) * sn;
        }
        // X_k = a - i b = (a.x + b.y, a.y - b.x);  X_{R-k} = a + i b
        v[k] = cadd_i<false>(upk(a), upk(b));
        v[R - k] = cadd_i<true>(upk(a), upk(b));
    }
}

template <int R>
__device__ __forceinline__ void dft_fwd(float2* v) {
    if constexpr (R == 2 || R == 4 || R == 8)
        Dft<R, true>::run(v);
    else
        odd_dft<R>(v);
}

template <int T>
__device__ __forceinline__ void msync() {
    xsync<T>();
}

// Where a transform's points come from and go to.
//   MODE 0: complex rows (nout bins out, scaled; the inverse by conjugation).
//   MODE 4: real rows (imaginary zero), nout bins out.
//   MODE 5: real rows of length 2n through an n-point transform of
//           z[m] = x[2m] + i x[2m+1] and the split step (nout <= n + 1 bins).
//   MODE 1/2/3: STFT frames of a [ch][n] signal, frames (2j, 2j+1) of one
//           channel per complex transform (frame f starts at sample f*hop, zero
//           past the end, times the window: frame_gather's single rounded
//           product) -> |X| rows (1), complex rows (2) or |X|^2 for bins
//           0..n/2 (3).  Pairs never span channels.
struct MixIO {
    const void* in;
    float2* out;
    long long nout, in_dist, out_dist, rows;
    float scale;
    float isign;   // -1 for the inverse: conj(FFT(conj x))
    // STFT
    long long sig_n, ch_stride, frames, ppc, hop, out_ch_stride;
    const float* win;
    const float2* twn;   // MODE 5: W_n^k, k < n (n = 2 * the transform length)
    int var;   // A/B switch (VVHIP_MIX_VAR)
    int a16;   // STFT: output rows 16 B aligned (base and channel stride), for 16 B/lane row stores
};

template <int MODE>
struct Row {
    const float2* cin;
    const float *ra, *rb;   // real rows / frame starts (rb = ra when there is no second)
    const float* win;
    long long lima, limb;   // STFT: samples of each frame inside the signal
    bool has_b;
    float2 *ca, *cb;
    float *fa, *fb;

    __device__ __forceinline__ void open(const MixIO& io, long long f, int n) {
        if constexpr (MODE == 0) {
            cin = reinterpret_cast<const float2*>(io.in) + f * io.in_dist;
            ca = io.out + f * io.out_dist;
        } else if constexpr (MODE == 4 || MODE == 5) {
            ra = reinterpret_cast<const float*>(io.in) + f * io.in_dist;
            ca = io.out + f * io.out_dist;
        } else {
            const long long c = f / io.ppc, fra = 2 * (f - c * io.ppc);
            has_b = fra + 1 < io.frames;
            const long long st = fra * io.hop;
            ra = reinterpret_cast<const float*>(io.in) + c * io.ch_stride + st;
            rb = ra + io.hop;
            lima = io.sig_n - st;
            limb = has_b ? lima - io.hop : 0;
            win = io.win;
            const long long w = MODE == 3 ? n / 2 + 1 : n;
            const long long o = c * io.out_ch_stride + fra * w;
            ca = reinterpret_cast<float2*>(io.out) + o;
            cb = ca + w;
            fa = reinterpret_cast<float*>(io.out) + o;
            fb = fa + w;
        }
    }
    __device__ __forceinline__ float2 load(const MixIO& io, int e) const {
        if constexpr (MODE == 0) {   // the inverse conjugates (a sign, no branch)
            const float2 x = cin[e];
            return make_float2(x.x, x.y * io.isign);
        } else if constexpr (MODE == 4) {
            return make_float2(ra[e], 0.0f);
        } else if constexpr (MODE == 5) {   // z[m] = x[2m] + i x[2m+1]
            return make_float2(ra[2 * e], ra[2 * e + 1]);
        } else {
            // past the signal's end a load reads the window instead (always
            // mapped) and the value is zeroed: no branch around the loads
            const bool ia = e < lima, ib = e < limb;
            const float a = *(ia ? ra + e : win + e), b = *(ib ? rb + e : win + e);
            const float w = win[e];
            return make_float2((ia ? a : 0.0f) * w, (ib ? b : 0.0f) * w);
        }
    }
    // all outputs of the transform in buf (natural order), lane-contiguous
    template <int T>
    __device__ __forceinline__ void emit(const MixIO& io, const float2* buf, int t, int n) const {
        if constexpr (MODE == 0 || MODE == 4) {
            const float sx = io.scale, sy = io.scale * io.isign;
            for (int e = t; e < io.nout; e += T) {
                const float2 x = buf[e];
                // R2C (MODE 4): Im X[n/2] = 0 exactly, as the reference's R2C (fft_kiss.c:140-145)
                const bool nyq = MODE == 4 && 2 * e == n;
                ca[e] = make_float2(x.x * sx, nyq ? 0.0f : x.y * sy);
            }
        } else if constexpr (MODE == 5) {
            // real length 2n from the n-point transform of its even/odd pairs:
            // X[k] = (Z[k] + conj Z[n-k])/2 + W_2n^k (-i (Z[k] - conj Z[n-k])/2), k <= n
            for (int e = t; e < io.nout; e += T) {
                const float2 A = buf[e < n ? e : 0], B = cconj(buf[e == 0 || e == n ? 0 : n - e]);
                const float2 X = split_fwd(A, B, io.twn[e]);
                // Im X[n] (the row's Nyquist bin) = 0 exactly, as the reference (fft_kiss.c:140-145);
                // W_2n^n rounded from double is not exactly -1 + 0i
                ca[e] = make_float2(X.x * io.scale, e == n ? 0.0f : X.y * io.scale);
            }
        } else {
            const int lim = MODE == 3 ? n / 2 + 1 : n;
            const float h = 0.5f;
            for (int e = t; e < lim; e += T) {
                const float2 z = buf[e], m = buf[e == 0 ? 0 : n - e];
                const float2 xa = make_float2((z.x + m.x) * h, (z.y - m.y) * h);
                const float2 xb = make_float2((z.y + m.y) * h, (m.x - z.x) * h);
                if constexpr (MODE == 2) {
                    ca[e] = xa;
                    if (has_b) cb[e] = xb;
                } else if constexpr (MODE == 1) {
                    fa[e] = __builtin_amdgcn_sqrtf(__builtin_fmaf(xa.x, xa.x, xa.y * xa.y));
                    if (has_b) fb[e] = __builtin_amdgcn_sqrtf(__builtin_fmaf(xb.x, xb.x, xb.y * xb.y));
                } else {
                    fa[e] = __builtin_fmaf(xa.x, xa.x, xa.y * xa.y);
                    if (has_b) fb[e] = __builtin_fmaf(xb.x, xb.x, xb.y * xb.y);
                }
            }
        }
    }
};

// Copy a transform in (a plain strided loop measured 1.3x faster than loading
// all of a thread's points first: 400-point rows 0.26 vs 0.35 ms per GiB).
template <int T, int MODE>
__device__ __forceinline__ void mload(float2* buf, int t, int n, const MixIO& io, const Row<MODE>& row, bool act) {
    if (act)
        for (int e = t; e < n; e += T) buf[e] = row.load(io, e);
    msync<T>();
}

// One middle Stockham pass of radix R on the LDS-resident transform `buf`.
template <int R, int T>
__device__ __forceinline__ void mpass(float2* buf, const float2* tab, int t, int n, int Ns, int tstep, float rns,
                                      bool act) {
    constexpr int MAXB = (MIX_PTS + R - 1) / R;
    const int nb = n / R;
    float2 v[MAXB][R];
    if (act) {
#pragma unroll
        for (int b = 0; b < MAXB; ++b) {
            const int j = t + b * T;
            if (j < nb) {
#pragma unroll
                for (int r = 0; r < R; ++r) v[b][r] = buf[j + r * nb];
            }
        }
    }
    msync<T>();
    if (act) {
#pragma unroll
        for (int b = 0; b < MAXB; ++b) {
            const int j = t + b * T;
            if (j < nb) {
                int q = (int)((float)j * rns);
                int k = j - q * Ns;
                if (k >= Ns) { k -= Ns; ++q; }
                else if (k < 0) { k += Ns; --q; }
                if (Ns > 1) {
                    const int kt = k * tstep;
#pragma unroll
                    for (int r = 1; r < R; ++r) v[b][r] = cmul(v[b][r], tab[r * kt]);
                }
                dft_fwd<R>(v[b]);
                float2* dst = buf + q * Ns * R + k;
#pragma unroll
                for (int r = 0; r < R; ++r) dst[r * Ns] = v[b][r];
            }
        }
    }
    msync<T>();
}

#define VVH_MIX_RADIX_SWITCH(RAD, CALL) \
    switch (RAD) {                      \
        case 2: CALL(2); break;         \
        case 3: CALL(3); break;         \
        case 4: CALL(4); break;         \
        case 5: CALL(5); break;         \
        case 7: CALL(7); break;         \
        default: CALL(8); break;        \
    }

template <int T, int MODE>
__global__ void __launch_bounds__(256, LB)
k_fft_mixed(MixedPlan pl, MixIO io, long long batch, const float2* __restrict__ gtab) {
    constexpr int F = 256 / T;
    extern __shared__ float2 sm[];
    const int n = pl.n;
    float2* tab = sm;
    const int lt = threadIdx.x, slot = lt / T, t = lt % T;
    float2* buf = sm + n + slot * n;
    for (int i = lt; i < n; i += 256) tab[i] = gtab[i];
    __syncthreads();
    const long long stride = (long long)gridDim.x * F;
    for (long long f0 = (long long)blockIdx.x * F; f0 < batch; f0 += stride) {
        const long long f = f0 + slot;
        const bool act = f < batch;
        Row<MODE> row;
        if (act) row.open(io, f, n);
        mload<T, MODE>(buf, t, n, io, row, act);
        // one call site for every pass: the radix switch is instantiated once
        for (int p = 0; p < pl.np; ++p) {
            const int Ns = pl.ns[p], ts = pl.tstep[p];
            const float rn = pl.rns[p];
#define VVH_MM(RR) mpass<RR, T>(buf, tab, t, n, Ns, ts, rn, act)
            VVH_MIX_RADIX_SWITCH(pl.radix[p], VVH_MM)
#undef VVH_MM
        }
        if (act) row.template emit<T>(io, buf, t, n);
        msync<T>();   // the next transform's loads overwrite buf
    }
}

// ------------------------------------------------------------------------
// Four-step for 7-smooth n > 4096 (n = N1 * N2, both <= 4096): the columns
// pass takes N2 columns of length N1 (x[n1 * N2 + n2]), FFTs them and applies
// W_n^(n2 * k1) into an intermediate [N1][N2]; the rows pass FFTs each row
// k1 along n2 and stores X[k1 + N1 * k2].  The strided side of each pass is
// cooperative over the workgroup: its F transform slots own F adjacent
// columns (rows), so for one element index the workgroup touches F adjacent
// complex values (128 B at F = 16) instead of one per transform.
// ------------------------------------------------------------------------
struct FsIO {
    const void* in;
    float2* mid;
    float2* out;
    long long in_dist, out_dist, nout, n;
    int N1, N2, real_in;
    float scale, isign;
    const float2* twn;        // W_n two-level: lo[m & (2^lo_bits - 1)] * hi[m >> lo_bits]
    int lo_bits;
    long long groups_per_b;   // ceil(N2 / F) (columns) or ceil(N1 / F) (rows)
};

template <int T, int PASS>
__global__ void __launch_bounds__(256)
k_fft_mixed_fs(MixedPlan pl, FsIO io, long long groups, const float2* __restrict__ gtab) {
    constexpr int F = 256 / T;
    extern __shared__ float2 sm[];
    const int m = pl.n;   // this pass's FFT length: N1 (columns) or N2 (rows)
    float2* tab = sm;
    const int lt = threadIdx.x, slot = lt / T, t = lt % T;
    float2* buf = sm + m + slot * m;
    float2* bufs = sm + m;
    for (int i = lt; i < m; i += 256) tab[i] = gtab[i];
    // PASS 0: the two-level W_n table (2 sqrt(n) entries) in LDS after the
    // tile, so the twiddle of each stored element is two LDS reads instead of
    // two dependent global loads
    const int nlo = 1 << io.lo_bits;
    float2* const ltw = sm + (long long)m * (1 + F);
    if constexpr (PASS == 0) {
        const int ntw = nlo + (int)((io.n + nlo - 1) >> io.lo_bits);
        for (int i = lt; i < ntw; i += 256) ltw[i] = io.twn[i];
    }
    __syncthreads();
    const int N1 = io.N1, N2 = io.N2;
    const int width = PASS == 0 ? N2 : N1;   // columns or rows per transform of the batch
    for (long long g = blockIdx.x; g < groups; g += gridDim.x) {
        const long long b = g / io.groups_per_b;
        const int i0 = (int)(g - b * io.groups_per_b) * F;
        if constexpr (PASS == 0) {
            const float* rin = reinterpret_cast<const float*>(io.in) + b * io.in_dist;
            const float2* cin = reinterpret_cast<const float2*>(io.in) + b * io.in_dist;
            for (int idx = lt; idx < m * F; idx += 256) {
                const int e = idx / F, sl = idx % F, col = i0 + sl;
                if (col < N2) {
                    const long long o = (long long)e * N2 + col;
                    float2 x;
                    if (io.real_in) x = make_float2(rin[o], 0.0f);
                    else { x = cin[o]; x.y *= io.isign; }
                    bufs[sl * m + e] = x;
                }
            }
        } else {
            if (i0 + slot < N1) {
                const float2* src = io.mid + (b * N1 + i0 + slot) * (long long)N2;
                for (int e = t; e < m; e += T) buf[e] = src[e];
            }
        }
        __syncthreads();
        const bool act = i0 + slot < width;
        for (int p = 0; p < pl.np; ++p) {
            const int Ns = pl.ns[p], ts = pl.tstep[p];
            const float rn = pl.rns[p];
#define VVH_MM(RR) mpass<RR, T>(buf, tab, t, m, Ns, ts, rn, act)
            VVH_MIX_RADIX_SWITCH(pl.radix[p], VVH_MM)
#undef VVH_MM
        }
        __syncthreads();   // the stores read every slot's buffer
        if constexpr (PASS == 0) {
            float2* dst = io.mid + b * io.n;
            for (int idx = lt; idx < m * F; idx += 256) {
                const int k1 = idx / F, sl = idx % F, col = i0 + sl;
                if (col < N2) {
                    const int tw = col * k1;   // < n <= 2^24
                    const float2 w = cmul(ltw[tw & (nlo - 1)], ltw[nlo + (tw >> io.lo_bits)]);
                    dst[(long long)k1 * N2 + col] = cmul(bufs[sl * m + k1], w);
                }
            }
        } else {
            float2* dst = io.out + b * io.out_dist;
            const float sx = io.scale, sy = io.scale * io.isign;
            for (int idx = lt; idx < m * F; idx += 256) {
                const int k2 = idx / F, sl = idx % F, k1 = i0 + sl;
                const long long k = k1 + (long long)N1 * k2;
                if (k1 < N1 && k < io.nout) {
                    const float2 x = bufs[sl * m + k2];
                    dst[k] = make_float2(x.x * sx, x.y * sy);
                }
            }
        }
        __syncthreads();   // the next group's loads overwrite the buffers
    }
}

// ------------------------------------------------------------------------
// STFT frames of n = N1 * N2 (both <= 32) in registers: the speech lengths
// 400 = 20 x 20, 480 = 20 x 24, 960 = 30 x 32.  The generic kernel above runs
// a runtime radix plan through LDS with a barrier per pass and is bound by
// that (400-point STFT: 0.31 of the HBM roofline); here a transform (a frame
// pair, as MODE 1-3 above) is owned by max(N1, N2) lanes of one wave and
// takes two register passes with one LDS exchange:
//   pass 1, lane m2 < N2:  N1-point DFT of x[m1 N2 + m2] over m1, times W_n^(m2 k1)
//   pass 2, lane k1 < N1:  N2-point DFT over m2 -> X[k1 + N1 k2]
// The N-point DFTs are composed at compile time (R = A x B, constant
// twiddles), the W_n factors come from the n-entry table in LDS.  Results go
// back to LDS in natural order and the wave writes its pairs' rows as one
// contiguous run (rows a and b of consecutive pairs are adjacent).
// ------------------------------------------------------------------------
constexpr double cx_pi = 3.14159265358979323846264338327950288;
// cos / sin(2 pi j / R) in double at compile time (Taylor series on [-pi, pi])
constexpr double cx_cos2pi(int j, int R) {
    j %= R;
    double x = 2.0 * cx_pi * (double)j / (double)R;
    if (2 * j > R) x -= 2.0 * cx_pi;
    double term = 1.0, sum = 1.0;
    for (int i = 1; i < 24; ++i) {
        term *= -x * x / ((2.0 * i - 1.0) * (2.0 * i));
        sum += term;
    }
    return sum;
}
constexpr double cx_sin2pi(int j, int R) {
    j %= R;
    double x = 2.0 * cx_pi * (double)j / (double)R;
    if (2 * j > R) x -= 2.0 * cx_pi;
    double term = x, sum = x;
    for (int i = 1; i < 24; ++i) {
        term *= -x * x / ((2.0 * i) * (2.0 * i + 1.0));
        sum += term;
    }
    return sum;
}

// v * W_R^J (forward, W_R = exp(-2 pi i / R)); quarter and half turns exact
template <int J, int R>
__device__ __forceinline__ float2 twk(float2 v) {
    constexpr int m = J % R;
    if constexpr (m == 0) {
        return v;
    } else if constexpr (2 * m == R) {
        return upk(-pk(v));
    } else if constexpr (4 * m == R) {
        return cmul_mi(v);
    } else if constexpr (4 * m == 3 * R) {
        return cmul_pi(v);
    } else {
        constexpr float c = (float)cx_cos2pi(m, R), s = (float)-cx_sin2pi(m, R);
        return cmul(v, make_float2(c, s));
    }
}

template <int R>
struct RegFac {   // R = A * B for the composite DFT (A = 1: a base case)
    static constexpr bool BASE = R == 1 || R == 2 || R == 3 || R == 4 || R == 5 || R == 7 || R == 8 || R == 16;
    static constexpr int A = BASE ? 1 : R % 8 == 0 ? 8 : R % 4 == 0 ? 4 : R % 2 == 0 ? 2 : R % 3 == 0 ? 3 : R % 5 == 0 ? 5 : 7;
    static constexpr int B = BASE ? R : R / A;
};

// forward DFT of length R on registers, natural order in and out
template <int R>
__device__ __forceinline__ void reg_dft(float2* v) {
    if constexpr (RegFac<R>::BASE) {
        if constexpr (R == 1) {
        } else if constexpr (R == 2 || R == 4 || R == 8 || R == 16) {
            Dft<R, true>::run(v);
        } else {
            odd_dft<R>(v);
        }
    } else {
        constexpr int A = RegFac<R>::A, B = RegFac<R>::B;
        float2 y[A][B];
        static_for<0, B>([&](auto m2c) {
            constexpr int m2 = decltype(m2c)::value;
            float2 col[A];
#pragma unroll
            for (int m1 = 0; m1 < A; ++m1) col[m1] = v[m1 * B + m2];
            reg_dft<A>(col);
            static_for<0, A>([&](auto k1c) {
                constexpr int k1 = decltype(k1c)::value;
                y[k1][m2] = twk<k1 * m2, R>(col[k1]);
            });
        });
#pragma unroll
        for (int k1 = 0; k1 < A; ++k1) {
            reg_dft<B>(y[k1]);
#pragma unroll
            for (int k2 = 0; k2 < B; ++k2) v[k1 + A * k2] = y[k1][k2];
        }
    }
}

template <int N1, int N2, int MODE = 0>
struct Sq {
    static constexpr int N = N1 * N2;
    static constexpr int TT = N1 > N2 ? N1 : N2;   // lanes per transform
    static constexpr int TPW = 64 / TT;            // transforms per wave
    static constexpr int P2 = N2 + 1;              // padded pass-1 row (k1 rows of N2)
    // float2 per transform, even: 16 B aligned transform buffers (the staged row flush reads float4s)
    static constexpr int LT = ((N1 * P2 > N ? N1 * P2 : N) + 1) / 2 * 2;
    // + the W_n table and the window (MODE 5: W_2n^k, k <= n, for the split step)
    static constexpr int LDS = 4 * TPW * LT + N + (MODE == 5 ? N + 1 : N / 2);
    // workgroups per CU the LDS allows, at most 3 (<= 168 VGPRs), or 4 when
    // both factors are <= 20 (the transform's registers then fit 128 VGPRs
    // without spills: 320 = 16 x 20 measured 3.4 % faster at 4 than at 3; 480 =
    // 20 x 24 spills at 128 and measured 21 % slower, profiles/r03_kbench_sq_lb4.jsonl).
    // Latency-bound, so occupancy matters.
    static constexpr int FIT = (160 * 1024) / (8 * LDS);
    static constexpr int CAP = (N1 <= 20 && N2 <= 20) ? 4 : 3;
    static constexpr int LB = FIT < CAP ? (FIT < 1 ? 1 : FIT) : CAP;
    // magnitude rows (MODE 1) are staged in LDS and flushed as one contiguous
    // run per pair: 16 B/lane when the row length is a multiple of 4 floats
    // (and the output 16 B aligned), 4 B/lane otherwise
    // (not for magnitude rows of 600 = 20 x 30 / 640 = 20 x 32: at 3 waves per
    // SIMD the held magnitudes make the 30/32-point pass spill, 1.16-1.34x
    // slower, profiles/r03_ab_sq_stage_pow.jsonl -- those keep the symmetric emit)
    static constexpr bool STG = MODE == 3 || (MODE == 1 && !(LB == 3 && (N1 > 24 || N2 > 24)));
    static constexpr bool ST16 = STG && MODE == 1 && N % 4 == 0;
};

// MODE 0 c2c rows (`pairs` = rows), MODE 5 real rows of 2n (even/odd pairs
// + split step, as k_fft_mixed); STFT frame pairs: MODE 1 |X| rows, 2 complex
// rows, 3 |X|^2 for bins 0..n/2 (as k_fft_mixed).  A wave reads its rows whole
// before it writes them, so in == out is safe.
template <int N1, int N2, int MODE>
__global__ void __launch_bounds__(256, (Sq<N1, N2, MODE>::LB)) k_stft_sq(MixIO io, long long pairs, const float2* __restrict__ gtab) {
    using S = Sq<N1, N2, MODE>;
    constexpr int n = S::N, TT = S::TT, TPW = S::TPW, P2 = S::P2, LT = S::LT;
    constexpr int W = MODE == 3 ? n / 2 + 1 : n;   // bins per row
    __shared__ __attribute__((aligned(16))) float2 sm[S::LDS];
    float2* const tab = sm + 4 * TPW * LT;
    float* const lwin = reinterpret_cast<float*>(tab + n);
    float2* const ltw = tab + n;   // MODE 5 (in the window's place)
    // pass 1's twiddles W_n^(k1 t) stored [k1][t] (t < N2): for one k1 the lanes
    // read consecutive entries (tab[k1 t] had k1-strided, bank-conflicting reads)
    for (int i = threadIdx.x; i < n; i += 256) {
        const int k1 = i / N2, tt = i - k1 * N2;
        tab[i] = gtab[k1 * tt];
        if constexpr (MODE != 0 && MODE != 5) lwin[i] = io.win[i];
    }
    if constexpr (MODE == 5) {   // the split step's W_2n^k from LDS, not a dependent global load per bin
        for (int i = threadIdx.x; i <= n; i += 256) ltw[i] = io.twn[i];
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int slot = lane / TT, t = lane - slot * TT;
    const bool lane_ok = slot < TPW;
    float2* const wbuf = sm + wave * TPW * LT;
    float2* const L = wbuf + (lane_ok ? slot : 0) * LT;
    __syncthreads();
    const long long step = (long long)gridDim.x * 4 * TPW;
    for (long long g = ((long long)blockIdx.x * 4 + wave) * TPW; g < pairs; g += step) {
        // pass 1: lane t < N2 of slot `slot` on pair g + slot
        {
            const long long q = g + slot;
            if ((MODE == 0 || MODE == 5) && lane_ok && q < pairs && t < N2) {
                float2 v[N1];
                if constexpr (MODE == 0) {   // complex row q (the inverse by conjugation)
                    const float2* x = reinterpret_cast<const float2*>(io.in) + q * io.in_dist + t;
#pragma unroll
                    for (int m1 = 0; m1 < N1; ++m1) {
                        const float2 a = x[m1 * N2];
                        v[m1] = make_float2(a.x, a.y * io.isign);
                    }
                } else {   // real row q of length 2n: z[m] = x[2m] + i x[2m+1]
                    const float* x = reinterpret_cast<const float*>(io.in) + q * io.in_dist + 2 * t;
#pragma unroll
                    for (int m1 = 0; m1 < N1; ++m1) v[m1] = make_float2(x[2 * m1 * N2], x[2 * m1 * N2 + 1]);
                }
                reg_dft<N1>(v);
#pragma unroll
                for (int k1 = 0; k1 < N1; ++k1) L[k1 * P2 + t] = k1 == 0 ? v[0] : cmul(v[k1], tab[k1 * N2 + t]);
            } else if (MODE != 0 && MODE != 5 && lane_ok && q < pairs && t < N2) {
                const long long c = q / io.ppc, fra = 2 * (q - c * io.ppc);
                const long long st = fra * io.hop;
                const float* ra = reinterpret_cast<const float*>(io.in) + c * io.ch_stride + st;
                const float* rb = ra + io.hop;
                const long long lima = io.sig_n - st;
                const long long limb = fra + 1 < io.frames ? lima - io.hop : 0;
                float2 v[N1];
                if (limb >= n) {   // both frames inside the signal: base + immediate loads
                    const float* pa = ra + t;
                    const float* pb = rb + t;
#pragma unroll
                    for (int m1 = 0; m1 < N1; ++m1) {
                        const float w = lwin[m1 * N2 + t];
                        v[m1] = make_float2(pa[m1 * N2] * w, pb[m1 * N2] * w);
                    }
                } else {
#pragma unroll
                    for (int m1 = 0; m1 < N1; ++m1) {
                        const int s = m1 * N2 + t;
                        // past the end a load reads the window (always mapped), zeroed
                        const bool ia = s < lima, ib = s < limb;
                        const float a = *(ia ? ra + s : io.win + s), b = *(ib ? rb + s : io.win + s);
                        const float w = lwin[s];
                        v[m1] = make_float2((ia ? a : 0.0f) * w, (ib ? b : 0.0f) * w);
                    }
                }
                reg_dft<N1>(v);
#pragma unroll
                for (int k1 = 0; k1 < N1; ++k1) L[k1 * P2 + t] = k1 == 0 ? v[0] : cmul(v[k1], tab[k1 * N2 + t]);
            }
        }
        xsync<64>();
        // pass 2: lane t < N1 on row k1 = t
        if (lane_ok && g + slot < pairs && t < N1) {
            float2 u[N2];
#pragma unroll
            for (int m2 = 0; m2 < N2; ++m2) u[m2] = L[t * P2 + m2];
            reg_dft<N2>(u);
#pragma unroll
            for (int k2 = 0; k2 < N2; ++k2) L[t + N1 * k2] = u[k2];
        }
        xsync<64>();
        if constexpr (MODE == 5) {   // split step: X[k] = (Z[k] + conj Z[n-k])/2 + W_2n^k (-i (Z[k] - conj Z[n-k])/2)
#pragma unroll
            for (int s = 0; s < TPW; ++s) {
                const long long q = g + s;
                if (q >= pairs) break;   // wave-uniform
                const float2* X = wbuf + s * LT;
                float2* y = io.out + q * io.out_dist;
                for (int e = lane; e < io.nout; e += 64) {
                    const float2 A = X[e < n ? e : 0], B = cconj(X[e == 0 || e == n ? 0 : n - e]);
                    const float2 Y = split_fwd(A, B, ltw[e]);
                    y[e] = make_float2(Y.x * io.scale, e == n ? 0.0f : Y.y * io.scale);   // Im Nyquist = 0
                }
            }
        }
        if constexpr (MODE == 0) {   // the wave's rows, scaled (and conjugated back for the inverse)
            const float sx = io.scale, sy = io.scale * io.isign;
#pragma unroll
            for (int s = 0; s < TPW; ++s) {
                const long long q = g + s;
                if (q >= pairs) break;   // wave-uniform
                const float2* X = wbuf + s * LT;
                float2* y = io.out + q * io.out_dist;
                for (int e = lane; e < io.nout; e += 64) {
                    const float2 z = X[e];
                    y[e] = make_float2(z.x * sx, z.y * sy);
                }
            }
        }
        // Magnitude / complex rows of real frames from their conjugate symmetry:
        // bins e and n - e of both rows from one read of Z[e], Z[n - e] and one
        // split/magnitude (|X[n-e]| = |X[e]|, X[n-e] = conj X[e], bit-identical
        // to computing bin n - e on its own).  n < 900: 12-18 % faster than
        // emitting each row bin by bin (480-point rows 6.00 -> 4.92 ms for 32 ch x
        // 10 min at 48 kHz, profiles/r03_kbench_sq_sym.jsonl); n >= 900 keeps the
        // per-bin emit of both rows below (2 % faster there).
        if constexpr (S::STG) {
            // Magnitude (and power) rows staged in the transform's own (now consumed) LDS
            // buffer and written as 16 B/lane stores of the pair's 2W-float run
            // (4 B/lane plain stores for power rows and rows not a multiple of 4 floats):
            // |X| of bins e and n - e of both rows from one read of Z[e], Z[n-e]
            // (conjugate symmetry), held in registers until every read is done.
            // 12-18 % faster than the 4 B/lane stores of the symmetric emit below
            // at 400 / 480 / 720 / 900 / 960 (profiles/r03_kbench_sq_stage.jsonl,
            // r03_ab_sq_stage_all.jsonl).
            constexpr int IT = (n / 2 + 1 + 63) / 64;
#pragma unroll
            for (int s = 0; s < TPW; ++s) {
                const long long q = g + s;
                if (q >= pairs) break;   // wave-uniform
                float* const X = reinterpret_cast<float*>(wbuf + s * LT);
                const float2* const Z = wbuf + s * LT;
                float ma[IT], mb[IT];
#pragma unroll
                for (int i = 0; i < IT; ++i) {
                    const int e = lane + 64 * i;
                    const int ec = 2 * e <= n ? e : 0;
                    const float2 z = Z[ec], m = Z[ec == 0 ? 0 : n - ec];
                    const float h = 0.5f;
                    const float2 xa = make_float2((z.x + m.x) * h, (z.y - m.y) * h);
                    const float2 xb = make_float2((z.y + m.y) * h, (m.x - z.x) * h);
                    ma[i] = __builtin_fmaf(xa.x, xa.x, xa.y * xa.y);
                    mb[i] = __builtin_fmaf(xb.x, xb.x, xb.y * xb.y);
                    if constexpr (MODE == 1) {
                        ma[i] = __builtin_amdgcn_sqrtf(ma[i]);
                        mb[i] = __builtin_amdgcn_sqrtf(mb[i]);
                    }
                }
                xsync<64>();   // every read of Z before the rows overwrite it
#pragma unroll
                for (int i = 0; i < IT; ++i) {
                    const int e = lane + 64 * i;
                    if (2 * e <= n) {
                        X[e] = ma[i];
                        X[W + e] = mb[i];
                        if (MODE == 1 && e != 0 && 2 * e != n) {   // power rows (MODE 3) end at bin n/2
                            X[n - e] = ma[i];
                            X[W + n - e] = mb[i];
                        }
                    }
                }
                xsync<64>();
                const long long c = q / io.ppc, fra = 2 * (q - c * io.ppc);
                const int lim = fra + 1 < io.frames ? 2 * W : W;   // floats of the run (row b may not exist)
                float* const fo = reinterpret_cast<float*>(io.out) + c * io.out_ch_stride + fra * W;
                if (S::ST16 && io.a16) {
                    const vf4_t* const X4 = reinterpret_cast<const vf4_t*>(X);
#pragma unroll
                    for (int o = lane; o < (2 * W) / 4; o += 64)
                        if (4 * o < lim) __builtin_nontemporal_store(X4[o], reinterpret_cast<vf4_t*>(fo) + o);
                } else {   // plain stores: runs that are not whole lines merge in L2
                    for (int o = lane; o < lim; o += 64) fo[o] = X[o];
                }
            }
        } else if constexpr ((MODE == 1 || MODE == 2) && n < 900) {
#pragma unroll
            for (int s = 0; s < TPW; ++s) {
                const long long q = g + s;
                if (q >= pairs) break;   // wave-uniform
                const long long c = q / io.ppc, fra = 2 * (q - c * io.ppc);
                const bool hbq = fra + 1 < io.frames;
                const long long bs = c * io.out_ch_stride + fra * W;
                const float2* X = wbuf + s * LT;
                for (int e = lane; 2 * e <= n; e += 64) {
                    const float2 z = X[e], m = X[e == 0 ? 0 : n - e];
                    const float h = 0.5f;
                    const float2 xa = make_float2((z.x + m.x) * h, (z.y - m.y) * h);
                    const float2 xb = make_float2((z.y + m.y) * h, (m.x - z.x) * h);
                    const bool mir = e != 0 && 2 * e != n;
                    if constexpr (MODE == 1) {
                        float* fo = reinterpret_cast<float*>(io.out) + bs;
                        const float ma = __builtin_amdgcn_sqrtf(__builtin_fmaf(xa.x, xa.x, xa.y * xa.y));
                        const float mb = __builtin_amdgcn_sqrtf(__builtin_fmaf(xb.x, xb.x, xb.y * xb.y));
                        fo[e] = ma;
                        if (mir) fo[n - e] = ma;
                        if (hbq) {
                            fo[W + e] = mb;
                            if (mir) fo[W + n - e] = mb;
                        }
                    } else {
                        float2* co = io.out + bs;
                        co[e] = xa;
                        if (mir) co[n - e] = cconj(xa);
                        if (hbq) {
                            co[W + e] = xb;
                            if (mir) co[W + n - e] = cconj(xb);
                        }
                    }
                }
            }
        } else {
        // rows a and b of each of the wave's pairs: 2W adjacent bins, the whole wave on each
#pragma unroll
        for (int s = 0; s < (MODE == 0 || MODE == 5 ? 0 : TPW); ++s) {
            const long long q = g + s;
            if (q >= pairs) break;   // wave-uniform
            const long long c = q / io.ppc, fra = 2 * (q - c * io.ppc);
            if constexpr (n >= 900) {   // both rows per read of Z[e], Z[n-e]: 960-pt 5.83 -> 4.57 ms;
                                        // 400 / 480 measured 1.3-1.4x slower that way (profiles/r02_ab_sq_emit.jsonl)
                const bool hbq = fra + 1 < io.frames;
                const long long bs = c * io.out_ch_stride + fra * W;
                const float2* X = wbuf + s * LT;
                // bin e of both rows from one read of Z[e] and Z[n - e]
#pragma unroll 4
                for (int e = lane; e < W; e += 64) {
                    const float2 z = X[e], m = X[e == 0 ? 0 : n - e];
                    const float h = 0.5f;
                    const float2 xa = make_float2((z.x + m.x) * h, (z.y - m.y) * h);
                    const float2 xb = make_float2((z.y + m.y) * h, (m.x - z.x) * h);
                    if constexpr (MODE == 2) {
                        io.out[bs + e] = xa;
                        if (hbq) io.out[bs + W + e] = xb;
                    } else {
                        float* fo = reinterpret_cast<float*>(io.out) + bs + e;
                        if constexpr (MODE == 1) {
                            fo[0] = __builtin_amdgcn_sqrtf(__builtin_fmaf(xa.x, xa.x, xa.y * xa.y));
                            if (hbq) fo[W] = __builtin_amdgcn_sqrtf(__builtin_fmaf(xb.x, xb.x, xb.y * xb.y));
                        } else {
                            fo[0] = __builtin_fmaf(xa.x, xa.x, xa.y * xa.y);
                            if (hbq) fo[W] = __builtin_fmaf(xb.x, xb.x, xb.y * xb.y);
                        }
                    }
                }
            } else {
                const int lim = fra + 1 < io.frames ? 2 * W : W;
                const long long bs = c * io.out_ch_stride + fra * W;
                const float2* X = wbuf + s * LT;
#pragma unroll 4
                for (int o = lane; o < 2 * W; o += 64) {
                    if (o < lim) {
                        const bool isb = o >= W;
                        const int e = isb ? o - W : o;
                        const float2 z = X[e], m = X[e == 0 ? 0 : n - e];
                        const float h = 0.5f;
                        const float2 x = isb ? make_float2((z.y + m.y) * h, (m.x - z.x) * h)
                                             : make_float2((z.x + m.x) * h, (z.y - m.y) * h);
                        if constexpr (MODE == 2) {
                            io.out[bs + o] = x;
                        } else {
                            float* fo = reinterpret_cast<float*>(io.out) + bs + o;
                            if constexpr (MODE == 1) *fo = __builtin_amdgcn_sqrtf(__builtin_fmaf(x.x, x.x, x.y * x.y));
                            else *fo = __builtin_fmaf(x.x, x.x, x.y * x.y);
                        }
                    }
                }
            }
        }
        }
        xsync<64>();   // the next group's pass 1 overwrites the buffers
    }
}

template <int N1, int N2, int MODE>
hipError_t run_stft_sq(const MixIO& io, long long pairs, hipStream_t s) {
    const float2* tab = twiddle_table(N1 * N2);
    if (!tab) return hipErrorOutOfMemory;
    constexpr int TPW = Sq<N1, N2, MODE>::TPW;
    const long long work = (pairs + 4 * TPW - 1) / (4 * TPW);
    // batched C2C (MODE 0) and R2C (MODE 5) rows: a non-persistent grid, each
    // wave's transforms once -- -4..-11 % (C2C 320..960) and -7..-14 % (R2C 400 /
    // 480 / 960) on the same buffers, bit-identical; the STFT modes measured 6-10 %
    // slower that way and stay persistent (profiles/r05_ab2_analytic_mixed_grid.jsonl).
    // Knob MIX_TPW = 0 / 1 forces the persistent / non-persistent grid (A/B)
    const bool once = knob(KNOB_MIX_TPW, (MODE == 0 || MODE == 5) ? 1 : 0) == 1;
    const int grid = once ? (int)(work < (1LL << 30) ? work : (1LL << 30))
                          : persistent_grid((const void*)k_stft_sq<N1, N2, MODE>, 256, 0, work);
    hipLaunchKernelGGL((k_stft_sq<N1, N2, MODE>), dim3(grid), dim3(256), 0, s, io, pairs, tab);
    return hipGetLastError();
}

// Lengths the register kernel takes (n, N1, N2; N1, N2 <= 32): speech and
// audio frames of 20 / 25 / 30 / 60 ms at 16, 32, 44.1 and 48 kHz
#define VVH_SQ_LENGTHS(X) \
    X(320, 16, 20) X(400, 20, 20) X(441, 21, 21) X(480, 20, 24) X(600, 20, 30) X(640, 20, 32) \
    X(720, 24, 30) X(800, 25, 32) X(900, 30, 30) X(960, 30, 32)
// half lengths of the real (R2C) rows: the list plus 200 and 240 (R2C at 400 / 480)
#define VVH_SQ_HALF_LENGTHS(X) X(200, 10, 20) X(240, 12, 20) VVH_SQ_LENGTHS(X)

bool sq_enabled() {
    return knob(KNOB_STFT_SQ, 1) != 0;   // 0: the generic kernel (A/B)
}

// c2c rows of n = N1 * N2 through the register kernel
bool sq_c2c(long long n, const MixIO& io, long long batch, hipStream_t s, hipError_t* e) {
    if (!sq_enabled()) return false;
    switch (n) {
#define VVH_SQ_C2C(L, A, B) \
    case L: *e = run_stft_sq<A, B, 0>(io, batch, s); return true;
        VVH_SQ_LENGTHS(VVH_SQ_C2C)
#undef VVH_SQ_C2C
        default: return false;
    }
}

// real rows of n2 = 2 x (N1 * N2) through the register kernel (MODE 5)
bool sq_r2c(long long n2, const MixIO& io, long long batch, hipStream_t s, hipError_t* e) {
    if (!sq_enabled() || n2 % 2) return false;
    switch (n2 / 2) {
#define VVH_SQ_R2C(L, A, B) \
    case L: *e = run_stft_sq<A, B, 5>(io, batch, s); return true;
        VVH_SQ_HALF_LENGTHS(VVH_SQ_R2C)
#undef VVH_SQ_R2C
        default: return false;
    }
}

template <int N1, int N2>
hipError_t run_stft_sq_kind(int kind, const MixIO& io, long long pairs, hipStream_t s) {
    switch (kind) {
        case 0: return run_stft_sq<N1, N2, 1>(io, pairs, s);
        case 1: return run_stft_sq<N1, N2, 2>(io, pairs, s);
        default: return run_stft_sq<N1, N2, 3>(io, pairs, s);
    }
}

// radices largest first: 8s, then a 4 or 2, then 7, 5, 3
bool make_plan(long long n, MixedPlan* pl) {
    if (n < 2 || n > MIX_MAXN) return false;
    int m = (int)n, np = 0;
    int rad[32];
    while (m % 8 == 0) { rad[np++] = 8; m /= 8; }
    if (m % 4 == 0) { rad[np++] = 4; m /= 4; }
    if (m % 2 == 0) { rad[np++] = 2; m /= 2; }
    for (int p : {7, 5, 3})
        while (m % p == 0) { rad[np++] = p; m /= p; }
    if (m != 1 || np > MIX_MAXP) return false;
    pl->n = (int)n;
    pl->np = np;
    int ns = 1;
    for (int p = 0; p < np; ++p) {
        pl->radix[p] = rad[p];
        pl->ns[p] = ns;
        pl->tstep[p] = (int)n / (ns * rad[p]);
        pl->rns[p] = 1.0f / (float)ns;
        ns *= rad[p];
    }
    return true;
}

int mixed_threads(long long n) { return n <= 256 ? 16 : n <= 512 ? 32 : n <= 1024 ? 64 : 256; }

template <int T, int MODE>
hipError_t run_mixed_t(const MixedPlan& pl, const MixIO& io, long long batch, hipStream_t s) {
    const float2* tab = twiddle_table(pl.n);
    if (!tab) return hipErrorOutOfMemory;
    constexpr int F = 256 / T;
    const size_t lds = sizeof(float2) * (size_t)pl.n * (1 + F);
    const long long work = (batch + F - 1) / F;
    // knob MIX_TPW = 1: a non-persistent grid (A/B; 1000-4000-point C2C measured
    // 8-22 % slower that way, profiles/r05_ab2_analytic_mixed_grid.jsonl)
    const int grid = knob(KNOB_MIX_TPW, 0) == 1 ? (int)(work < (1LL << 30) ? work : (1LL << 30))
                                                 : persistent_grid((const void*)k_fft_mixed<T, MODE>, 256, lds, work);
    hipLaunchKernelGGL((k_fft_mixed<T, MODE>), dim3(grid), dim3(256), lds, s, pl, io, batch, tab);
    return hipGetLastError();
}

template <int MODE>
hipError_t run_mixed(const MixedPlan& pl, MixIO io, long long batch, hipStream_t s) {
    io.var = (int)knob(KNOB_MIX_VAR, 0);
    switch (mixed_threads(pl.n)) {
        case 16: return run_mixed_t<16, MODE>(pl, io, batch, s);
        case 32: return run_mixed_t<32, MODE>(pl, io, batch, s);
        case 64: return run_mixed_t<64, MODE>(pl, io, batch, s);
        default: return run_mixed_t<256, MODE>(pl, io, batch, s);
    }
}

template <int T, int PASS>
hipError_t run_fs_t(const MixedPlan& pl, const FsIO& io0, long long batch, hipStream_t s) {
    const float2* tab = twiddle_table(pl.n);
    if (!tab) return hipErrorOutOfMemory;
    constexpr int F = 256 / T;
    FsIO io = io0;
    io.groups_per_b = ((PASS == 0 ? io.N2 : io.N1) + F - 1) / F;
    const long long groups = batch * io.groups_per_b;
    const long long nlo = 1LL << io.lo_bits;
    const size_t lds = sizeof(float2) * ((size_t)pl.n * (1 + F) + (PASS == 0 ? (size_t)(nlo + ((io.n + nlo - 1) >> io.lo_bits)) : 0));
    const int grid = persistent_grid((const void*)k_fft_mixed_fs<T, PASS>, 256, lds, groups);
    hipLaunchKernelGGL((k_fft_mixed_fs<T, PASS>), dim3(grid), dim3(256), lds, s, pl, io, groups, tab);
    return hipGetLastError();
}

template <int PASS>
hipError_t run_fs(const MixedPlan& pl, const FsIO& io, long long batch, hipStream_t s) {
    switch (mixed_threads(pl.n)) {
        case 16: return run_fs_t<16, PASS>(pl, io, batch, s);
        case 32: return run_fs_t<32, PASS>(pl, io, batch, s);
        case 64: return run_fs_t<64, PASS>(pl, io, batch, s);
        default: return run_fs_t<256, PASS>(pl, io, batch, s);
    }
}

// n = N1 * N2 with both factors plannable, max(N1, N2) smallest (N1 <= N2)
bool fs_split(long long n, int* n1, int* n2) {
    if (n <= MIX_MAXN || n > (long long)MIX_MAXN * MIX_MAXN) return false;
    MixedPlan pl;
    int best = 0;
    for (long long a = 2; a * a <= n; ++a) {
        if (n % a || !make_plan(a, &pl) || !make_plan(n / a, &pl)) continue;
        best = (int)a;   // ascending: the last admissible a is the most balanced
    }
    if (!best) return false;
    *n1 = best;
    *n2 = (int)(n / best);
    return true;
}

}  // namespace

bool mixed_supported(long long n) {
    if ((n & (n - 1)) == 0) return false;
    MixedPlan pl;
    int n1, n2;
    return make_plan(n, &pl) || fs_split(n, &n1, &n2);
}

// the fused STFT (launch_stft_mixed) needs a single-pass plan: n <= MIX_MAXN.
// Larger smooth nfft take the generic gather + FFT path (which uses the four-step).
bool stft_mixed_supported(long long n) {
    if ((n & (n - 1)) == 0) return false;
    MixedPlan pl;
    return make_plan(n, &pl);
}

// four-step over an intermediate of at most VVHIP_MIX_CHUNK_MB (default: the
// whole batch) per chunk of transforms
static hipError_t launch_fft_mixed_fs(long long n, int fwd, const void* in, int real_in, float2* out,
                                      long long nout, long long batch, long long in_dist, long long out_dist,
                                      float scale, hipStream_t s) {
    int n1, n2;
    MixedPlan p1, p2;
    if (!fs_split(n, &n1, &n2) || !make_plan(n1, &p1) || !make_plan(n2, &p2)) return hipErrorInvalidValue;
    int lo_bits = 0;
    const float2* twn = twiddle_split(n, &lo_bits);   // sqrt(n)-sized, not an n-entry table
    if (!twn) return hipErrorOutOfMemory;
    const long long cmb = knob(KNOB_MIX_CHUNK_MB, 0);
    long long chunk = cmb > 0 ? (cmb << 20) / (8 * n) : batch;
    if (chunk < 1) chunk = 1;
    if (chunk > batch) chunk = batch;
    float2* mid = nullptr;
    hipError_t e = hipMallocAsync((void**)&mid, sizeof(float2) * (size_t)n * (size_t)chunk, s);
    if (e != hipSuccess) return e;
    FsIO io{};
    io.mid = mid;
    io.nout = nout;
    io.n = n;
    io.N1 = n1;
    io.N2 = n2;
    io.real_in = real_in;
    io.scale = scale;
    io.isign = fwd ? 1.0f : -1.0f;
    io.twn = twn;
    io.lo_bits = lo_bits;
    io.in_dist = in_dist;
    io.out_dist = out_dist;
    for (long long c = 0; c < batch && e == hipSuccess; c += chunk) {
        const long long nb = batch - c < chunk ? batch - c : chunk;
        io.in = real_in ? (const void*)(reinterpret_cast<const float*>(in) + c * in_dist)
                        : (const void*)(reinterpret_cast<const float2*>(in) + c * in_dist);
        io.out = out + c * out_dist;
        e = run_fs<0>(p1, io, nb, s);
        if (e == hipSuccess) e = run_fs<1>(p2, io, nb, s);
    }
    (void)hipFreeAsync(mid, s);
    return e;
}

hipError_t launch_fft_mixed(long long n, int fwd, const void* in, int real_in, float2* out, long long nout,
                            long long batch, long long in_dist, long long out_dist, float scale, hipStream_t s) {
    if (batch <= 0) return hipSuccess;
    MixedPlan pl;
    if (!make_plan(n, &pl))
        return launch_fft_mixed_fs(n, fwd, in, real_in, out, nout, batch, in_dist, out_dist, scale, s);
    MixIO io{};
    io.in = in;
    io.out = out;
    io.nout = nout;
    io.in_dist = in_dist;
    io.out_dist = out_dist;
    io.rows = batch;
    io.scale = scale;
    io.isign = fwd ? 1.0f : -1.0f;
    // Real rows are not paired across the batch (unlike STFT frames), so a row's
    // result does not depend on the batch it came in.  Even n with a plannable
    // n/2 (forward, the R2C case): the n/2-point transform of the row's
    // even/odd pairs and the split step (MODE 5, half the FFT work); otherwise
    // the row with imaginary part zero (MODE 4).
    if (real_in) {
        MixedPlan ph;
        // knob MIX_R2C_FULL = 1: MODE 4 for even n too (A/B)
        const bool half = fwd && n % 2 == 0 && nout <= n / 2 + 1 && knob(KNOB_MIX_R2C_FULL, 0) != 1 && make_plan(n / 2, &ph);
        if (half) {
            io.twn = twiddle_table((int)n);
            if (!io.twn) return hipErrorOutOfMemory;
            hipError_t e = hipSuccess;
            if (sq_r2c(n, io, batch, s, &e)) return e;
            return run_mixed<5>(ph, io, batch, s);
        }
        return run_mixed<4>(pl, io, batch, s);
    }
    hipError_t e = hipSuccess;
    if (sq_c2c(n, io, batch, s, &e)) return e;
    return run_mixed<0>(pl, io, batch, s);
}

hipError_t launch_stft_mixed(long long nfft, long long hop, int kind, const float* sig, long long n, long long nch,
                             long long ch_stride, long long frames, const float* win, void* out,
                             long long out_ch_stride, hipStream_t s) {
    MixedPlan pl;
    if (!make_plan(nfft, &pl) || kind < 0 || kind > 2) return hipErrorInvalidValue;
    const long long ppc = (frames + 1) / 2;
    const long long batch = nch * ppc;
    if (batch <= 0) return hipSuccess;
    MixIO io{};
    io.in = sig;
    io.out = reinterpret_cast<float2*>(out);
    io.sig_n = n;
    io.ch_stride = ch_stride;
    io.frames = frames;
    io.ppc = ppc;
    io.hop = hop;
    io.out_ch_stride = out_ch_stride;
    io.win = win;
    io.a16 = ((uintptr_t)out & 15) == 0 && (out_ch_stride & 3) == 0;
    // speech lengths: the two-pass register kernel (VVHIP_STFT_SQ=0: the generic one, A/B)
    if (sq_enabled()) {
        switch (nfft) {
#define VVH_SQ_STFT(L, A, B) \
    case L: return run_stft_sq_kind<A, B>(kind, io, batch, s);
            VVH_SQ_LENGTHS(VVH_SQ_STFT)
#undef VVH_SQ_STFT
            default: break;
        }
    }
    switch (kind) {
        case 0: return run_mixed<1>(pl, io, batch, s);
        case 1: return run_mixed<2>(pl, io, batch, s);
        default: return run_mixed<3>(pl, io, batch, s);
    }
}

}  // namespace vvh
