// large_fft.hip -- power-of-two C2C transforms longer than one workgroup's
// register/LDS FFT (n > 4096, up to 2^24), and Bluestein for other lengths.
//
// The reference computes every power of two with one radix-2 DIT
// (src/spectral/fft_kiss.c:27-74).  Here n = N1*N2 and
//   X[k1 + N1*k2] = sum_n2 W_N2^(n2 k2) * W_n^(n2 k1) * sum_n1 x[n1 N2 + n2] W_N1^(n1 k1)
//
// n <= 2^20 (N1, N2 <= 1024): TWO HBM passes, no transposes.
//   columns: a workgroup owns G = 16 adjacent columns n2 of [N1][N2]; lane l
//            works on column l % G, so every load x[n1][n2..n2+15] and every
//            store Y[k1][n2..n2+15] is a 128-B line.  N1-pt FFT down each
//            column, times W_n^(n2 k1), stored in place of the column.
//   rows:    a workgroup owns G = 16 adjacent rows k1; loads are row-contiguous
//            (lanes along the row); the last Stockham exchange re-maps the
//            threads so lanes run across the G rows, and the stores
//            X[k1..k1+15 + N1*k2] are 128-B lines again.
//   Batches are processed in chunks whose intermediate fits the 256 MiB
//   Infinity Cache, so the rows pass reads the columns pass's output on-die.
// n > 2^20: transpose -> N1-pt FFTs -> twiddled transpose -> N2-pt FFTs ->
//   transpose (five passes of 8n bytes each way).
// The backward 1/n is applied once, in the last pass.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

namespace vvh {

// ---------------------------------------------------------------------------
// Two-pass four-step
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wg_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// G transforms of length N per workgroup; LDS region per transform of S
// elements (floats when RI, float2 otherwise).  S is odd, so the same offset in
// the G regions falls in G different banks (lanes of one instruction work on
// different transforms in the interleaved mapping).
template <int N, int G, bool RI>
struct FsGeo {
    using Ge = Geo<N>;
    static constexpr int T = Ge::T;
    static constexpr int THREADS = G * T;
    static constexpr int S = Ge::LDS | 1;
    static constexpr int LDS_BYTES = G * S * (RI ? 4 : 8);
    static_assert(THREADS <= 1024 && Ge::NPASS >= 2, "two-pass four-step geometry");
};

// Stockham exchange after pass p; the writer is thread wt of transform wj, the
// reader thread rt of transform rj (a re-map of the workgroup when they differ).
template <int N, int p, int S, bool RI>
__device__ __forceinline__ void fs_exchange(float2* v, void* lds, int wj, int wt, int rj, int rt) {
    using Ge = Geo<N>;
    constexpr int R = Ge::radix(p), Ns = Ge::ns(p), R2 = Ge::radix(p + 1), T = Ge::T;
    if constexpr (RI) {
        float* W = reinterpret_cast<float*>(lds) + wj * S;
        const float* Rd = reinterpret_cast<const float*>(lds) + rj * S;
        float nx[Ge::P];
#pragma unroll
        for (int i = 0; i < Ge::P / R; ++i) {
            const int b = wt + T * i, base = (b / Ns) * Ns * R + (b % Ns);
#pragma unroll
            for (int r = 0; r < R; ++r) W[Ge::pad(base + r * Ns)] = v[i * R + r].x;
        }
        wg_bar();
#pragma unroll
        for (int i = 0; i < Ge::P / R2; ++i) {
            const int b = rt + T * i;
#pragma unroll
            for (int r = 0; r < R2; ++r) nx[i * R2 + r] = Rd[Ge::pad(b + r * (N / R2))];
        }
        wg_bar();
#pragma unroll
        for (int i = 0; i < Ge::P / R; ++i) {
            const int b = wt + T * i, base = (b / Ns) * Ns * R + (b % Ns);
#pragma unroll
            for (int r = 0; r < R; ++r) W[Ge::pad(base + r * Ns)] = v[i * R + r].y;
        }
        wg_bar();
#pragma unroll
        for (int i = 0; i < Ge::P / R2; ++i) {
            const int b = rt + T * i;
#pragma unroll
            for (int r = 0; r < R2; ++r) v[i * R2 + r] = make_float2(nx[i * R2 + r], Rd[Ge::pad(b + r * (N / R2))]);
        }
        wg_bar();
    } else {
        float2* W = reinterpret_cast<float2*>(lds) + wj * S;
        const float2* Rd = reinterpret_cast<const float2*>(lds) + rj * S;
#pragma unroll
        for (int i = 0; i < Ge::P / R; ++i) {
            const int b = wt + T * i, base = (b / Ns) * Ns * R + (b % Ns);
#pragma unroll
            for (int r = 0; r < R; ++r) W[Ge::pad(base + r * Ns)] = v[i * R + r];
        }
        wg_bar();
#pragma unroll
        for (int i = 0; i < Ge::P / R2; ++i) {
            const int b = rt + T * i;
#pragma unroll
            for (int r = 0; r < R2; ++r) v[i * R2 + r] = Rd[Ge::pad(b + r * (N / R2))];
        }
        wg_bar();
    }
}

// Pass chain; with REMAP the last pass runs in mapping (j2, t2), all others in (j1, t1).
template <int N, bool FWD, int p, int S, bool RI, bool REMAP>
struct FsChain {
    __device__ __forceinline__ static void run(float2* v, void* lds, const TwTab<N>& tw, int j1, int t1, int j2,
                                               int t2) {
        constexpr int NP = Geo<N>::NPASS;
        constexpr bool last = p == NP - 1;
        pass_compute<N, FWD, p, false>(v, (REMAP && last) ? t2 : t1, tw);
        if constexpr (!last) {
            if constexpr (REMAP && p + 1 == NP - 1) fs_exchange<N, p, S, RI>(v, lds, j1, t1, j2, t2);
            else fs_exchange<N, p, S, RI>(v, lds, j1, t1, j1, t1);
            FsChain<N, FWD, p + 1, S, RI, REMAP>::run(v, lds, tw, j1, t1, j2, t2);
        }
    }
};

// Optional fused element-wise stages of the two passes (Bluestein, below):
//   pre  (columns pass input):  x[m] = m < nsig ? raw[b*in_dist + m] * pre_chirp[m] : 0
//   mulv (rows pass output):    X[k] *= mulv[k]
//   post (rows pass output):    post_out[b*out_dist + k] = post_scale * post_chirp[k] * X[k], k < nout
// b counts from b0 (the chunk's first transform).  All null: the plain FFT.
struct FsHooks {
    const float2* mulv = nullptr;
    const float2* pre_chirp = nullptr;
    const void* raw = nullptr;
    long long in_dist = 0, nsig = 0;
    int real_in = 0;
    const float2* post_chirp = nullptr;
    float2* post_out = nullptr;
    long long out_dist = 0, nout = 0;
    float post_scale = 1.0f;
    long long b0 = 0;
};

// Columns pass: Y[b][k1][n2] = W_n^(+-n2 k1) * FFT_N1(x[b][.][n2])[k1]
template <int N1, int G, bool RI, bool FWD>
__global__ void __launch_bounds__(G * Geo<N1>::T)
k_fs_cols(const float2* __restrict__ in, float2* __restrict__ out, int N2, int cpb, const float2* gpass,
          const float2* gtab, const float2* __restrict__ split, int lo_bits, FsHooks hk) {
    using Ge = Geo<N1>;
    using F = FsGeo<N1, G, RI>;
    __shared__ __attribute__((aligned(16))) unsigned char lds[F::LDS_BYTES];
    __shared__ float2 ltab[TwLayout<N1>::ENTRIES];
    // two-level W_n table (lo[2^lo_bits] ++ hi[n >> lo_bits], n <= 2^20) in LDS
    __shared__ float2 lsplit[2048];
    stage_twiddles<N1, F::THREADS>(ltab, gpass, gtab);
    const long long n = (long long)N1 * N2;
    {
        const int nsplit = (1 << lo_bits) + (int)(n >> lo_bits);
        for (int i = threadIdx.x; i < nsplit; i += F::THREADS) lsplit[i] = split[i];
    }
    const long long b = blockIdx.x / cpb;
    const int col = (blockIdx.x % cpb) * G + (int)(threadIdx.x % G), t = threadIdx.x / G;
    float2 v[Ge::P];
    if (hk.pre_chirp) {
        const long long base = (hk.b0 + b) * hk.in_dist;
#pragma unroll
        for (int r = 0; r < Ge::P; ++r) {
            const long long m = (long long)(t + r * Ge::T) * N2 + col;
            float2 x = make_float2(0.0f, 0.0f);
            if (m < hk.nsig) {
                x = hk.real_in ? make_float2(reinterpret_cast<const float*>(hk.raw)[base + m], 0.0f)
                               : reinterpret_cast<const float2*>(hk.raw)[base + m];
                x = cmul(x, hk.pre_chirp[m]);
            }
            v[r] = x;
        }
    } else {
        const float2* src = in + b * n + col;
#pragma unroll
        for (int r = 0; r < Ge::P; ++r) v[r] = ld_nt(src + (long long)(t + r * Ge::T) * N2);
    }
    __syncthreads();
    const int j = threadIdx.x % G;
    FsChain<N1, FWD, 0, F::S, RI, false>::run(v, lds, TwTab<N1>{ltab}, j, t, j, t);
    const unsigned mask = (1u << lo_bits) - 1u;
    const float2* hi = lsplit + (1u << lo_bits);
    float2* dst = out + b * n + col;
#pragma unroll
    for (int q = 0; q < Ge::P; ++q) {
        const int k1 = out_pos<N1>(t, q);
        const unsigned k = (unsigned)col * (unsigned)k1;   // < n <= 2^20
        float2 w = cmul(lsplit[k & mask], hi[k >> lo_bits]);
        if (!FWD) w = cconj(w);
        st_nt(cmul(v[q], w), dst + (long long)k1 * N2);
    }
}

// Rows pass: X[b][k1 + N1 k2] = scale * FFT_N2(Y[b][k1][.])[k2], times mulv[k1 + N1 k2]
// when mulv is given (Bluestein's pointwise product with the chirp spectrum,
// the same n-vector for every transform of the batch)
template <int N2, int G, bool RI, bool FWD>
__global__ void __launch_bounds__(G * Geo<N2>::T)
k_fs_rows(const float2* __restrict__ in, float2* __restrict__ out, int N1, int rpb, const float2* gpass,
          const float2* gtab, float scale, FsHooks hk) {
    using Ge = Geo<N2>;
    using F = FsGeo<N2, G, RI>;
    __shared__ __attribute__((aligned(16))) unsigned char lds[F::LDS_BYTES];
    __shared__ float2 ltab[TwLayout<N2>::ENTRIES];
    stage_twiddles<N2, F::THREADS>(ltab, gpass, gtab);
    const long long n = (long long)N1 * N2;
    const long long b = blockIdx.x / rpb;
    const int r0 = (blockIdx.x % rpb) * G;
    const int j1 = threadIdx.x / Ge::T, t1 = threadIdx.x % Ge::T;   // lanes along a row
    const int j2 = threadIdx.x % G, t2 = threadIdx.x / G;           // lanes across rows
    const float2* src = in + b * n + (long long)(r0 + j1) * N2 + t1;
    float2 v[Ge::P];
#pragma unroll
    for (int r = 0; r < Ge::P; ++r) v[r] = ld_nt(src + r * Ge::T);
    __syncthreads();
    FsChain<N2, FWD, 0, F::S, RI, true>::run(v, lds, TwTab<N2>{ltab}, j1, t1, j2, t2);
    float2* dst = out + b * n + r0 + j2;
#pragma unroll
    for (int q = 0; q < Ge::P; ++q) {
        const int k2 = out_pos<N2>(t2, q);
        float2 x = FWD ? v[q] : cscale(v[q], scale);
        const long long k = r0 + j2 + (long long)k2 * N1;
        if (hk.mulv) x = cmul(x, hk.mulv[k]);
        if (hk.post_chirp) {
            if (k < hk.nout) hk.post_out[(hk.b0 + b) * hk.out_dist + k] = cscale(cmul(x, hk.post_chirp[k]), hk.post_scale);
        } else {
            st_nt(x, dst + (long long)k2 * N1);
        }
    }
}

namespace {
// variant: 0 = RI exchange, G 16; 1 = float2 exchange, G 16 (default: fastest measured,
// profiles/r01_kbench_fourstep.jsonl); 2 = float2, G 8; 3 = RI, G 8
template <int N, int G, bool RI, bool FWD>
hipError_t fs_cols_g(const float2* in, float2* out, int N2, long long batch, const float2* split, int lo_bits,
                     const FsHooks& hk, hipStream_t s) {
    const float2* tab = twiddle_table(N);
    const float2* pas = pass_twiddles(N);
    if (!tab || !pas) return hipErrorOutOfMemory;
    const int cpb = N2 / G;
    const long long blocks = (long long)cpb * batch;
    if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_fs_cols<N, G, RI, FWD>), dim3((unsigned)blocks), dim3(FsGeo<N, G, RI>::THREADS), 0, s, in,
                       out, N2, cpb, pas, tab, split, lo_bits, hk);
    return hipGetLastError();
}

template <int N, int G, bool RI, bool FWD>
hipError_t fs_rows_g(const float2* in, float2* out, int N1, long long batch, float scale, const FsHooks& hk,
                     hipStream_t s) {
    const float2* tab = twiddle_table(N);
    const float2* pas = pass_twiddles(N);
    if (!tab || !pas) return hipErrorOutOfMemory;
    const int rpb = N1 / G;
    const long long blocks = (long long)rpb * batch;
    if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_fs_rows<N, G, RI, FWD>), dim3((unsigned)blocks), dim3(FsGeo<N, G, RI>::THREADS), 0, s, in,
                       out, N1, rpb, pas, tab, scale, hk);
    return hipGetLastError();
}

template <int N, bool FWD>
hipError_t fs_cols(int var, const float2* in, float2* out, int N2, long long batch, const float2* split, int lo_bits,
                   const FsHooks& hk, hipStream_t s) {
    switch (var) {
        case 1: return fs_cols_g<N, 16, false, FWD>(in, out, N2, batch, split, lo_bits, hk, s);
        case 2: return fs_cols_g<N, 8, false, FWD>(in, out, N2, batch, split, lo_bits, hk, s);
        case 3: return fs_cols_g<N, 8, true, FWD>(in, out, N2, batch, split, lo_bits, hk, s);
        default: return fs_cols_g<N, 16, true, FWD>(in, out, N2, batch, split, lo_bits, hk, s);
    }
}

template <int N, bool FWD>
hipError_t fs_rows(int var, const float2* in, float2* out, int N1, long long batch, float scale, const FsHooks& hk,
                   hipStream_t s) {
    switch (var) {
        case 1: return fs_rows_g<N, 16, false, FWD>(in, out, N1, batch, scale, hk, s);
        case 2: return fs_rows_g<N, 8, false, FWD>(in, out, N1, batch, scale, hk, s);
        case 3: return fs_rows_g<N, 8, true, FWD>(in, out, N1, batch, scale, hk, s);
        default: return fs_rows_g<N, 16, true, FWD>(in, out, N1, batch, scale, hk, s);
    }
}

template <bool FWD>
hipError_t fs_cols_any(int N1, int var, const float2* in, float2* out, int N2, long long batch, const float2* split,
                       int lo_bits, const FsHooks& hk, hipStream_t s) {
    switch (N1) {
        case 64: return fs_cols<64, FWD>(var, in, out, N2, batch, split, lo_bits, hk, s);
        case 128: return fs_cols<128, FWD>(var, in, out, N2, batch, split, lo_bits, hk, s);
        case 256: return fs_cols<256, FWD>(var, in, out, N2, batch, split, lo_bits, hk, s);
        case 512: return fs_cols<512, FWD>(var, in, out, N2, batch, split, lo_bits, hk, s);
        case 1024: return fs_cols<1024, FWD>(var, in, out, N2, batch, split, lo_bits, hk, s);
        default: return hipErrorInvalidValue;
    }
}

template <bool FWD>
hipError_t fs_rows_any(int N2, int var, const float2* in, float2* out, int N1, long long batch, float scale,
                       const FsHooks& hk, hipStream_t s) {
    switch (N2) {
        case 64: return fs_rows<64, FWD>(var, in, out, N1, batch, scale, hk, s);
        case 128: return fs_rows<128, FWD>(var, in, out, N1, batch, scale, hk, s);
        case 256: return fs_rows<256, FWD>(var, in, out, N1, batch, scale, hk, s);
        case 512: return fs_rows<512, FWD>(var, in, out, N1, batch, scale, hk, s);
        case 1024: return fs_rows<1024, FWD>(var, in, out, N1, batch, scale, hk, s);
        default: return hipErrorInvalidValue;
    }
}

// n = N1*N2, 64 <= N1 <= N2 <= 1024
// One two-pass transform chain over a batch in chunks.  With hooks, the
// columns pass may read the raw Bluestein input (pre) instead of `in`, and the
// rows pass may multiply by a vector (mulv) and/or write scaled, chirped and
// truncated rows to another buffer (post) instead of `out`.
hipError_t twopass_chain(long long n, int lg, int fwd, const float2* in, float2* out, long long batch, hipStream_t s,
                         FsHooks hk) {
    const int N1 = 1 << (lg / 2), N2 = (int)(n / N1);
    int lo_bits = 0;
    const float2* split = twiddle_split(n, &lo_bits);
    if (!split) return hipErrorOutOfMemory;
    const int var = (int)knob(KNOB_FS_VAR, 1);
    // chunk of transforms whose intermediate stays in the Infinity Cache
    const long long chunk_bytes = knob(KNOB_FS_CHUNK_MB, 0) << 20;
    long long chunk = chunk_bytes > 0 ? chunk_bytes / (8 * n) : batch;
    if (chunk < 1) chunk = 1;
    if (chunk > batch) chunk = batch;
    float2* y = nullptr;
    hipError_t e = hipMallocAsync((void**)&y, sizeof(float2) * (size_t)n * (size_t)chunk, s);
    if (e != hipSuccess) return e;
    const float scale = 1.0f / (float)n;
    for (long long c = 0; c < batch && e == hipSuccess; c += chunk) {
        const long long nb = batch - c < chunk ? batch - c : chunk;
        const float2* src = hk.pre_chirp ? nullptr : in + c * n;
        float2* dst = hk.post_chirp ? nullptr : out + c * n;
        hk.b0 = c;
        e = fwd ? fs_cols_any<true>(N1, var, src, y, N2, nb, split, lo_bits, hk, s)
                : fs_cols_any<false>(N1, var, src, y, N2, nb, split, lo_bits, hk, s);
        if (e == hipSuccess)
            e = fwd ? fs_rows_any<true>(N2, var, y, dst, N1, nb, scale, hk, s)
                    : fs_rows_any<false>(N2, var, y, dst, N1, nb, scale, hk, s);
    }
    (void)hipFreeAsync(y, s);
    return e;
}

hipError_t launch_c2c_twopass(long long n, int lg, int fwd, const float2* in, float2* out, long long batch,
                              hipStream_t s) {
    return twopass_chain(n, lg, fwd, in, out, batch, s, FsHooks{});
}
}  // namespace

// ---------------------------------------------------------------------------
// Five-pass four-step (n > 2^20)
// ---------------------------------------------------------------------------

constexpr int TT = 64;   // transpose tile

// out_b[c][r] = in_b[r][c] (* W_n^(+-r*c) when TW), matrices R x C, batch-major.
template <bool TW>
__global__ void __launch_bounds__(256)
k_transpose(const float2* __restrict__ in, float2* __restrict__ out, long long R, long long C, long long tiles_c,
            long long tiles_per_mat, const float2* __restrict__ tw, int lo_bits, long long nlo, int fwd) {
    __shared__ float2 tile[TT][TT + 1];
    const long long b = blockIdx.x / tiles_per_mat, tt = blockIdx.x % tiles_per_mat;
    const long long r0 = (tt / tiles_c) * TT, c0 = (tt % tiles_c) * TT;
    const float2* src = in + b * R * C;
    float2* dst = out + b * R * C;
    const int tx = threadIdx.x % TT, ty = threadIdx.x / TT;
    for (int i = ty; i < TT; i += 256 / TT) {
        const long long r = r0 + i, c = c0 + tx;
        if (r < R && c < C) tile[i][tx] = src[r * C + c];
    }
    __syncthreads();
    for (int i = ty; i < TT; i += 256 / TT) {
        const long long c = c0 + i, r = r0 + tx;
        if (r < R && c < C) {
            float2 v = tile[tx][i];
            if constexpr (TW) {
                const long long k = r * c;   // < n: r < N2, c < N1
                float2 w = cmul(tw[k & (nlo - 1)], tw[nlo + (k >> lo_bits)]);
                if (!fwd) w.y = -w.y;
                v = cmul(v, w);
            }
            dst[c * R + r] = v;
        }
    }
}

static hipError_t transpose(const float2* in, float2* out, long long R, long long C, long long batch, bool tw,
                            const float2* tab, int lo_bits, long long n, int fwd, hipStream_t s) {
    const long long tc = (C + TT - 1) / TT, tr = (R + TT - 1) / TT, per = tc * tr;
    const long long blocks = per * batch;
    if (blocks <= 0) return hipSuccess;
    if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
    const long long nlo = 1LL << lo_bits;
    if (tw)
        hipLaunchKernelGGL(k_transpose<true>, dim3((unsigned)blocks), dim3(256), 0, s, in, out, R, C, tc, per, tab,
                           lo_bits, nlo, fwd);
    else
        hipLaunchKernelGGL(k_transpose<false>, dim3((unsigned)blocks), dim3(256), 0, s, in, out, R, C, tc, per,
                           tab, lo_bits, nlo, fwd);
    (void)n;
    return hipGetLastError();
}

bool c2c_large_supported(long long n) { return n > 4096 && n <= (1LL << 24) && (n & (n - 1)) == 0; }

hipError_t launch_c2c_large(long long n, int fwd, const float2* in, float2* out, long long batch, hipStream_t s) {
    if (!c2c_large_supported(n)) return hipErrorInvalidValue;
    if (batch <= 0) return hipSuccess;
    if (c2c_supported(n))   // 8192: one pass in LDS (fft_kernels.hip)
        return launch_c2c(n, fwd, in, out, batch, n, n, 1.0f / (float)n, s);
    int lg = 0;
    while ((1LL << lg) < n) ++lg;
    if (lg <= 20 && knob(KNOB_FS_OLD, 0) == 0) return launch_c2c_twopass(n, lg, fwd, in, out, batch, s);
    const long long N1 = 1LL << (lg / 2), N2 = n / N1;   // N1 <= N2 <= 4096
    int lo_bits = 0;
    const float2* tab = twiddle_split(n, &lo_bits);
    if (!tab) return hipErrorOutOfMemory;
    float2 *s1 = nullptr, *s2 = nullptr;
    const size_t bytes = sizeof(float2) * (size_t)n * (size_t)batch;
    hipError_t e = hipMallocAsync((void**)&s1, bytes, s);
    if (e != hipSuccess) return e;
    e = hipMallocAsync((void**)&s2, bytes, s);
    if (e != hipSuccess) {
        (void)hipFreeAsync(s1, s);
        return e;
    }
    do {
        if ((e = transpose(in, s1, N1, N2, batch, false, tab, lo_bits, n, fwd, s)) != hipSuccess) break;
        if ((e = launch_c2c(N1, fwd, s1, s2, batch * N2, N1, N1, 1.0f / (float)N1, s)) != hipSuccess) break;
        if ((e = transpose(s2, s1, N2, N1, batch, true, tab, lo_bits, n, fwd, s)) != hipSuccess) break;
        if ((e = launch_c2c(N2, fwd, s1, s2, batch * N1, N2, N2, 1.0f / (float)N2, s)) != hipSuccess) break;
        e = transpose(s2, out, N1, N2, batch, false, tab, lo_bits, n, fwd, s);
    } while (false);
    (void)hipFreeAsync(s1, s);
    (void)hipFreeAsync(s2, s);
    return e;
}

// ---------------------------------------------------------------------------
// Bluestein (chirp-z) for non-power-of-two n: O(M log M), M = pow2 >= 2n-1.
// With a[m] = exp(-+i*pi*m^2/n) (sign of the transform), n*k = (n^2 + k^2 -
// (k-n)^2)/2 gives X[k] = a[k] * sum_j (x[j] a[j]) conj(a[k-j]): a length-M
// circular convolution of u = x*a (zero padded) with v[m] = conj(a[m]) for
// |m| < n, done as IFFT(FFT(u) * V) with V = FFT(v) cached per (n, sign).
// The reference computes these lengths with an O(n^2) f32 DFT
// (src/spectral/fft_kiss.c:76-92); this path replaces it above
// BLUESTEIN_MIN, where it is both faster and closer to f64.
// ---------------------------------------------------------------------------
namespace {
struct ChirpPlan {
    long long M;
    float2* chirp;   // a[m], m < n
    float2* V;       // FFT_M(v)
};
std::mutex g_bmu;
std::map<std::tuple<int, long long, int>, ChirpPlan> g_bplans;   // (device, n, fwd)

long long pow2_ge(long long x) {
    long long m = 1;
    while (m < x) m <<= 1;
    return m;
}

hipError_t fft_pow2(long long m, int fwd, const float2* in, float2* out, long long batch, hipStream_t s) {
    if (c2c_supported(m)) return launch_c2c(m, fwd, in, out, batch, m, m, 1.0f / (float)m, s);
    return launch_c2c_large(m, fwd, in, out, batch, s);
}

__global__ void k_chirp_v(const float2* __restrict__ a, float2* __restrict__ v, long long n, long long M) {
    const long long m = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    float2 r = make_float2(0.0f, 0.0f);
    if (m < n) r = a[m];
    else if (m > M - n) r = a[M - m];
    v[m] = make_float2(r.x, -r.y);   // conj(a[|m|])
}

// u[f][m] = x[f][m] * a[m] (m < n), 0 up to M
__global__ void k_bluestein_pre(const void* __restrict__ in, int real_in, long long in_dist,
                                const float2* __restrict__ a, float2* __restrict__ u, long long n, long long M,
                                long long total) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const long long f = i / M, m = i - f * M;
        float2 r = make_float2(0.0f, 0.0f);
        if (m < n) {
            const float2 x = real_in ? make_float2(reinterpret_cast<const float*>(in)[f * in_dist + m], 0.0f)
                                     : reinterpret_cast<const float2*>(in)[f * in_dist + m];
            r = cmul(x, a[m]);
        }
        u[i] = r;
    }
}

__global__ void k_mul_bcast(float2* __restrict__ U, const float2* __restrict__ V, long long M, long long total) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride)
        U[i] = cmul(U[i], V[i % M]);
}

// X[f][k] = scale * a[k] * y[f][k], k < nout
__global__ void k_bluestein_post(const float2* __restrict__ y, const float2* __restrict__ a, float2* __restrict__ out,
                                 long long M, long long nout, long long out_dist, float scale, long long total) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const long long f = i / nout, k = i - f * nout;
        out[f * out_dist + k] = cscale(cmul(y[f * M + k], a[k]), scale);
    }
}

unsigned grid_for(long long total) {
    long long b = (total + 255) / 256;
    return (unsigned)(b > 65536 ? 65536 : (b < 1 ? 1 : b));
}

const ChirpPlan* chirp_plan(long long n, int fwd, hipStream_t s) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    const auto key = std::make_tuple(dev, n, fwd);
    std::lock_guard<std::mutex> lk(g_bmu);
    auto it = g_bplans.find(key);
    if (it != g_bplans.end()) return &it->second;
    ChirpPlan p{pow2_ge(2 * n - 1), nullptr, nullptr};
    if (p.M > (1LL << 24)) return nullptr;
    // a[m] = exp(-+i*pi*(m^2 mod 2n)/n), reduced exactly in integers, rounded from double
    std::vector<float2> h((size_t)n);
    for (long long m = 0; m < n; ++m) {
        const long long q = (long long)(((unsigned __int128)m * (unsigned __int128)m) % (unsigned __int128)(2 * n));
        const double ang = (fwd ? -M_PI : M_PI) * (double)q / (double)n;
        h[(size_t)m] = make_float2((float)std::cos(ang), (float)std::sin(ang));
    }
    float2* v = nullptr;
    bool ok = hipMalloc(&p.chirp, sizeof(float2) * n) == hipSuccess &&
              hipMalloc(&p.V, sizeof(float2) * p.M) == hipSuccess && hipMalloc(&v, sizeof(float2) * p.M) == hipSuccess &&
              hipMemcpyAsync(p.chirp, h.data(), sizeof(float2) * n, hipMemcpyHostToDevice, s) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_chirp_v, dim3((unsigned)((p.M + 255) / 256)), dim3(256), 0, s, p.chirp, v, n, p.M);
        ok = hipGetLastError() == hipSuccess && fft_pow2(p.M, 1, v, p.V, 1, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
    }
    if (v) (void)hipFree(v);
    if (!ok) {
        if (p.chirp) (void)hipFree(p.chirp);
        if (p.V) (void)hipFree(p.V);
        return nullptr;
    }
    return &(g_bplans[key] = p);
}
}  // namespace

bool bluestein_supported(long long n) { return n >= 2 && pow2_ge(2 * n - 1) <= (1LL << 24); }

hipError_t launch_bluestein(long long n, int fwd, const void* in, int real_in, float2* out, long long nout,
                            long long batch, long long in_dist, long long out_dist, float scale, hipStream_t s) {
    if (batch <= 0) return hipSuccess;
    const ChirpPlan* p = chirp_plan(n, fwd, s);
    if (!p) return hipErrorOutOfMemory;
    const long long M = p->M, total = M * batch;
    const int lgM = ilog2((int)(M < (1LL << 30) ? M : (1LL << 30)));
    if (!c2c_supported(M) && lgM <= 20 && knob(KNOB_FS_OLD, 0) == 0 && knob(KNOB_BLUE_UNFUSED, 0) == 0) {
        // two-pass M (8192..2^20): chirp pre-multiply and zero padding in the forward
        // columns pass, the product with V in its rows pass, and the post-multiply,
        // scale and truncation to nout in the inverse rows pass -- four kernels,
        // no u / padded-input pass and no full-length output pass
        float2* U = nullptr;
        hipError_t e = hipMallocAsync((void**)&U, sizeof(float2) * total, s);
        if (e != hipSuccess) return e;
        FsHooks f;
        f.pre_chirp = p->chirp;
        f.raw = in;
        f.in_dist = in_dist;
        f.nsig = n;
        f.real_in = real_in;
        f.mulv = p->V;
        e = twopass_chain(M, lgM, 1, nullptr, U, batch, s, f);
        if (e == hipSuccess) {
            FsHooks b;
            b.post_chirp = p->chirp;
            b.post_out = out;
            b.out_dist = out_dist;
            b.nout = nout;
            b.post_scale = scale;
            e = twopass_chain(M, lgM, 0, U, nullptr, batch, s, b);
        }
        (void)hipFreeAsync(U, s);
        return e;
    }
    float2 *u = nullptr, *U = nullptr;
    hipError_t e = hipMallocAsync((void**)&u, sizeof(float2) * total, s);
    if (e != hipSuccess) return e;
    e = hipMallocAsync((void**)&U, sizeof(float2) * total, s);
    if (e != hipSuccess) {
        (void)hipFreeAsync(u, s);
        return e;
    }
    do {
        hipLaunchKernelGGL(k_bluestein_pre, dim3(grid_for(total)), dim3(256), 0, s, in, real_in, in_dist, p->chirp, u,
                           n, M, total);
        if ((e = hipGetLastError()) != hipSuccess) break;
        if ((e = fft_pow2(M, 1, u, U, batch, s)) != hipSuccess) break;
        hipLaunchKernelGGL(k_mul_bcast, dim3(grid_for(total)), dim3(256), 0, s, U, p->V, M, total);
        if ((e = hipGetLastError()) != hipSuccess) break;
        if ((e = fft_pow2(M, 0, U, u, batch, s)) != hipSuccess) break;   // includes 1/M
        const long long tot_out = nout * batch;
        hipLaunchKernelGGL(k_bluestein_post, dim3(grid_for(tot_out)), dim3(256), 0, s, u, p->chirp, out, M, nout,
                           out_dist, scale, tot_out);
        e = hipGetLastError();
    } while (false);
    (void)hipFreeAsync(u, s);
    (void)hipFreeAsync(U, s);
    return e;
}

__global__ void k_promote_real(const float* __restrict__ in, float2* __restrict__ out, long long count) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride)
        out[i] = make_float2(in[i], 0.0f);
}

hipError_t launch_promote_real(const float* in, float2* out, long long count, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    long long blocks = (count + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_promote_real, dim3((unsigned)blocks), dim3(256), 0, s, in, out, count);
    return hipGetLastError();
}

}  // namespace vvh
