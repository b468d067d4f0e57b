// large_fft.hip -- power-of-two C2C transforms longer than one workgroup's
// register/LDS FFT (n > 4096, up to 2^24), as a four-step FFT over the fused
// batched kernels of fft_kernels.hip.
//
// The reference computes every power of two with one radix-2 DIT
// (src/spectral/fft_kiss.c:27-74).  Here n = N1*N2 (N1, N2 <= 4096) and
//   X[k1 + N1*k2] = sum_n2 W_N2^(n2 k2) * W_n^(n2 k1) * sum_n1 x[n1 N2 + n2] W_N1^(n1 k1)
// runs as: transpose [N1][N2] -> [N2][N1]; N2 row FFTs of length N1; transpose
// with the twiddle W_n^(n2 k1) fused; N1 row FFTs of length N2; transpose to
// natural order.  Five HBM passes of 8n bytes each -- bandwidth-bound like the
// rest of the path.  The backward 1/n is split as 1/N1 and 1/N2 over the two
// FFT passes.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

#include <cmath>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

namespace vvh {

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
    int lg = 0;
    while ((1LL << lg) < n) ++lg;
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
