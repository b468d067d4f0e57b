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
