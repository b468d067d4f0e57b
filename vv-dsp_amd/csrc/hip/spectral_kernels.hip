// spectral_kernels.hip -- Hilbert mask, FFT-based DCT pre/post steps, the
// O(N^2) DCT for non-power-of-two N, and the NaN policy for gfx950.
//
// Hilbert (src/spectral/hilbert.c:14-75): Z = one-sided mask of the R2C
// spectrum (x1 at DC and N/2, x2 on 1..ceil(N/2)-1, 0 on negative bins), then
// inverse C2C.  The mask kernel expands the N/2+1 half spectrum straight into
// the length-N buffer the inverse FFT reads.
//
// DCT-II (src/spectral/dct.c:21-30, X[k] = sum x[n] cos(pi (n+1/2) k / N)) is
// computed as Makhoul's permutation v[n] = x[2n], v[N-1-n] = x[2n+1], an N-point
// R2C, and X[k] = Re(W_4N^k V[k]).  Its inverse (dct3_inverse_from_ii,
// dct.c:32-42) is V[k] = W_4N^-k (X[k] - i X[N-k]), an N-point C2R and the
// inverse permutation.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

namespace vvh {

static inline unsigned nblocks(long long count) {
    long long b = (count + 255) / 256;
    if (b > 65536) b = 65536;
    if (b < 1) b = 1;
    return (unsigned)b;
}

#define GRID_STRIDE(i, count) \
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < (count); i += (long long)gridDim.x * blockDim.x)

__global__ void k_hilbert_mask(long long n, const float2* half, float2* full, long long batch,
                               long long half_dist) {
    const long long total = n * batch;
    GRID_STRIDE(i, total) {
        const long long f = i / n, k = i - f * n;
        const float2* h = half + f * half_dist;
        float2 z = make_float2(0.0f, 0.0f);
        if (k == 0) z = h[0];
        else if ((n % 2 == 0) && k == n / 2) z = h[k];
        else if (2 * k < n) z = cscale(h[k], 2.0f);
        full[i] = z;
    }
}

hipError_t launch_hilbert_mask(long long n, const float2* half, float2* full, long long batch,
                               long long half_dist, hipStream_t s) {
    hipLaunchKernelGGL(k_hilbert_mask, dim3(nblocks(n * batch)), dim3(256), 0, s, n, half, full, batch,
                       half_dist);
    return hipGetLastError();
}

__global__ void k_dct2_pre(long long n, const float* x, float* v, long long batch) {
    const long long total = n * batch;
    GRID_STRIDE(i, total) {
        const long long f = i / n, m = i - f * n;
        // v[m] = x[2m] for m < n/2 ; v[m] = x[2(n-1-m)+1] for m >= n/2
        const long long src = (m < n / 2) ? 2 * m : 2 * (n - 1 - m) + 1;
        v[i] = x[f * n + src];
    }
}

hipError_t launch_dct2_pre(long long n, const float* x, float* v, long long batch, hipStream_t s) {
    hipLaunchKernelGGL(k_dct2_pre, dim3(nblocks(n * batch)), dim3(256), 0, s, n, x, v, batch);
    return hipGetLastError();
}

// V: [batch][n/2+1] half spectrum of v; X[k] = Re(W4N^k * V[k]) (V[k] = conj(V[n-k]) above n/2)
__global__ void k_dct2_post(long long n, const float2* V, float* X, long long batch,
                            const float2* __restrict__ tw4n) {
    const long long total = n * batch;
    const long long nh = n / 2 + 1;
    GRID_STRIDE(i, total) {
        const long long f = i / n, k = i - f * n;
        const float2 vk = (k < nh) ? V[f * nh + k] : cconj(V[f * nh + (n - k)]);
        const float2 w = tw4n[k];
        X[i] = vk.x * w.x - vk.y * w.y;
    }
}

hipError_t launch_dct2_post(long long n, const float2* V, float* X, long long batch,
                            const float2* tw4n, hipStream_t s) {
    hipLaunchKernelGGL(k_dct2_post, dim3(nblocks(n * batch)), dim3(256), 0, s, n, V, X, batch, tw4n);
    return hipGetLastError();
}

// X: [batch][n] -> V: [batch][n/2+1],  V[k] = conj(W4N^k) * (X[k] - i X[n-k]),  X[n] := 0
__global__ void k_dct3_pre(long long n, const float* X, float2* V, long long batch,
                           const float2* __restrict__ tw4n) {
    const long long nh = n / 2 + 1;
    const long long total = nh * batch;
    GRID_STRIDE(i, total) {
        const long long f = i / nh, k = i - f * nh;
        const float a = X[f * n + k];
        const float b = (k == 0) ? 0.0f : X[f * n + (n - k)];
        const float2 w = cconj(tw4n[k]);
        V[i] = cmul(make_float2(a, -b), w);
    }
}

hipError_t launch_dct3_pre(long long n, const float* X, float2* V, long long batch, const float2* tw4n,
                           hipStream_t s) {
    hipLaunchKernelGGL(k_dct3_pre, dim3(nblocks((n / 2 + 1) * batch)), dim3(256), 0, s, n, X, V, batch,
                       tw4n);
    return hipGetLastError();
}

// x[2m] = v[m], x[2m+1] = v[n-1-m]  (times scale)
__global__ void k_dct3_post(long long n, const float* v, float* x, long long batch, float scale) {
    const long long total = n * batch;
    GRID_STRIDE(i, total) {
        const long long f = i / n, e = i - f * n;
        const long long src = (e % 2 == 0) ? e / 2 : n - 1 - e / 2;
        x[i] = v[f * n + src] * scale;
    }
}

hipError_t launch_dct3_post(long long n, const float* v, float* x, long long batch, float scale,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_dct3_post, dim3(nblocks(n * batch)), dim3(256), 0, s, n, v, x, batch, scale);
    return hipGetLastError();
}

// O(N^2) DCT for any N with f64 accumulation; angles reduced exactly in
// integer arithmetic (the reference's own complexity: dct.c:21-68).
//   type 2 dir +1 : X[k] = sum_n x[n] cos(pi (2n+1) k / 2N)
//   type 2/3 dir -1: x[n] = (2/N) (X[0]/2 + sum_{k>=1} X[k] cos(pi k (2n+1) / 2N))
//   type 3 dir +1 : Y[k] = x[0] + 2 sum_{n>=1} x[n] cos(pi k (2n+1) / 2N)
//   type 4        : X[k] = sum_n x[n] cos(pi (2n+1)(2k+1) / 4N)   (x 2/N for dir -1)
__global__ void k_dct_naive(long long n, int type, int dir, const float* in, float* out,
                            long long batch) {
    const long long total = n * batch;
    GRID_STRIDE(i, total) {
        const long long f = i / n, k = i - f * n;
        const float* x = in + f * n;
        double acc = 0.0;
        if (type == 4) {
            const long long period = 8 * n;   // angle unit pi/(4N)
            for (long long m = 0; m < n; ++m) {
                const long long a = ((2 * m + 1) * (2 * k + 1)) % period;
                acc += (double)x[m] * cospi((double)a / (double)(4 * n));
            }
            if (dir < 0) acc *= 2.0 / (double)n;
        } else if (type == 2 && dir > 0) {
            const long long period = 4 * n;   // angle unit pi/(2N)
            for (long long m = 0; m < n; ++m) {
                const long long a = ((2 * m + 1) * k) % period;
                acc += (double)x[m] * cospi((double)a / (double)(2 * n));
            }
        } else if (dir < 0) {   // type 2 or 3 inverse
            acc = 0.5 * (double)x[0];
            const long long period = 4 * n;
            for (long long m = 1; m < n; ++m) {
                const long long a = (m * (2 * k + 1)) % period;
                acc += (double)x[m] * cospi((double)a / (double)(2 * n));
            }
            acc *= 2.0 / (double)n;
        } else {   // type 3 forward
            acc = (double)x[0];
            const long long period = 4 * n;
            for (long long m = 1; m < n; ++m) {
                const long long a = (k * (2 * m + 1)) % period;
                acc += 2.0 * (double)x[m] * cospi((double)a / (double)(2 * n));
            }
        }
        out[i] = (float)acc;
    }
}

hipError_t launch_dct_naive(long long n, int type, int dir, const float* in, float* out, long long batch,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_dct_naive, dim3(nblocks(n * batch)), dim3(256), 0, s, n, type, dir, in, out, batch);
    return hipGetLastError();
}

// NaN/Inf policy (src/core/nan_policy.c): 0 propagate, 1 ignore (->0), 2 error (flag), 3 clamp
__global__ void k_nan_policy(float* p, long long count, int policy, int* flag) {
    GRID_STRIDE(i, count) {
        const float v = p[i];
        if (isfinite(v)) continue;
        if (policy == 1) p[i] = 0.0f;
        else if (policy == 2) atomicOr(flag, 1);
        else if (policy == 3) p[i] = isnan(v) ? 0.0f : (v > 0 ? 3.402823466e+38f : -3.402823466e+38f);
    }
}

hipError_t launch_nan_policy(float* p, long long count, int policy, int* flag, hipStream_t s) {
    if (policy == 0 || count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_nan_policy, dim3(nblocks(count)), dim3(256), 0, s, p, count, policy, flag);
    return hipGetLastError();
}

}  // namespace vvh
