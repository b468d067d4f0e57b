// spectral_utils_kernels.hip -- the data-format helpers of src/spectral/utils.c
// for gfx950, on `batch` contiguous rows:
//   fftshift / ifftshift (:5-49): out[j] = in[(j + k) mod n], k = n/2
//     (fftshift) or n - n/2 (ifftshift) -- a permutation copy, bit-exact;
//   phase_wrap (:51-61): x moved into (-pi, pi] by repeated +-2 pi in float,
//     the reference's loops verbatim -- bit-exact.
// (phase_unwrap, a prefix sum, is in phase_kernels.hip.)  HBM-bound copies.
#include "vvhip_internal.hpp"

namespace vvh {

static inline unsigned util_blocks(long long count) {
    long long b = (count + 255) / 256;
    if (b > 65536) b = 65536;
    if (b < 1) b = 1;
    return (unsigned)b;
}

template <class T>
__global__ void k_roll_rows(const T* __restrict__ in, T* __restrict__ out, long long n, long long k, long long total) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long r = i / n, j = i - r * n;
        long long src = j + k;
        if (src >= n) src -= n;
        out[i] = in[r * n + src];
    }
}

// inverse 0: fftshift, 1: ifftshift; complex rows of float2 when cpx
hipError_t launch_fftshift(const void* in, void* out, long long n, long long batch, int cpx, int inverse,
                           hipStream_t s) {
    const long long total = n * batch;
    if (total <= 0) return hipSuccess;
    const long long k = inverse ? n - n / 2 : n / 2;
    if (cpx)
        hipLaunchKernelGGL(k_roll_rows<float2>, dim3(util_blocks(total)), dim3(256), 0, s, (const float2*)in,
                           (float2*)out, n, k, total);
    else
        hipLaunchKernelGGL(k_roll_rows<float>, dim3(util_blocks(total)), dim3(256), 0, s, (const float*)in,
                           (float*)out, n, k, total);
    return hipGetLastError();
}

__global__ void k_phase_wrap(const float* __restrict__ in, float* __restrict__ out, long long total) {
    const float kPi = (float)3.141592653589793238462643383279502884;
    const float kTwoPi = (float)(2.0 * 3.141592653589793238462643383279502884);
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        float x = in[i];
        while (x <= -kPi) x += kTwoPi;
        while (x > kPi) x -= kTwoPi;
        out[i] = x;
    }
}

hipError_t launch_phase_wrap(const float* in, float* out, long long count, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_phase_wrap, dim3(util_blocks(count)), dim3(256), 0, s, in, out, count);
    return hipGetLastError();
}

}  // namespace vvh
