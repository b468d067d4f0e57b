// phase_kernels.hip -- instantaneous phase and frequency of analytic rows.
//
// Reference: src/spectral/hilbert.c:77-113.
//   phase[0] = atan2(im0, re0); phase[i] = phase[i-1] + atan2(Im(z_i conj z_{i-1}),
//   Re(z_i conj z_{i-1})), every step in double, stored as float;
//   freq[0] = 0; freq[i] = (double(p[i]) - double(p[i-1])) * fs / (2 pi), stored as float.
//
// The phase is a prefix sum of per-sample increments, all in f64 as in the
// reference: a block of 256 threads owns PH_CHUNK = 4096 samples of a row
// (16 consecutive per thread), computes their increments, and scans them in
// three levels (thread-serial, block via LDS, row via the block totals of the
// first pass).  Only the association order of the f64 sum differs from the
// reference's left-to-right loop (errors ~1e-16 relative, far below the f32
// rounding of the output).  The frequency is elementwise and bit-identical.
// Both are HBM-bound: 8 B in + 4 B out per sample (phase), 4 + 4 (frequency).
#include "vvhip_internal.hpp"

namespace vvh {

constexpr int PH_T = 256, PH_PER = 16, PH_CHUNK = PH_T * PH_PER;

// increment at sample i of a row (i == 0: the principal phase of z_0)
__device__ __forceinline__ double phase_inc(const float2* z, long long i) {
    const float2 c = z[i];
    if (i == 0) return atan2((double)c.y, (double)c.x);
    const float2 p = z[i - 1];
    const double re = (double)c.x * (double)p.x + (double)c.y * (double)p.y;
    const double im = (double)c.y * (double)p.x - (double)c.x * (double)p.y;
    return atan2(im, re);
}

// vv_dsp_phase_unwrap (src/spectral/utils.c:63-73): out[0] = in[0], then the
// float difference of neighbours wrapped once by +-2 pi (float VV_DSP_PI /
// VV_DSP_TWO_PI), accumulated.  The increments are the reference's float
// values exactly; their sum runs in f64 (the reference sums in float left to
// right, so the two differ by that loop's own rounding, ~sqrt(n) ulp).
__device__ __forceinline__ double phase_inc(const float* p, long long i) {
    if (i == 0) return (double)p[0];
    const float kPi = (float)3.141592653589793238462643383279502884;
    const float kTwoPi = (float)(2.0 * 3.141592653589793238462643383279502884);
    float d = p[i] - p[i - 1];
    if (d > kPi) d -= kTwoPi;
    else if (d < -kPi) d += kTwoPi;
    return (double)d;
}

// block-inclusive scan of per-thread totals (256 doubles) in LDS; returns this
// thread's exclusive offset, *total the block's sum
__device__ __forceinline__ double block_excl_scan(double v, double* sh, double* total) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int off = 1; off < PH_T; off <<= 1) {
        const double a = t >= off ? sh[t - off] : 0.0;
        __syncthreads();
        sh[t] += a;
        __syncthreads();
    }
    *total = sh[PH_T - 1];
    const double ex = t > 0 ? sh[t - 1] : 0.0;
    __syncthreads();
    return ex;
}

// pass 1: block totals, part[row][blk]
template <class In>
__global__ void __launch_bounds__(PH_T) k_phase_part(const In* z, long long n, long long nblk, double* part) {
    __shared__ double sh[PH_T];
    const long long row = blockIdx.y, blk = blockIdx.x;
    const In* zr = z + row * n;
    const long long i0 = blk * PH_CHUNK + (long long)threadIdx.x * PH_PER;
    double s = 0.0;
#pragma unroll 4
    for (int k = 0; k < PH_PER; ++k)
        if (i0 + k < n) s += phase_inc(zr, i0 + k);
    double tot;
    (void)block_excl_scan(s, sh, &tot);
    if (threadIdx.x == 0) part[row * nblk + blk] = tot;
}

// pass 2: outputs = offset of the preceding blocks + block-exclusive + thread-serial sums
template <class In>
__global__ void __launch_bounds__(PH_T) k_phase_out(const In* z, long long n, long long nblk, const double* part,
                                                    float* phase) {
    __shared__ double sh[PH_T];
    const long long row = blockIdx.y, blk = blockIdx.x;
    const In* zr = z + row * n;
    // offset: sum of the preceding blocks' totals, in block order
    double off = 0.0;
    {
        double s = 0.0;
        for (long long b = threadIdx.x; b < blk; b += PH_T) s += part[row * nblk + b];
        double tot;
        (void)block_excl_scan(s, sh, &tot);
        off = tot;
    }
    const long long i0 = blk * PH_CHUNK + (long long)threadIdx.x * PH_PER;
    double d[PH_PER];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < PH_PER; ++k) {
        d[k] = i0 + k < n ? phase_inc(zr, i0 + k) : 0.0;
        s += d[k];
    }
    double tot;
    double acc = off + block_excl_scan(s, sh, &tot);
    float* pr = phase + row * n;
#pragma unroll
    for (int k = 0; k < PH_PER; ++k) {
        acc += d[k];
        if (i0 + k < n) pr[i0 + k] = (float)acc;
    }
}

__global__ void k_inst_freq(const float* p, long long n, long long total, double scale, float* f) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long k = i % n;
        if (k == 0) {
            f[i] = 0.0f;
        } else {
            const double dphi = (double)p[i] - (double)p[i - 1];
            f[i] = (float)(dphi * scale);
        }
    }
}

template <class In>
static hipError_t phase_scan(const In* z, long long n, long long batch, float* phase, hipStream_t s) {
    if (n <= 0 || batch <= 0) return hipSuccess;
    const long long nblk = (n + PH_CHUNK - 1) / PH_CHUNK;
    if (nblk > 0x7fffffffLL || batch > 65535) return hipErrorInvalidValue;
    double* part = nullptr;
    hipError_t e = hipMallocAsync((void**)&part, sizeof(double) * (size_t)(nblk * batch), s);
    if (e != hipSuccess) return e;
    const dim3 grid((unsigned)nblk, (unsigned)batch);
    hipLaunchKernelGGL((k_phase_part<In>), grid, dim3(PH_T), 0, s, z, n, nblk, part);
    hipLaunchKernelGGL((k_phase_out<In>), grid, dim3(PH_T), 0, s, z, n, nblk, part, phase);
    e = hipGetLastError();
    (void)hipFreeAsync(part, s);
    return e;
}

hipError_t launch_inst_phase(const float2* z, long long n, long long batch, float* phase, hipStream_t s) {
    return phase_scan(z, n, batch, phase, s);
}

hipError_t launch_phase_unwrap(const float* p, long long n, long long batch, float* out, hipStream_t s) {
    return phase_scan(p, n, batch, out, s);
}

hipError_t launch_inst_freq(const float* phase, long long n, long long batch, double scale, float* freq,
                            hipStream_t s) {
    const long long total = n * batch;
    if (total <= 0) return hipSuccess;
    long long b = (total + 255) / 256;
    if (b > 65536) b = 65536;
    hipLaunchKernelGGL(k_inst_freq, dim3((unsigned)b), dim3(256), 0, s, phase, n, total, scale, freq);
    return hipGetLastError();
}

}  // namespace vvh
