// framing_kernels.hip -- batched framing for gfx950: the frame gather of
// vv_dsp_fetch_frame and the overlap-add of vv_dsp_overlap_add
// (src/core/framing.c:58-146), many frames per launch.
//
// Both are HBM-bound data movement (4 B read + 4 B written per frame sample;
// overlapping frames re-read the signal from L2).  Results are bit-identical
// to the reference loops: the gather is a copy (times the window, one
// rounded multiply), and the overlap-add sums each output sample's
// contributions in increasing frame order, the order of a caller's loop over
// frame_index.
#include "vvhip_internal.hpp"

namespace vvh {

// framing.c:21-56 (reflection about the ends, period 2n for far indices)
__host__ __device__ __forceinline__ long long reflect_index(long long idx, long long n) {
    if (idx < 0) {
        long long a = -idx - 1;
        if (a >= n) {
            const long long period = 2 * n;
            a %= period;
            if (a >= n) a = period - 1 - a;
        }
        return a;
    }
    if (idx >= n) {
        long long r = n - 1 - (idx - n);
        if (r < 0) {
            r = -r - 1;
            if (r >= n) {
                const long long period = 2 * n;
                r %= period;
                if (r >= n) r = period - 1 - r;
            }
        }
        return r < 0 ? 0 : (r > n - 1 ? n - 1 : r);
    }
    return idx;
}

// frames [frame0, frame0 + count) -> out[count][len]; one thread per output sample.
// `sig` holds samples [base, ...) of the n-sample signal (base > 0: a host
// call uploads only the span one frame touches)
__global__ void __launch_bounds__(256) k_fetch_frames(const float* __restrict__ sig, long long base, long long n,
                                                      float* __restrict__ out, long long len, long long hop,
                                                      long long frame0, long long count, int center,
                                                      const float* __restrict__ win) {
    const long long total = count * len;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        const long long f = e / len, i = e - f * len;
        const long long start = (frame0 + f) * hop - (center ? len / 2 : 0);
        const long long k = start + i;
        float v;
        if (center) v = sig[reflect_index(k, n) - base];
        else v = (k < 0 || k >= n) ? 0.0f : sig[k - base];
        if (win) v = v * win[i];
        __builtin_nontemporal_store(v, out + e);
    }
}

// out[j] += frames[f][j - (frame0+f)*hop] for every frame covering j, in
// increasing f (the sequential loop's rounding), for j < out_len
__global__ void __launch_bounds__(256) k_overlap_add(const float* __restrict__ frames, long long count,
                                                     float* __restrict__ out, long long out_len, long long len,
                                                     long long hop, long long frame0, long long j0,
                                                     long long j1) {
    for (long long j = j0 + (long long)blockIdx.x * blockDim.x + threadIdx.x; j < j1;
         j += (long long)gridDim.x * blockDim.x) {
        // frames f (relative) with (frame0+f)*hop <= j < (frame0+f)*hop + len
        const long long rel = j - frame0 * hop;
        long long fhi = rel / hop;
        if (fhi > count - 1) fhi = count - 1;
        long long flo = rel - len + 1 <= 0 ? 0 : (rel - len + hop) / hop;
        float acc = out[j];
        for (long long f = flo; f <= fhi; ++f) acc += frames[f * len + (rel - f * hop)];
        out[j] = acc;
    }
}

long long reflect_sample(long long idx, long long n) { return reflect_index(idx, n); }

hipError_t launch_fetch_frames(const float* sig, long long base, long long n, float* out, long long len,
                               long long hop, long long frame0, long long count, int center, const float* win,
                               hipStream_t s) {
    const long long total = count * len;
    if (total <= 0) return hipSuccess;
    long long blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_fetch_frames, dim3((unsigned)blocks), dim3(256), 0, s, sig, base, n, out, len, hop, frame0,
                       count, center, win);
    return hipGetLastError();
}

hipError_t launch_overlap_add(const float* frames, long long count, float* out, long long out_len, long long len,
                              long long hop, long long frame0, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    const long long j0 = frame0 * hop;
    long long j1 = (frame0 + count - 1) * hop + len;
    if (j1 > out_len) j1 = out_len;
    if (j0 >= j1) return hipSuccess;
    long long blocks = (j1 - j0 + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_overlap_add, dim3((unsigned)blocks), dim3(256), 0, s, frames, count, out, out_len, len, hop,
                       frame0, j0, j1);
    return hipGetLastError();
}

}  // namespace vvh
