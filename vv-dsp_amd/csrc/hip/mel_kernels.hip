// mel_kernels.hip -- log-mel spectrogram and MFCC for gfx950 (src/features/mel.c).
//
// One wave per frame, frames walked grid-stride.  A frame's power row
// (n_fft/2+1 floats) is read once, coalesced, into LDS; lane m sums its
// triangular filter over the filter's non-zero bin range only (the reference
// also adds the zero weights outside it, which changes nothing: x + 0*p = x for
// finite non-negative power), in the reference's bin order with every product
// and sum separately rounded (mel.c:235-237), then takes logf(e + eps)
// (mel.c:240).  The MFCC kernel keeps the log-mel row in LDS and applies
// DCT-II (cos table rounded from double; dct.c:21-30 formula) and the lifter
// (factors computed on the host with mel.c:300-302's arithmetic).
// Filter weights, ranges, the DCT table and lifter factors are staged in LDS
// once per workgroup.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

namespace vvh {

// MODE 0: power rows -> log-mel rows; 1: power rows -> MFCC rows (fused);
// 2: log-mel rows -> MFCC rows (vv_dsp_mfcc)
template <int MODE>
__global__ void k_mel(const float* __restrict__ in, long long frames, int nbins, int n_mels, int n_coeffs,
                      const float* __restrict__ W, const int* __restrict__ meta, int nnz,
                      const float* __restrict__ D, const float* __restrict__ lift, float eps,
                      float* __restrict__ out, int waves_per_block, int row_floats) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int M = n_mels, C = n_coeffs;
    // LDS layout (must match launch_mel's size): the filter tables only when
    // the kernel sums filters, the DCT table and lifter only when it makes MFCC
    constexpr bool FILT = MODE != 2, DCT = MODE != 0;
    float* sW = smem;                                                  // nnz
    int* sMeta = reinterpret_cast<int*>(sW + (FILT ? nnz : 0));        // 3*M: lo, len, off
    float* sD = reinterpret_cast<float*>(sMeta + (FILT ? 3 * M : 0));  // C*M
    float* sL = sD + (DCT ? C * M : 0);                                // C
    float* wave_base = sL + (DCT ? C : 0);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float* row = wave_base + wv * (row_floats + M);     // power row (or log-mel row for MODE 2)
    float* lm = row + row_floats;                       // log-mel row
    if constexpr (MODE != 2) {
        for (int i = threadIdx.x; i < nnz; i += blockDim.x) sW[i] = W[i];
        for (int i = threadIdx.x; i < 3 * M; i += blockDim.x) sMeta[i] = meta[i];
    }
    if constexpr (MODE != 0) {
        for (int i = threadIdx.x; i < C * M; i += blockDim.x) sD[i] = D[i];
        for (int i = threadIdx.x; i < C; i += blockDim.x) sL[i] = lift[i];
    }
    __syncthreads();
    const int in_len = MODE == 2 ? M : nbins;
    const long long stride = (long long)gridDim.x * waves_per_block;
    for (long long f = (long long)blockIdx.x * waves_per_block + wv; f < frames; f += stride) {
        const float* src = in + f * in_len;
        float* dst_row = MODE == 2 ? lm : row;
        for (int k = lane; k < in_len; k += 64) dst_row[k] = src[k];
        xsync<64>();
        if constexpr (MODE != 2) {
            for (int m = lane; m < M; m += 64) {
                const int lo = sMeta[3 * m], len = sMeta[3 * m + 1], off = sMeta[3 * m + 2];
                float e = 0.0f;
                for (int j = 0; j < len; ++j) {
                    float pr = row[lo + j] * sW[off + j];
                    asm volatile("" : "+v"(pr));   // keep mul and add separately rounded (no FMA)
                    e = e + pr;
                }
                const float v = logf(e + eps);
                if constexpr (MODE == 0) out[f * M + m] = v;
                else lm[m] = v;
            }
        }
        if constexpr (MODE != 0) {
            xsync<64>();
            for (int i = lane; i < C; i += 64) {
                float c = 0.0f;
                for (int m = 0; m < M; ++m) c = __builtin_fmaf(lm[m], sD[i * M + m], c);
                out[f * C + i] = c * sL[i];
            }
        }
        xsync<64>();   // the next frame overwrites this wave's rows
    }
}

hipError_t launch_mel(int mode, const float* in, long long frames, int nbins, int n_mels, int n_coeffs,
                      const float* W, const int* meta, int nnz, const float* D, const float* lift, float eps,
                      float* out, hipStream_t s) {
    if (frames <= 0) return hipSuccess;
    const int row_floats = mode == 2 ? 0 : ((nbins + 3) & ~3);
    const size_t shared = sizeof(float) * ((mode == 2 ? 0 : (size_t)nnz + 3 * (size_t)n_mels) +
                                           (mode == 0 ? 0 : (size_t)n_coeffs * n_mels + n_coeffs));
    const size_t per_wave = sizeof(float) * (size_t)(row_floats + n_mels);
    const size_t budget = 64 * 1024;
    int wpb = 4;
    while (wpb > 1 && shared + wpb * per_wave > budget) --wpb;
    const size_t lds = shared + wpb * per_wave;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    long long blocks = (frames + wpb - 1) / wpb;
    if (blocks > 4096) blocks = 4096;
    const dim3 grid((unsigned)blocks), block(64 * wpb);
#define L(MM)                                                                                                  \
    hipLaunchKernelGGL(k_mel<MM>, grid, block, lds, s, in, frames, nbins, n_mels, n_coeffs, W, meta, nnz, D, \
                       lift, eps, out, wpb, row_floats)
    if (mode == 0) L(0);
    else if (mode == 1) L(1);
    else L(2);
#undef L
    return hipGetLastError();
}

}  // namespace vvh
