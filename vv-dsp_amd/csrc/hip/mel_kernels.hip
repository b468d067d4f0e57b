// mel_kernels.hip -- log-mel spectrogram and MFCC for gfx950 (src/features/mel.c).
//
// Default: k_mel_grp (below) -- FR = 4 frames per wave step, their power rows
// (one contiguous block of the input) brought into LDS by 16 B LDS-DMA, the
// filters' non-zero ranges cut into balanced chunks over the 64 lanes, then
// logf(e + eps) (mel.c:240), and for MFCC the DCT-II (cos table rounded from
// double; dct.c:21-30 formula) and lifter (mel.c:298-304) over (frame,
// coefficient) lanes.  Filter weights, chunk table, the DCT table and lifter
// factors are staged in LDS once per workgroup.
//
// Round 1's one-wave-per-frame kernel (lane m summing its whole filter) is
// gone: a wave waited for its widest filter and for each row load in turn.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

#include <vector>

namespace vvh {

// ------------------------------------------------------------------------
// k_mel_grp<MODE, FR>: FR frames per wave step, work balanced across lanes.
// A one-wave-per-frame kernel gives lane m the whole filter m, so a
// wave takes as long as the widest filter (mel filters widen with frequency:
// ~92 bins for the top filter of a 40-mel bank at 48 kHz / 1024 points, ~26 on
// average) with most lanes idle, and every lane's sum is one dependent chain.
// Here the host cuts each filter's non-zero range into chunks of at most Lc
// bins (Lc chosen so that the chunks fill whole rounds of 64 lanes), lane c
// sums chunk c for FR frames at once (FR independent FMA chains sharing each
// weight read), and lane m then adds its filter's chunk partials in order
// and takes logf(e + eps).  The MFCC step spreads (frame, coefficient) pairs
// over the lanes.  The rows of FR consecutive frames are one contiguous block
// of the input, copied into LDS with coalesced dword loads.
// Not bit-identical to mel.c's single running sum per filter (the chunk sums
// are added at the end, and products are fused): within a few ulp.
// ------------------------------------------------------------------------
template <int MODE, int FR>
__global__ void __launch_bounds__(256)
k_mel_grp(const float* __restrict__ in, long long frames, int in_len, int n_mels, int n_coeffs,
          const float* __restrict__ W, int nnz, const int* __restrict__ chunks, int nc,
          const int* __restrict__ cbeg, const float* __restrict__ D, const float* __restrict__ lift, float eps,
          float* __restrict__ out, int waves_per_block, int row_floats, int dma, int row_len) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr bool FILT = MODE != 2, DCT = MODE != 0;
    const int M = n_mels, C = n_coeffs;
    float* sW = smem;                                                   // nnz
    int* sCh = reinterpret_cast<int*>(sW + (FILT ? nnz : 0));           // 3*nc: lo, len, off
    int* sCb = sCh + (FILT ? 3 * nc : 0);                               // M+1
    // the DCT table, the per-wave areas and the log-mel rows start 16 B aligned
    // (float4 reads in the DCT); the host sizes the shared part the same way
    const int dpos = ((FILT ? nnz + 3 * nc + M + 1 : 0) + 3) & ~3;
    float* sD = smem + dpos;                                            // C*M
    float* sL = sD + (DCT ? C * M : 0);                                 // C
    float* wave_base = smem + ((dpos + (DCT ? C * M + C : 0) + 3) & ~3);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int part_floats = FILT ? (FR * nc + 3) & ~3 : 0;
    const int per_wave = row_floats + part_floats + (MODE == 1 ? FR * M : 0);
    float* row = wave_base + wv * per_wave;                             // FR input rows (row_floats >= FR*in_len)
    float* part = row + row_floats;                                     // [FR][nc] chunk sums
    float* lm = MODE == 2 ? row : part + part_floats;                   // [FR][M] log-mel rows
    if constexpr (FILT) {
        for (int i = threadIdx.x; i < nnz; i += blockDim.x) sW[i] = W[i];
        for (int i = threadIdx.x; i < 3 * nc; i += blockDim.x) sCh[i] = chunks[i];
        for (int i = threadIdx.x; i <= M; i += blockDim.x) sCb[i] = cbeg[i];
    }
    if constexpr (DCT) {
        for (int i = threadIdx.x; i < C * M; i += blockDim.x) sD[i] = D[i];
        for (int i = threadIdx.x; i < C; i += blockDim.x) sL[i] = lift[i];
    }
    __syncthreads();
    const long long groups = (frames + FR - 1) / FR;
    const long long stride = (long long)gridDim.x * waves_per_block;
    for (long long g = (long long)blockIdx.x * waves_per_block + wv; g < groups; g += stride) {
        const long long f0 = g * FR;
        const int nf = (int)(frames - f0 < FR ? frames - f0 : FR);
        // FR consecutive rows = one contiguous block (rows in_len floats apart, the
        // last one read up to its row_len data floats only); missing rows read as 0
        const float* src = in + f0 * in_len;
        const int valid = (nf - 1) * in_len + row_len;
        if (dma && nf == FR && (g + 1 < groups || (valid & 3) == 0)) {
            // full group: HBM -> LDS by 16 B/lane LDS-DMA, every piece in flight
            // at once (a load-then-store loop would serialise on each load)
            for (int u = 0; u * 256 < valid; ++u) {
                const int e = u * 256 + lane * 4;
                glds16(src + (e < valid ? e : 0), row + u * 256);
            }
            vm_wait<0>();
        } else {
            constexpr int U = 8;
            for (int b = 0; b < FR * in_len; b += 64 * U) {
                float r[U];
#pragma unroll
                for (int k = 0; k < U; ++k) {
                    const int e = b + lane + 64 * k;
                    r[k] = e < valid ? src[e] : 0.0f;
                }
#pragma unroll
                for (int k = 0; k < U; ++k) {
                    const int e = b + lane + 64 * k;
                    if (e < FR * in_len) row[e] = r[k];
                }
            }
        }
        xsync<64>();
        if constexpr (FILT) {
            for (int c = lane; c < nc; c += 64) {
                const int lo = sCh[3 * c], len = sCh[3 * c + 1], off = sCh[3 * c + 2];
                float acc[FR];
#pragma unroll
                for (int f = 0; f < FR; ++f) acc[f] = 0.0f;
#pragma unroll 4
                for (int j = 0; j < len; ++j) {
                    const float w = sW[off + j];
#pragma unroll
                    for (int f = 0; f < FR; ++f) acc[f] = __builtin_fmaf(row[f * in_len + lo + j], w, acc[f]);
                }
#pragma unroll
                for (int f = 0; f < FR; ++f) part[f * nc + c] = acc[f];
            }
            xsync<64>();
            for (int m = lane; m < M; m += 64) {
                const int cb = sCb[m], ce = sCb[m + 1];
#pragma unroll
                for (int f = 0; f < FR; ++f) {
                    float e = 0.0f;
                    for (int c = cb; c < ce; ++c) e += part[f * nc + c];
                    const float v = logf(e + eps);
                    if constexpr (MODE == 0) {
                        if (f < nf) out[(f0 + f) * M + m] = v;
                    } else {
                        lm[f * M + m] = v;
                    }
                }
            }
        }
        if constexpr (DCT) {
            xsync<64>();
            for (int idx = lane; idx < nf * C; idx += 64) {
                const int f = idx / C, i = idx - f * C;
                const float* l = lm + f * M;
                const float* d = sD + i * M;
                float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f, c3 = 0.0f;
                int m = 0;
                if ((M & 3) == 0) {   // 16 B LDS reads: a quarter of the read instructions
                    for (; m < M; m += 4) {
                        const vf4_t a = *reinterpret_cast<const vf4_t*>(l + m);
                        const vf4_t b = *reinterpret_cast<const vf4_t*>(d + m);
                        c0 = __builtin_fmaf(a[0], b[0], c0);
                        c1 = __builtin_fmaf(a[1], b[1], c1);
                        c2 = __builtin_fmaf(a[2], b[2], c2);
                        c3 = __builtin_fmaf(a[3], b[3], c3);
                    }
                } else {
                    for (; m + 1 < M; m += 2) {
                        c0 = __builtin_fmaf(l[m], d[m], c0);
                        c1 = __builtin_fmaf(l[m + 1], d[m + 1], c1);
                    }
                    if (m < M) c0 = __builtin_fmaf(l[m], d[m], c0);
                }
                out[f0 * C + idx] = ((c0 + c1) + (c2 + c3)) * sL[i];
            }
        }
        xsync<64>();   // the next group overwrites this wave's rows
    }
}

// Chunk schedule of the filters' non-zero ranges (host): chunks of at most Lc
// bins, Lc minimising rounds(64 lanes) x Lc.  chunks = {lo, len, off} per chunk;
// cbeg[m] .. cbeg[m+1] are filter m's chunks (an empty filter has none).
int mel_chunk_schedule(const int* meta, int n_mels, std::vector<int>* chunks, std::vector<int>* cbeg) {
    int best_lc = 1, best_cost = -1;
    int maxlen = 1;
    for (int m = 0; m < n_mels; ++m) maxlen = meta[3 * m + 1] > maxlen ? meta[3 * m + 1] : maxlen;
    for (int lc = 4; lc < 2 * maxlen + 4; lc += 4) {
        long long nc = 0;
        for (int m = 0; m < n_mels; ++m) nc += (meta[3 * m + 1] + lc - 1) / lc;
        const long long rounds = (nc + 63) / 64;
        const long long cost = rounds * (lc + 8);   // + per-round overhead
        if (best_cost < 0 || cost < best_cost) {
            best_cost = (int)cost;
            best_lc = lc;
        }
        if (lc >= maxlen) break;
    }
    chunks->clear();
    cbeg->assign(n_mels + 1, 0);
    for (int m = 0; m < n_mels; ++m) {
        (*cbeg)[m] = (int)(chunks->size() / 3);
        const int lo = meta[3 * m], len = meta[3 * m + 1], off = meta[3 * m + 2];
        for (int j = 0; j < len; j += best_lc) {
            chunks->push_back(lo + j);
            chunks->push_back(len - j < best_lc ? len - j : best_lc);
            chunks->push_back(off + j);
        }
    }
    (*cbeg)[n_mels] = (int)(chunks->size() / 3);
    return best_lc;
}

hipError_t launch_mel_grp(int mode, const float* in, long long frames, int nbins, int n_mels, int n_coeffs,
                          const float* W, int nnz, const int* chunks, int nc, const int* cbeg, const float* D,
                          const float* lift, float eps, float* out, hipStream_t s, int in_pitch) {
    if (frames <= 0) return hipSuccess;
    const bool filt = mode != 2, dct = mode != 0;
    // floats per input row: power rows may sit in_pitch apart (a group of FR rows
    // is still one contiguous block; the pad floats come along and are never read)
    const int in_len = mode == 2 ? n_mels : (in_pitch > 0 ? in_pitch : nbins);
    // layout as in k_mel_grp: DCT table and per-wave areas 16 B aligned
    const size_t dpos = ((filt ? (size_t)nnz + 3 * (size_t)nc + n_mels + 1 : 0) + 3) & ~(size_t)3;
    const size_t shared = sizeof(float) * ((dpos + (dct ? (size_t)n_coeffs * n_mels + n_coeffs : 0) + 3) & ~(size_t)3);
    // frames per wave step: 4, fewer when the rows are long
    int fr = 4;
    // row area: whole 256-float LDS-DMA pieces
    auto row_floats = [&](int f) { return (f * in_len + 255) / 256 * 256; };
    auto per_wave = [&](int f) {
        return sizeof(float) * (size_t)(row_floats(f) + (filt ? (f * nc + 3) & ~3 : 0) + (mode == 1 ? f * n_mels : 0));
    };
    while (fr > 1 && per_wave(fr) > 16 * 1024) fr >>= 1;
    int wpb = 4;
    while (wpb > 1 && shared + wpb * per_wave(fr) > 64 * 1024) --wpb;
    const size_t lds = shared + wpb * per_wave(fr);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    const long long groups = (frames + fr - 1) / fr;
    // LDS-DMA needs 16 B aligned group blocks: base aligned, fr * in_len a multiple of 4
    const int dma = ((uintptr_t)in & 15) == 0 && (fr * in_len) % 4 == 0;
    long long blocks = (groups + wpb - 1) / wpb;
    if (blocks > 8192) blocks = 8192;
    const dim3 grid((unsigned)blocks), block(64 * wpb);
#define L(MM, FF)                                                                                            \
    hipLaunchKernelGGL((k_mel_grp<MM, FF>), grid, block, lds, s, in, frames, in_len, n_mels, n_coeffs, W, nnz, \
                       chunks, nc, cbeg, D, lift, eps, out, wpb, row_floats(FF), dma, mode == 2 ? in_len : nbins)
#define LF(MM) \
    if (fr == 4) L(MM, 4); else if (fr == 2) L(MM, 2); else L(MM, 1);
    if (mode == 0) { LF(0) }
    else if (mode == 1) { LF(1) }
    else { LF(2) }
#undef LF
#undef L
    return hipGetLastError();
}

}  // namespace vvh
