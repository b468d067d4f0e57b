// fft_kernels.hip -- batched C2C / R2C / C2R kernels for gfx950.
//
// Power-of-two lengths use the persistent register/LDS Stockham kernels of
// fft_core.hpp: each slot (a wave, or the whole block for N >= 2048) loops over
// transforms with the NEXT transform's points prefetched into a second register
// set, reading one transform with lane-contiguous loads and writing it with
// lane-contiguous stores: one HBM read + one HBM write per transform
// (8 B/point each way for C2C).  Twiddle tables live in LDS, so vmcnt only
// waits on streamed data.
//
// R2C of real length 2M runs an M-point complex FFT on z[m] = x[2m] + i x[2m+1]
// and the split step X[k] = Fe + W_{2M}^k (-i Fo) with Z[k] and Z[M-k] held in
// the same thread (mirror-paired last pass); C2R runs the inverse split step
// and an M-point inverse FFT.  Real transforms move 4 B/point.  Lengths that
// are not powers of two use an O(n^2) DFT kernel with f64 accumulation (the
// reference's own complexity for them: fft_kiss.c:76-92).
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

#include <cstdlib>

namespace vvh {

// ------------------------------------------------------------------------
// C2C
// ------------------------------------------------------------------------
// The exchange reads are single ds_read_b32 into the complex register pairs
// (pass_exchange_ri RIV 1; the compiler's ds_read2 pairs and v_movs measured
// 0.1850 vs 0.1827 ms on the same buffers, profiles/r04_kbench_riv_ab.jsonl).
// (Two transforms per loop trip with alternating prefetch buffers, to drop the
// loop-carried copy, spilled at the 128 VGPRs of four waves per SIMD.)  A grid-
// wide interleaved front: per-XCD eighths measured 0.1992 vs 0.1836 ms
// (profiles/r04_kbench_c2c_walk.jsonl).
// N = 1024 exchanges through the half-size real/imaginary buffer
// (pass_exchange_ri): 26 KB of LDS per workgroup instead of 43 KB, so four
// workgroups (16 waves) fit per CU and keep more transforms' loads in flight.
template <int N, bool FWD, bool ONE = false>
__global__ void __launch_bounds__(Wg<N>::value, (N == 1024 || (ONE && N >= 16 && N <= 128)) ? 4 : 1)
k_c2c(const float2* in, float2* out, long long batch, long long in_dist, long long out_dist,
      const float2* gpass, const float2* gtab, float scale) {
    using G = Geo<N>;
    constexpr int WG = Wg<N>::value, F = Wg<N>::F;
    constexpr bool RI = N == 1024;
    constexpr int XF = RI ? ri_floats<N>() / 2 : G::LDS;   // float2 per transform
    // ONE with 16..128 points: each wave's 1024-point block staged through LDS
    constexpr bool SMALL = ONE && G::T < 16 && G::P == 16;
    constexpr int LDSX = G::NPASS > 1 ? F * XF : 1, LDSN = SMALL && F * G::LDS > LDSX ? F * G::LDS : LDSX;
    __shared__ __attribute__((aligned(16))) float2 lds[LDSN];
    __shared__ float2 ltab[TwLayout<N>::ENTRIES];
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T;
    float2* my = lds + (G::NPASS > 1 ? slot * XF : 0);
    const TwTab<N> tw{ltab};
    const long long fend = batch;
    if constexpr (SMALL) {
        // small N (16..128): a wave's 64 / T transforms are 1024 consecutive points
        // (8 KB).  Lane-strided loads would touch 16..64 lines per instruction, so
        // the block moves as 16 B per lane, coalesced, and is re-laid through the
        // wave's LDS area (its slots' exchange buffers, padded 1 per 16) in both
        // directions.  The host takes this only for dense rows (dist == N).
        constexpr int WS = 64 / G::T;   // transforms per wave
        const int wv = lt >> 6, lane = lt & 63, sl = slot - wv * WS;
        const long long fw = (long long)blockIdx.x * F + (long long)wv * WS;   // the wave's first transform
        const long long nvl = fend - fw < WS ? fend - fw : WS;                   // its transforms in the batch
        const int nval = nvl > 0 ? (int)nvl * N : 0;                            // valid points of the block
        float2* wa = lds + wv * WS * G::LDS;                                    // the wave's LDS area
        stage_twiddles<N, WG>(ltab, gpass, gtab);
        __syncthreads();
        if (nval == 0) return;
        {
            vf4_t blk[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int e = i * 128 + 2 * lane;
                blk[i] = e < nval ? __builtin_nontemporal_load(reinterpret_cast<const vf4_t*>(in + fw * N + e))
                                  : vf4_t{0.0f, 0.0f, 0.0f, 0.0f};
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int e = i * 128 + 2 * lane;
                wa[G::pad(e)] = make_float2(blk[i][0], blk[i][1]);
                wa[G::pad(e + 1)] = make_float2(blk[i][2], blk[i][3]);
            }
        }
        xsync<64>();
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = wa[G::pad(sl * N + t + r * G::T)];
        xsync<64>();   // the FFT's exchanges reuse the area
        fft_regs<N, FWD, false, RI, TwTab<N>, false, false, 1>(v, t, my, tw);
        xsync<64>();
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            float2 o = v[q];
            if (!FWD) o = cscale(o, scale);
            wa[G::pad(sl * N + out_pos<N>(t, q))] = o;
        }
        xsync<64>();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int e = i * 128 + 2 * lane;
            if (e < nval) {
                const float2 a = wa[G::pad(e)], b = wa[G::pad(e + 1)];
                __builtin_nontemporal_store(vf4_t{a.x, a.y, b.x, b.y}, reinterpret_cast<vf4_t*>(out + fw * N + e));
            }
        }
        return;
    } else if constexpr (ONE) {
        // one transform per slot, no loop and no prefetch registers.  One-wave
        // transforms (N <= 1024) issue their loads before the block stages its
        // twiddles, so the load latency overlaps the staging: 1024 points 0.1815 ->
        // 0.1739 ms, 256 -1.8 %; for 2048 / 4096 (a transform over several waves)
        // that order measured +23 % / +2 %, so they load after the barrier
        // (profiles/r05_ab2_c2c_grid.jsonl)
        constexpr bool EARLY = G::T <= 64;
        const long long f = uni<G::T>((long long)blockIdx.x * F + slot);
        const bool act = f < fend;
        float2 v[G::P];
        if (EARLY && act) {
#pragma unroll
            for (int r = 0; r < G::P; ++r) v[r] = ld_nt(in + f * in_dist + t + r * G::T);
        }
        stage_twiddles<N, WG>(ltab, gpass, gtab);
        __syncthreads();
        if (!act) return;
        if constexpr (!EARLY) {
#pragma unroll
            for (int r = 0; r < G::P; ++r) v[r] = ld_nt(in + f * in_dist + t + r * G::T);
        }
        fft_regs<N, FWD, false, RI, TwTab<N>, false, false, 1>(v, t, my, tw);
        float2* dst = out + f * out_dist;
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            float2 o = v[q];
            if (!FWD) o = cscale(o, scale);
            st_nt(o, dst + out_pos<N>(t, q));
        }
        return;
    }
    stage_twiddles<N, WG>(ltab, gpass, gtab);
    __syncthreads();
    const long long stride = (long long)gridDim.x * F;
    long long f = uni<G::T>((long long)blockIdx.x * F + slot);
    float2 nx[G::P];
    if (f < fend) {
#pragma unroll
        for (int r = 0; r < G::P; ++r) nx[r] = ld_nt(in + f * in_dist + t + r * G::T);
    }
    for (; f < fend; f += stride) {
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = nx[r];
        const long long fn = f + stride;
        if (fn < fend) {
#pragma unroll
            for (int r = 0; r < G::P; ++r) nx[r] = ld_nt(in + fn * in_dist + t + r * G::T);
        }
        fft_regs<N, FWD, false, RI, TwTab<N>, false, false, 1>(v, t, my, tw);
        float2* dst = out + f * out_dist;
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            float2 o = v[q];
            if (!FWD) o = cscale(o, scale);
            st_nt(o, dst + out_pos<N>(t, q));
        }
    }
}

template <int N, bool FWD>
static hipError_t run_c2c(const float2* in, float2* out, long long batch, long long in_dist,
                          long long out_dist, float scale, hipStream_t s) {
    const float2* tab = twiddle_table(N);
    const float2* pas = pass_twiddles(N);
    if (!tab || !pas) return hipErrorOutOfMemory;
    constexpr int WG = Wg<N>::value, F = Wg<N>::F;
    static std::atomic<int> capc;
    const int grid_cap = cached_grid(capc, (const void*)k_c2c<N, FWD>, WG, 0, 1LL << 40);
    // 256 <= N <= 4096: one transform per wave slot, a grid of batch / F workgroups
    // (not persistent), so the dispatcher hands out the next workgroup as one ends:
    // config 2 (65536 x 1024) 0.1847 -> 0.1766 ms on the same buffers, 256 / 2048
    // points -3.6 / -4.5 %, 4096 -0.5 %; 64 points +10 % and 8192 +32 % keep the
    // persistent grid (profiles/r05_ab2_c2c_grid.jsonl).  Knob C2C_TPW = t > 0:
    // t transforms per wave slot; 0: the persistent grid (A/B)
    // 16..128 points with dense rows: the same one-transform grid, each wave's
    // 1024-point block moved as 16 B per lane and re-laid through LDS (k_c2c ONE,
    // G::T < 16): 32 / 64 / 128 points 0.650 / 0.332 / 0.230 -> 0.177 ms for 2^26
    // points (0.21 / 0.40 / 0.58 -> 0.76; profiles/r05_ab2_c2c_small.jsonl), bit-identical;
    // knob C2C_SMALL = 0 keeps the persistent grid (A/B)
    const bool small = N >= 16 && N <= 128 && in_dist == N && out_dist == N && ((uintptr_t)in & 15) == 0 &&
                       ((uintptr_t)out & 15) == 0 && knob(KNOB_C2C_SMALL, 1) == 1;
    const long long tpw = knob(KNOB_C2C_TPW, (N >= 256 && N <= 4096) || small ? 1 : -1);
    long long need = (batch + F - 1) / F, cap = grid_cap;
    if (tpw > 0) {
        need = (batch + F * tpw - 1) / (F * tpw);
        cap = 1LL << 30;
    }
    const int grid = (int)(need < cap ? need : cap);
    if (grid < 1) return hipSuccess;
    // one transform per slot: the loop-free kernel (no prefetch registers: 58 instead
    // of 98 VGPRs at 1024 points, 6 workgroups per CU): equal at 256 / 1024 points,
    // -1.3 % at 2048, -6.4 % at 4096 (profiles/r05_ab2_c2c_grid.jsonl); knob C2C_ONE = 0
    // keeps the looping kernel (A/B)
    // (two consecutive transforms per slot on this kernel measured +0.4 / +11 / +22 %
    // at 1024 / 2048 / 4096 points)
    if (tpw == 1 && need <= cap && knob(KNOB_C2C_ONE, 1) == 1 && (N >= 256 || small)) {   // (every slot's one transform in the grid)
        hipLaunchKernelGGL((k_c2c<N, FWD, true>), dim3(grid), dim3(WG), 0, s, in, out, batch, in_dist, out_dist, pas,
                           tab, scale);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((k_c2c<N, FWD>), dim3(grid), dim3(WG), 0, s, in, out, batch, in_dist, out_dist, pas, tab,
                       scale);
    return hipGetLastError();
}

// 8192: one workgroup of 512 threads per transform, the transform in 70 KB of
// LDS (gfx950 gives one workgroup up to 160 KB).  16384 would need 1024
// threads at <= 128 VGPRs and spills: it stays on the two-pass four-step.
bool c2c_supported(long long n) {
    const long long mx = knob(KNOB_C2C_MAX, 8192);   // A/B: 4096 sends 8192 to the two-pass four-step
    return n >= 2 && n <= mx && n <= 8192 && (n & (n - 1)) == 0;
}

hipError_t launch_c2c(long long n, int fwd, const float2* in, float2* out, long long batch,
                      long long in_dist, long long out_dist, float scale, hipStream_t s) {
#define VVH_C2C(NN)                                                                           \
    case NN:                                                                                  \
        return fwd ? run_c2c<NN, true>(in, out, batch, in_dist, out_dist, scale, s)           \
                   : run_c2c<NN, false>(in, out, batch, in_dist, out_dist, scale, s);
    switch (n) {
        VVH_C2C(2) VVH_C2C(4) VVH_C2C(8) VVH_C2C(16) VVH_C2C(32) VVH_C2C(64) VVH_C2C(128)
        VVH_C2C(256) VVH_C2C(512) VVH_C2C(1024) VVH_C2C(2048) VVH_C2C(4096) VVH_C2C(8192)
        default: return hipErrorInvalidValue;
    }
#undef VVH_C2C
}

// ------------------------------------------------------------------------
// R2C / C2R (real length 2M)
// ------------------------------------------------------------------------
template <int M>
__global__ void __launch_bounds__(Wg<M>::value)
k_r2c(const float* in, float2* out, long long batch, long long in_dist, long long out_dist,
      const float2* gpass, const float2* gtabM, const float2* gtab2M) {
    using G = Geo<M>;
    constexpr bool PAIR = G::CAN_PAIR;
    constexpr int WG = Wg<M>::value, F = Wg<M>::F;
    __shared__ float2 lds[F * G::LDS];
    __shared__ float2 ltab[TwLayout<M>::ENTRIES];
    __shared__ float2 lpost[PostLayout<M>::ENTRIES];
    stage_twiddles<M, WG>(ltab, gpass, gtabM);
    stage_post<M, WG>(lpost, gtab2M);
    __syncthreads();
    const TwTab<M> tw{ltab};
    const PostTab<M> pw{lpost};
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T;
    float2* my = lds + slot * G::LDS;
    long long stride = (long long)gridDim.x * F;
    long long f = uni<G::T>((long long)blockIdx.x * F + slot);
    long long fend = batch;
    float2 nx[G::P];
    if (f < fend) {
        const float2* src = reinterpret_cast<const float2*>(in + f * in_dist);
#pragma unroll
        for (int r = 0; r < G::P; ++r) nx[r] = ld_nt(src + t + r * G::T);
    }
    for (; f < fend; f += stride) {
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = nx[r];
        const long long fn = f + stride;
        if (fn < fend) {
            const float2* src = reinterpret_cast<const float2*>(in + fn * in_dist);
#pragma unroll
            for (int r = 0; r < G::P; ++r) nx[r] = ld_nt(src + t + r * G::T);
        }
        fft_regs<M, true, PAIR>(v, t, my, tw);
        float2* dst = out + f * out_dist;
        if constexpr (PAIR) {
#pragma unroll
            for (int q = 0; q < G::P; ++q) {
                const int k = out_pos<M, true>(t, q);
                const float2 A = v[q];
                if (k == 0) {
                    *(dst) = make_float2(A.x + A.y, 0.0f);
                    *(dst + M) = make_float2(A.x - A.y, 0.0f);
                } else {
                    *(dst + k) = split_fwd(A, cconj(mirror_of<M, true>(v, t, q)), pw(k));
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < G::P; ++q) my[G::pad(out_pos<M>(t, q))] = v[q];
            xsync<G::T>();
#pragma unroll
            for (int q = 0; q < G::P; ++q) {
                const int k = t + G::T * q;
                const float2 A = my[G::pad(k)];
                if (k == 0) {
                    *(dst) = make_float2(A.x + A.y, 0.0f);
                    *(dst + M) = make_float2(A.x - A.y, 0.0f);
                } else {
                    *(dst + k) = split_fwd(A, cconj(my[G::pad(M - k)]), pw(k));
                }
            }
            xsync<G::T>();
        }
    }
}

template <int M>
__global__ void __launch_bounds__(Wg<M>::value)
k_c2r(const float2* in, float* out, long long batch, long long in_dist, long long out_dist,
      const float2* gpass, const float2* gtabM, const float2* gtab2M, float scale) {
    using G = Geo<M>;
    constexpr int WG = Wg<M>::value, F = Wg<M>::F;
    __shared__ float2 lds[F * G::LDS];
    __shared__ float2 ltab[TwLayout<M>::ENTRIES];
    __shared__ float2 lpost[PostLayout<M>::ENTRIES];
    stage_twiddles<M, WG>(ltab, gpass, gtabM);
    stage_post<M, WG>(lpost, gtab2M);
    __syncthreads();
    const TwTab<M> tw{ltab};
    const PostTab<M> pw{lpost};
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T;
    float2* my = lds + slot * G::LDS;
    const long long stride = (long long)gridDim.x * F;
    long long f = uni<G::T>((long long)blockIdx.x * F + slot);
    float2 nx[G::P];
    float2 nxm = make_float2(0.0f, 0.0f);
    if (f < batch) {
        const float2* src = in + f * in_dist;
#pragma unroll
        for (int r = 0; r < G::P; ++r) nx[r] = ld_nt(src + t + r * G::T);
        nxm = src[M];
    }
    for (; f < batch; f += stride) {
        float2 xm = nxm;
#pragma unroll
        for (int r = 0; r < G::P; ++r) my[G::pad(t + r * G::T)] = nx[r];
        const long long fn = f + stride;
        if (fn < batch) {
            const float2* src = in + fn * in_dist;
#pragma unroll
            for (int r = 0; r < G::P; ++r) nx[r] = ld_nt(src + t + r * G::T);
            nxm = src[M];
        }
        xsync<G::T>();
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            const int k = t + r * G::T;
            float2 A = my[G::pad(k)];
            float2 B;
            if (k == 0) {   // imag of DC and Nyquist ignored (the fft_kiss.c:158-171 result)
                A.y = 0.0f;
                B = make_float2(xm.x, 0.0f);
            } else {
                B = my[G::pad(M - k)];
            }
            v[r] = split_inv(A, B, pw(k));
        }
        xsync<G::T>();
        fft_regs<M, false>(v, t, my, tw);
        float2* dst = reinterpret_cast<float2*>(out + f * out_dist);
#pragma unroll
        for (int q = 0; q < G::P; ++q) st_nt(cscale(v[q], scale), dst + out_pos<M>(t, q));
    }
}

// R2C of 32..128 real points (M = 16..64) with dense rows: the mirror of
// k_c2r_small -- each wave's 64 / T rows (1024 float2) loaded as 16 B per lane
// through its LDS area (padded 1 per 16), the FFT's bins back through the area
// for the split step's mirror, and the M + 1 bins per row staged and stored as
// 8 B per lane, coalesced.  A wave-uniform loop.
template <int M>
__global__ void __launch_bounds__(256, 4)
k_r2c_small(const float* __restrict__ in, float2* __restrict__ out, long long batch, const float2* gpass,
            const float2* gtabM, const float2* gtab2M) {
    using G = Geo<M>;
    static_assert(G::P == 16 && G::T <= 4, "M = 16..64");
    constexpr int F = 256 / G::T, WS = 64 / G::T, WA = WS * G::LDS;   // float2 per wave area
    static_assert(WS * (M + 1) <= WA && 1024 + 64 <= WA, "the wave area holds the rows and the bins");
    __shared__ __attribute__((aligned(16))) float2 lds[F * G::LDS];
    __shared__ float2 ltab[TwLayout<M>::ENTRIES];
    __shared__ float2 lpost[PostLayout<M>::ENTRIES];
    stage_twiddles<M, 256>(ltab, gpass, gtabM);
    stage_post<M, 256>(lpost, gtab2M);
    __syncthreads();
    const TwTab<M> tw{ltab};
    const PostTab<M> pw{lpost};
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T, wv = lt >> 6, lane = lt & 63, sl = slot - wv * WS;
    float2* my = lds + slot * G::LDS;
    float2* wa = lds + wv * WA;
    for (long long fw = (long long)blockIdx.x * F + (long long)wv * WS; fw < batch; fw += (long long)gridDim.x * F) {
        const long long nr = batch - fw < WS ? batch - fw : WS;
        const int nin = (int)nr * M, nout = (int)nr * (M + 1);   // valid input / output float2
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int e = i * 128 + 2 * lane;
            const vf4_t q = e < nin ? __builtin_nontemporal_load(reinterpret_cast<const vf4_t*>(in + 2 * (fw * M + e)))
                                    : vf4_t{0.0f, 0.0f, 0.0f, 0.0f};
            wa[G::pad(e)] = make_float2(q[0], q[1]);
            wa[G::pad(e + 1)] = make_float2(q[2], q[3]);
        }
        xsync<64>();
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = wa[G::pad(sl * M + t + r * G::T)];
        xsync<64>();   // the FFT's exchanges reuse the area
        fft_regs<M, true>(v, t, my, tw);
        xsync<64>();
#pragma unroll
        for (int q = 0; q < G::P; ++q) wa[G::pad(sl * M + out_pos<M>(t, q))] = v[q];
        xsync<64>();
        float2 o[G::P];
        float2 onyq = make_float2(0.0f, 0.0f);
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            const int k = t + r * G::T;
            const float2 A = wa[G::pad(sl * M + k)];
            if (k == 0) {
                o[r] = make_float2(A.x + A.y, 0.0f);
                onyq = make_float2(A.x - A.y, 0.0f);
            } else {
                o[r] = split_fwd(A, cconj(wa[G::pad(sl * M + M - k)]), pw(k));
            }
        }
        xsync<64>();
#pragma unroll
        for (int r = 0; r < G::P; ++r) wa[sl * (M + 1) + t + r * G::T] = o[r];
        if (t == 0) wa[sl * (M + 1) + M] = onyq;
        xsync<64>();
#pragma unroll
        for (int i = 0; i * 64 < WS * (M + 1); ++i) {
            const int e = i * 64 + lane;
            if (e < nout) st_nt(wa[e], out + fw * (M + 1) + e);
        }
        xsync<64>();
    }
}

template <int M>
static hipError_t run_r2c(const float* in, float2* out, long long batch, long long in_dist,
                          long long out_dist, hipStream_t s) {
    const float2* tM = twiddle_table(M);
    const float2* pM = pass_twiddles(M);
    const float2* t2M = twiddle_table(2 * M);
    if (!tM || !t2M || !pM) return hipErrorOutOfMemory;
    constexpr int WG = Wg<M>::value, F = Wg<M>::F;
    static std::atomic<int> capc;
    // one resident workgroup per CU: measured 15-20 % faster than the 3 the
    // LDS/VGPR budget allows (the partial-line n/2+1 rows combine better with
    // fewer concurrent writers; profiles/r01_kbench_occupancy.jsonl)
    const int cap = cached_grid(capc, (const void*)k_r2c<M>, WG, 0, 1LL << 40, 1);
    long long need = (batch + F - 1) / F;
    int grid = (int)(need < cap ? need : cap);
    // knob REAL_TPW = 1: one transform per slot, not persistent (A/B; 3.6 % slower
    // at 256 points, 9.8 % at 4096, equal at 1024: profiles/r05_ab2_real_grid.jsonl)
    if (knob(KNOB_REAL_TPW, 0) == 1) grid = (int)(need < (1LL << 30) ? need : (1LL << 30));
    if (grid < 1) return hipSuccess;
    if constexpr (M >= 16 && M <= 64) {
        // 32..128 real points, dense rows: the staged kernel -- 0.404 / 0.479 / 0.285 ->
        // 0.198 / 0.215 / 0.221 ms for 2^27 points, bit-identical
        // (profiles/r05_ab2_r2c_small.jsonl); knob R2C_SMALL = 0 keeps k_r2c (A/B)
        if (in_dist == 2 * M && out_dist == M + 1 && ((uintptr_t)in & 15) == 0 && knob(KNOB_R2C_SMALL, 1) == 1) {
            constexpr int FS = 256 / Geo<M>::T;
            const long long ns = (batch + FS - 1) / FS;
            hipLaunchKernelGGL(k_r2c_small<M>, dim3((unsigned)(ns < (1LL << 30) ? ns : (1LL << 30))), dim3(256), 0, s,
                               in, out, batch, pM, tM, t2M);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL(k_r2c<M>, dim3(grid), dim3(WG), 0, s, in, out, batch, in_dist, out_dist, pM, tM, t2M);
    return hipGetLastError();
}

// C2R of 32..128 real points (M = 16..64) with dense rows: k_c2r's arithmetic,
// each wave's 64 / T rows of M + 1 complex values loaded as 8 B per lane
// (coalesced) into its LDS area and read from there by the split step, and its
// real outputs (64 / T rows x 2M floats = 1024 float2) staged back (padded 1 per
// 16) and stored as 16 B per lane.  A wave-uniform loop.
template <int M>
__global__ void __launch_bounds__(256, 4)
k_c2r_small(const float2* __restrict__ in, float* __restrict__ out, long long batch, const float2* gpass,
            const float2* gtabM, const float2* gtab2M, float scale) {
    using G = Geo<M>;
    static_assert(G::P == 16 && G::T <= 4, "M = 16..64");
    constexpr int F = 256 / G::T, WS = 64 / G::T, WA = WS * G::LDS;   // float2 per wave area
    static_assert(WS * (M + 1) <= WA && 1024 + 64 <= WA, "the wave area holds the rows and the outputs");
    __shared__ __attribute__((aligned(16))) float2 lds[F * G::LDS];
    __shared__ float2 ltab[TwLayout<M>::ENTRIES];
    __shared__ float2 lpost[PostLayout<M>::ENTRIES];
    stage_twiddles<M, 256>(ltab, gpass, gtabM);
    stage_post<M, 256>(lpost, gtab2M);
    __syncthreads();
    const TwTab<M> tw{ltab};
    const PostTab<M> pw{lpost};
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T, wv = lt >> 6, lane = lt & 63, sl = slot - wv * WS;
    float2* my = lds + slot * G::LDS;
    float2* wa = lds + wv * WA;
    for (long long fw = (long long)blockIdx.x * F + (long long)wv * WS; fw < batch; fw += (long long)gridDim.x * F) {
        const long long nr = batch - fw < WS ? batch - fw : WS;
        const int nin = (int)nr * (M + 1), nout = (int)nr * M;   // valid input / output float2
#pragma unroll
        for (int i = 0; i * 64 < WS * (M + 1); ++i) {
            const int e = i * 64 + lane;
            if (e < WS * (M + 1)) wa[e] = e < nin ? in[fw * (M + 1) + e] : make_float2(0.0f, 0.0f);
        }
        xsync<64>();
        const float2* row = wa + sl * (M + 1);
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            const int k = t + r * G::T;
            float2 A = row[k], B;
            if (k == 0) {   // imag of DC and Nyquist ignored (the fft_kiss.c:158-171 result)
                A.y = 0.0f;
                B = make_float2(row[M].x, 0.0f);
            } else {
                B = row[M - k];
            }
            v[r] = split_inv(A, B, pw(k));
        }
        xsync<64>();   // the FFT's exchanges reuse the area
        fft_regs<M, false>(v, t, my, tw);
        xsync<64>();
#pragma unroll
        for (int q = 0; q < G::P; ++q) wa[G::pad(sl * M + out_pos<M>(t, q))] = cscale(v[q], scale);
        xsync<64>();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int e = i * 128 + 2 * lane;   // float2 index among the wave's outputs
            if (e < nout) {
                const float2 c0 = wa[G::pad(e)], c1 = wa[G::pad(e + 1)];
                __builtin_nontemporal_store(vf4_t{c0.x, c0.y, c1.x, c1.y},
                                            reinterpret_cast<vf4_t*>(out + 2 * (fw * M + e)));
            }
        }
        xsync<64>();
    }
}

template <int M>
static hipError_t run_c2r(const float2* in, float* out, long long batch, long long in_dist,
                          long long out_dist, hipStream_t s) {
    const float2* tM = twiddle_table(M);
    const float2* pM = pass_twiddles(M);
    const float2* t2M = twiddle_table(2 * M);
    if (!tM || !t2M || !pM) return hipErrorOutOfMemory;
    constexpr int WG = Wg<M>::value, F = Wg<M>::F;
    static std::atomic<int> capc;
    const int cap = cached_grid(capc, (const void*)k_c2r<M>, WG, 0, 1LL << 40);
    long long need = (batch + F - 1) / F;
    int grid = (int)(need < cap ? need : cap);
    // n <= 1024: one transform per slot, not persistent -- 256 points -6.1 %, 1024
    // -4.4 %, 4096 equal, bit-identical (profiles/r05_ab2_real_grid.jsonl); knob
    // REAL_TPW = 0 / 1 forces the persistent / one-per-slot grid (A/B)
    if (knob(KNOB_REAL_TPW, M <= 512 ? 1 : 0) == 1) grid = (int)(need < (1LL << 30) ? need : (1LL << 30));
    if (grid < 1) return hipSuccess;
    if constexpr (M >= 16 && M <= 64) {
        // 32..128 real points, dense rows: the staged kernel (knob REAL_SMALL = 0 keeps k_c2r, A/B)
        if (in_dist == M + 1 && out_dist == 2 * M && ((uintptr_t)out & 15) == 0 && knob(KNOB_REAL_SMALL, 1) == 1) {
            constexpr int FS = 256 / Geo<M>::T;
            const long long ns = (batch + FS - 1) / FS;
            hipLaunchKernelGGL(k_c2r_small<M>, dim3((unsigned)(ns < (1LL << 30) ? ns : (1LL << 30))), dim3(256), 0, s,
                               in, out, batch, pM, tM, t2M, 1.0f / (float)M);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL(k_c2r<M>, dim3(grid), dim3(WG), 0, s, in, out, batch, in_dist, out_dist, pM, tM, t2M,
                       1.0f / (float)M);
    return hipGetLastError();
}

// real 16384: the 8192-point complex kernel geometry (512 threads, 70 KB of LDS)
bool r2c_supported(long long n) {
    const long long mx = 2 * knob(KNOB_C2C_MAX, 8192);   // A/B: 4096 keeps real 16384 on the promote + four-step path
    return n >= 4 && n <= mx && n <= 16384 && (n & (n - 1)) == 0;
}

#define VVH_REAL_SWITCH(CALL)                                                                   \
    switch (n / 2) {                                                                            \
        case 2: return CALL(2); case 4: return CALL(4); case 8: return CALL(8);                 \
        case 16: return CALL(16); case 32: return CALL(32); case 64: return CALL(64);           \
        case 128: return CALL(128); case 256: return CALL(256); case 512: return CALL(512);     \
        case 1024: return CALL(1024); case 2048: return CALL(2048); case 4096: return CALL(4096); \
        case 8192: return CALL(8192);                                                           \
        default: return hipErrorInvalidValue;                                                   \
    }

hipError_t launch_r2c(long long n, const float* in, float2* out, long long batch, long long in_dist,
                      long long out_dist, hipStream_t s) {
#define CALL(MM) run_r2c<MM>(in, out, batch, in_dist, out_dist, s)
    VVH_REAL_SWITCH(CALL)
#undef CALL
}

hipError_t launch_c2r(long long n, const float2* in, float* out, long long batch, long long in_dist,
                      long long out_dist, hipStream_t s) {
#define CALL(MM) run_c2r<MM>(in, out, batch, in_dist, out_dist, s)
    VVH_REAL_SWITCH(CALL)
#undef CALL
}

// ------------------------------------------------------------------------
// O(n^2) DFT for arbitrary n (f64 accumulation, exact index reduction)
// ------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_dft_naive(long long n, int fwd, const void* in, int real_in, float2* out, long long nout,
            long long in_dist, long long out_dist, float scale, const double2* __restrict__ tab,
            long long kblocks) {
    __shared__ double2 tile[256];
    const long long f = (long long)blockIdx.x / kblocks;
    const long long k = ((long long)blockIdx.x % kblocks) * 256 + threadIdx.x;
    const float* rin = reinterpret_cast<const float*>(in) + (real_in ? f * in_dist : 0);
    const float2* cin = reinterpret_cast<const float2*>(in) + (real_in ? 0 : f * in_dist);
    double ar = 0.0, ai = 0.0;
    long long idx = 0;   // (k * t) mod n, advanced incrementally
    const long long kk = (k < n) ? k : 0;
    for (long long t0 = 0; t0 < n; t0 += 256) {
        const long long tt = t0 + threadIdx.x;
        if (tt < n) {
            if (real_in) tile[threadIdx.x] = make_double2((double)rin[tt], 0.0);
            else { const float2 c = cin[tt]; tile[threadIdx.x] = make_double2((double)c.x, (double)c.y); }
        }
        __syncthreads();
        const long long lim = (n - t0 < 256) ? (n - t0) : 256;
        for (long long j = 0; j < lim; ++j) {
            const double2 w = tab[idx];
            const double wi = fwd ? w.y : -w.y;
            const double2 x = tile[j];
            ar += x.x * w.x - x.y * wi;
            ai += x.x * wi + x.y * w.x;
            idx += kk;
            if (idx >= n) idx -= n;
        }
        __syncthreads();
    }
    if (k < nout) out[f * out_dist + k] = make_float2((float)(ar * scale), (float)(ai * scale));
}

hipError_t launch_dft_naive(long long n, int fwd, const void* in, int real_in, float2* out,
                            long long nout, long long batch, long long in_dist, long long out_dist,
                            float scale, hipStream_t s) {
    const double2* tab = twiddle_table_d(n);
    if (!tab) return hipErrorOutOfMemory;
    const long long kblocks = (nout + 255) / 256;
    if (kblocks * batch <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_dft_naive, dim3((unsigned)(kblocks * batch)), dim3(256), 0, s, n, fwd, in,
                       real_in, out, nout, in_dist, out_dist, scale, tab, kblocks);
    return hipGetLastError();
}

// ------------------------------------------------------------------------
// Real transforms above the fused kernels (pow2 n = 2M > 16384): the M-point
// complex transform of z[m] = x[2m] + i x[2m+1] (the real rows reinterpreted,
// no copy) and the split step, as k_r2c / k_c2r do in registers.  W_n^k from
// the two-level table lo[k & mask] * hi[k >> lo_bits].
// ------------------------------------------------------------------------
__device__ __forceinline__ float2 tw_split_at(const float2* __restrict__ tab, long long k, int lo_bits) {
    const long long mask = (1LL << lo_bits) - 1;
    return cmul(tab[k & mask], tab[(1LL << lo_bits) + (k >> lo_bits)]);
}

// Z: [batch][M] -> X: [batch][M+1] (bins 0..n/2 of the real rows).  Thread j of
// row f (blockIdx.y) makes bins j and M - j from the same two loads z[j], z[M-j]
// (each bin's twiddle from the table as before, so the bins are unchanged);
// 32-bit indices within a row.
__global__ void k_real_split_fwd(const float2* __restrict__ Z, float2* __restrict__ X, long long M, long long batch,
                                 const float2* __restrict__ tab, int lo_bits) {
    const int m = (int)M, h = m / 2;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > h) return;
    for (long long f = blockIdx.y; f < batch; f += gridDim.y) {
        const float2* z = Z + f * M;
        float2* x = X + f * (M + 1);
        const float2 a = z[j];
        if (j == 0) {   // DC and Nyquist (fft_kiss.c:141-143: imaginary part 0)
            x[0] = make_float2(a.x + a.y, 0.0f);
            x[m] = make_float2(a.x - a.y, 0.0f);
        } else if (j == h && 2 * h == m) {
            x[j] = split_fwd(a, cconj(a), tw_split_at(tab, j, lo_bits));
        } else {
            const float2 b = z[m - j];
            x[j] = split_fwd(a, cconj(b), tw_split_at(tab, j, lo_bits));
            x[m - j] = split_fwd(b, cconj(a), tw_split_at(tab, m - j, lo_bits));
        }
    }
}

// X: [batch][M+1] -> V: [batch][M], the inverse split (imaginary parts of DC and
// Nyquist ignored, the fft_kiss.c:158-171 result), before the M-point inverse;
// thread j makes V[j] and V[M-j] from x[j], x[M-j]
__global__ void k_real_split_inv(const float2* __restrict__ X, float2* __restrict__ V, long long M, long long batch,
                                 const float2* __restrict__ tab, int lo_bits) {
    const int m = (int)M, h = m / 2;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > h) return;
    for (long long f = blockIdx.y; f < batch; f += gridDim.y) {
        const float2* x = X + f * (M + 1);
        float2* v = V + f * M;
        float2 a = x[j];
        if (j == 0) {
            a.y = 0.0f;
            v[0] = split_inv(a, make_float2(x[m].x, 0.0f), tw_split_at(tab, 0, lo_bits));
        } else if (j == h && 2 * h == m) {
            v[j] = split_inv(a, a, tw_split_at(tab, j, lo_bits));
        } else {
            const float2 b = x[m - j];
            v[j] = split_inv(a, b, tw_split_at(tab, j, lo_bits));
            v[m - j] = split_inv(b, a, tw_split_at(tab, m - j, lo_bits));
        }
    }
}

static dim3 split_grid(long long M, long long batch) {
    const long long bx = (M / 2 + 1 + 255) / 256;
    return dim3((unsigned)bx, (unsigned)(batch < 65535 ? (batch < 1 ? 1 : batch) : 65535));
}

hipError_t launch_real_split_fwd(const float2* Z, float2* X, long long M, long long batch, hipStream_t s) {
    int lo_bits = 0;
    const float2* tab = twiddle_split(2 * M, &lo_bits);
    if (!tab) return hipErrorOutOfMemory;
    hipLaunchKernelGGL(k_real_split_fwd, split_grid(M, batch), dim3(256), 0, s, Z, X, M, batch, tab, lo_bits);
    return hipGetLastError();
}

hipError_t launch_real_split_inv(const float2* X, float2* V, long long M, long long batch, hipStream_t s) {
    int lo_bits = 0;
    const float2* tab = twiddle_split(2 * M, &lo_bits);
    if (!tab) return hipErrorOutOfMemory;
    hipLaunchKernelGGL(k_real_split_inv, split_grid(M, batch), dim3(256), 0, s, X, V, M, batch, tab, lo_bits);
    return hipGetLastError();
}

__global__ void k_herm_expand(long long n, const float2* half, float2* full, long long half_dist,
                              int zero_imag, long long total) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const long long f = i / n, k = i % n;
    const long long nh = n / 2 + 1;
    const float2* h = half + f * half_dist;
    float2 v;
    if (k < nh) {
        v = h[k];
        if (zero_imag && (k == 0 || (2 * k == n))) v.y = 0.0f;
    } else {
        const long long m = n - k;
        v = (m > 0 && m < nh) ? cconj(h[m]) : make_float2(0.0f, 0.0f);
    }
    full[i] = v;
}

hipError_t launch_hermitian_expand(long long n, const float2* half, float2* full, long long batch,
                                   long long half_dist, int zero_dc_nyq_imag, hipStream_t s) {
    const long long total = n * batch;
    hipLaunchKernelGGL(k_herm_expand, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, n, half,
                       full, half_dist, zero_dc_nyq_imag, total);
    return hipGetLastError();
}

__global__ void k_take_real(const float2* in, float* out, long long count) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) out[i] = in[i].x;
}

hipError_t launch_take_real(const float2* in, float* out, long long count, hipStream_t s) {
    hipLaunchKernelGGL(k_take_real, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, in, out, count);
    return hipGetLastError();
}

__global__ void k_zero_nyq(float2* out, long long n, long long batch, long long dist) {
    const long long f = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (f < batch) out[f * dist + n / 2].y = 0.0f;
}

hipError_t launch_zero_nyquist_imag(float2* out, long long n, long long batch, long long dist,
                                    hipStream_t s) {
    if (n % 2) return hipSuccess;
    hipLaunchKernelGGL(k_zero_nyq, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0, s, out, n, batch,
                       dist);
    return hipGetLastError();
}

__global__ void k_scale_r(float* p, long long count, float s) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) p[i] *= s;
}
__global__ void k_scale_c(float2* p, long long count, float s) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) p[i] = cscale(p[i], s);
}
hipError_t launch_scale_real(float* p, long long count, float s, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_scale_r, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, p, count, s);
    return hipGetLastError();
}
hipError_t launch_scale_cpx(float2* p, long long count, float s, hipStream_t st) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_scale_c, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, p, count, s);
    return hipGetLastError();
}

}  // namespace vvh
