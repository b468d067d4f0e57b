// fir_kernels.hip -- FFT-domain FIR (overlap-save) for gfx950.
//
// vv_dsp_fir_apply_fft (src/filter/fir.c:75-135) is "the first n samples of the
// linear convolution with zero initial state"; vv_dsp_fir_apply (:160-196) is
// the same convolution continued from a (taps-1)-sample history.  Both are
// computed here as overlap-save with blocks of N real samples and an
// effective history LE >= taps-1 (the filter read as zero-padded to LE+1 taps,
// which changes nothing; LE is a multiple of 4 and >= N/4 so that block starts
// are 16 B aligned and a pair's input span fits its LDS buffer):
//
//   block j of channel c covers input samples [j*Lout - LE, j*Lout + Lout)
//   (Lout = N - LE); samples before 0 come from `prefix` (history) or are 0;
//   outputs j*Lout + [0, Lout) are the block's circular-convolution samples
//   LE .. N-1.
//
// Two real blocks per complex FFT: z = a + i b (blocks j and j+1), then
// Y = FFT(z) * H with H = FFT(h)/N over all N bins, and y = IFFT(Y) holds
// a*h in its real part and b*h in its imaginary part (h is real, so the
// product keeps the two convolutions apart -- no split step).  After the
// forward Stockham FFT thread t holds Z[t + T*m] for m < P, which is exactly
// the input set of the inverse transform: the multiply by H re-indexes
// registers and no LDS re-order is needed between the two transforms.
//
// k_fir_pair<N, true>  (bulk, T >= 64): the pair's input span comes HBM -> LDS
//   by 16 B/lane LDS-DMA issued one pair ahead with a hand-counted vmcnt;
//   outputs are dword stores of which lanes below LE go to a write sink, so
//   every pair issues exactly 2P stores.
// k_fir_pair<N, false> (edges and small N): register loads with the prefix /
//   zero padding, predicated stores.
// HBM traffic: the signal read once (the LE overlap comes from L2/LDS), the
// output written once -- 8 B per sample.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

#include <cstdint>
#include <cstdlib>

namespace vvh {

// samples s0 + t + r*T of one block (prefix before 0 -- only its last lm1
// samples exist, earlier ones meet zero taps -- and zero past n)
template <int N>
__device__ __forceinline__ void fir_blk_load(float* xr, const float* xs, const float* pre, long long s0,
                                             long long n, long long lm1, int t) {
    using G = Geo<N>;
    if (s0 >= 0 && s0 + N <= n) {
        const float* b = xs + s0;
#pragma unroll
        for (int r = 0; r < G::P; ++r) xr[r] = b[t + r * G::T];
    } else {
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            const long long i = s0 + t + r * G::T;
            float v = 0.0f;
            if (i < 0) {
                if (pre && i >= -lm1) v = pre[lm1 + i];
            } else if (i < n) {
                v = xs[i];
            }
            xr[r] = v;
        }
    }
}

// Y = Z * H with the register re-index forward-output -> inverse-input
template <int N>
__device__ __forceinline__ void fir_multiply(const float2* v, float2* u, const float2* lH, int t) {
    using G = Geo<N>;
#pragma unroll
    for (int q = 0; q < G::P; ++q) {
        const int m = q / G::RL + G::NPT * (q % G::RL);   // out_pos<N>(t, q) = t + T*m
        u[m] = cmul(v[q], lH[t + G::T * m]);
    }
}

// Pairs of channel c handled by a launch: idx < qlo -> pair idx, else pair
// qhi + (idx - qlo); cnt = pairs per channel in this launch.
template <int N, bool BULK>
__global__ void __launch_bounds__(Wg<N>::value)
k_fir_pair(long long lm1, long long le, const float2* Hg, const float* x, float* y, long long n,
           long long nch, long long x_stride, long long y_stride, const float* prefix, long long cnt,
           long long qlo, long long qhi, const float2* gpass, const float2* gtab, float* sink, long long chunk) {
    using G = Geo<N>;
    constexpr int WG = Wg<N>::value, F = Wg<N>::F;
    constexpr int SPAN = BULK ? N + (3 * N) / 4 : 1;   // N + Lout, Lout <= 3N/4
    constexpr int NST = 2 * G::P;                      // stores per pair (bulk)
    static_assert(!BULK || G::T >= 64, "LDS-DMA spans need whole waves per transform");
    __shared__ float2 lds[F * G::LDS];
    __shared__ float2 ltab[TwLayout<N>::ENTRIES];
    __shared__ float2 lH[N];
    __shared__ float span_all[BULK ? F * SPAN : 1];
    stage_twiddles<N, WG>(ltab, gpass, gtab);
    for (int i = threadIdx.x; i < N; i += WG) lH[i] = Hg[i];
    __syncthreads();
    const TwTab<N> tw{ltab};
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T;
    float2* my = lds + slot * G::LDS;
    const long long lout = N - le;
    long long p, p_end, p_step;
    work_walk(nch * cnt, F, slot, chunk, &p, &p_end, &p_step);
    p = uni<G::T>(p);
    p_end = uni<G::T>(p_end);
    p_step = uni<G::T>(p_step);
    if (p >= p_end) return;   // uniform per transform (F == 1 whenever T > 64)
    // item -> (channel, first block of the pair)
    auto locate = [&](long long it, long long* cc, long long* jj) {
        *cc = it / cnt;
        const long long i = it - *cc * cnt;
        *jj = 2 * (i < qlo ? i : qhi + (i - qlo));
    };
    long long c, j;
    locate(p, &c, &j);
    if constexpr (BULK) {
        float* span = span_all + slot * SPAN;
        float* snk = sink + ((((long long)blockIdx.x * (WG / 64) + (lt >> 6)) * 64) % SINK_FLOATS) + (lt & 63);
        auto issue_span = [&](long long cc, long long jj) {
            const float* s0 = x + cc * x_stride + jj * lout - le;
            const int len = (int)(N + lout), lane = t & 63;
            for (int u = t >> 6; u * 256 < len; u += G::T / 64) {
                const int e = u * 256 + lane * 4;
                glds16(s0 + (e < len ? e : 0), span + u * 256);
            }
        };
        issue_span(c, j);
        vm_wait<0>();
        for (; p < p_end; p += p_step) {
            const bool more = p + p_step < p_end;
            long long cn = c, jn = j;
            if (more) locate(p + p_step, &cn, &jn);
            vm_wait<NST>();   // younger than this span's DMA: the previous pair's stores
            if constexpr (G::T > 64) lds_barrier();
            float2 v[G::P];
#pragma unroll
            for (int r = 0; r < G::P; ++r) v[r] = make_float2(span[t + r * G::T], span[lout + t + r * G::T]);
            lgkm_wait0();
            if constexpr (G::T > 64) lds_barrier();
            if (more) issue_span(cn, jn);
            fft_regs<N, true>(v, t, my, tw);
            float2 u[G::P];
            fir_multiply<N>(v, u, lH, t);
            fft_regs<N, false>(u, t, my, tw);
            float* ya = y + c * y_stride + j * lout - le;   // + e: block j output (e >= le)
#pragma unroll
            for (int q = 0; q < G::P; ++q) {
                const long long e = out_pos<N>(t, q);
                const bool ok = e >= le;
                st4_counted(ok ? ya + e : snk, u[q].x);
                st4_counted(ok ? ya + e + lout : snk, u[q].y);
            }
            c = cn;
            j = jn;
        }
    } else {
        float xa[G::P], xb[G::P];
        auto load_pair = [&](long long cc, long long jj) {
            const float* xs = x + cc * x_stride;
            const float* pre = prefix ? prefix + cc * lm1 : nullptr;
            fir_blk_load<N>(xa, xs, pre, jj * lout - le, n, lm1, t);
            fir_blk_load<N>(xb, xs, pre, (jj + 1) * lout - le, n, lm1, t);
        };
        load_pair(c, j);
        for (; p < p_end; p += p_step) {
            float2 v[G::P];
#pragma unroll
            for (int r = 0; r < G::P; ++r) v[r] = make_float2(xa[r], xb[r]);
            const bool more = p + p_step < p_end;
            long long cn = c, jn = j;
            if (more) {
                locate(p + p_step, &cn, &jn);
                load_pair(cn, jn);
            }
            fft_regs<N, true>(v, t, my, tw);
            float2 u[G::P];
            fir_multiply<N>(v, u, lH, t);
            fft_regs<N, false>(u, t, my, tw);
            float* ys = y + c * y_stride;
            const long long oa0 = j * lout - le;
#pragma unroll
            for (int q = 0; q < G::P; ++q) {
                const long long e = out_pos<N>(t, q);
                if (e >= le) {
                    const long long oa = oa0 + e, ob = oa + lout;
                    if (oa < n) ys[oa] = u[q].x;
                    if (ob < n) ys[ob] = u[q].y;
                }
            }
            c = cn;
            j = jn;
        }
    }
}

// ------------------------------------------------------------------------
// k_fir_bulk_reg<N>: the bulk pairs (le == N/4) with the pair's two blocks
// loaded straight into registers (coalesced dword loads, the LE overlap re-read
// from L1/L2) instead of round 2's LDS span (k_fir_bulk, now in
// scripts/stftlab.hip only).  Without the 28 KB of spans a workgroup needs
// 24 KB of LDS, so four workgroups fit per CU (16 waves instead of 12): the
// kernel is latency-bound on its LDS exchanges (scripts/kbench.py firlab*).
// The next pair's loads are issued after the inverse FFT, ahead of this
// pair's stores (issued during the FFT they would need 32 more VGPRs than the
// four waves per SIMD allow).  All global accesses are compiler-visible.
// ------------------------------------------------------------------------
// DYN: the dynamic band walk of k_stft_pair VAR 4 (persistent grid, each
// wave's next pair from a per-(XCD group, slot) counter in `ctrs`, the last wave
// of each counter stream resets it); otherwise the static XCD walk.
template <int N, bool DYN = false>
__global__ void __launch_bounds__(256, 4)
k_fir_bulk_reg(const float2* Hg, const float* x, float* y, long long nch, long long x_stride, long long y_stride,
               long long cnt, long long q0, const float2* gpass, long long n, const float* prefix, long long lm1,
               long long qf, long long ql, unsigned* ctrs) {
    using G = Geo<N>;
    static_assert(G::T == 64 && N == 1024 && !TwLayout<N>::SPLIT, "one wave per transform (T = N/16), pass-major twiddles");
    constexpr int F = 4, RL = G::RL;
    constexpr int LE = N / 4, LOUT = N - LE;   // taps <= N/4 + 1
    constexpr int TWL = G::tw_off(G::NPASS - 1) > 0 ? G::tw_off(G::NPASS - 1) : 1;
    constexpr int XW = ri_floats<N>();   // the FFT exchanges as real / imaginary halves (b32)
    __shared__ __attribute__((aligned(16))) float xch[F * XW];
    __shared__ float2 ltab[TWL];
    __shared__ float2 lH[N / 2 + 1];
    for (int i = threadIdx.x; i < G::tw_off(G::NPASS - 1); i += 256) ltab[i] = gpass[i];
    for (int i = threadIdx.x; i <= N / 2; i += 256) lH[i] = Hg[i];
    const int lt = threadIdx.x, slot = lt >> 6, t = lt & 63;
    TwLastReg<N> tw;
    tw.tab = ltab;
    tw.load(gpass, t);
    __syncthreads();
    float2* my = reinterpret_cast<float2*>(xch + slot * XW);
    long long p, p_end, p_step;
    // DYN: counter value k of stream s (= XCD group, slot) is pair
    // (k / 64) * 8 F 64 + s * 64 + k % 64: the chip sweeps one moving band
    const int stream = __builtin_amdgcn_readfirstlane((int)(blockIdx.x & 7) * F + slot);
    unsigned* const ctr = DYN ? ctrs + 32 * stream : nullptr;
    auto band_pair = [&](unsigned k) -> long long {
        return (long long)(k >> 6) * (8 * F * 64) + (long long)stream * 64 + (long long)(k & 63);
    };
    unsigned rk = 0;   // lane 0: the counter value of the pair after p
    if constexpr (DYN) {
        unsigned r0 = 0;
        if (t == 0) r0 = atomicAdd(ctr, 1u);
        p = band_pair(__builtin_amdgcn_readfirstlane(r0));
        p_end = nch * cnt;
        p_step = 0;
        if (p < p_end && t == 0) rk = atomicAdd(ctr, 1u);
    } else {
        xcd_walk(nch * cnt, F, slot, &p, &p_end, &p_step);
        p = uni<64>(p);
        p_end = uni<64>(p_end);
        p_step = uni<64>(p_step);
        if (p >= p_end) return;
    }
    auto locate = [&](long long it, long long* cc, long long* jj) {
        *cc = it / cnt;
        *jj = 2 * (q0 + (it - *cc * cnt));
    };
    long long c = 0, j = 0;
    if (p < p_end) locate(p, &c, &j);
    float xa[G::P], xb[G::P];
    auto load_a = [&](long long cc, long long jj) {
        const float* a = x + cc * x_stride + jj * LOUT - LE;   // wave-uniform block base
#pragma unroll
        for (int r = 0; r < G::P; ++r) xa[r] = __builtin_nontemporal_load(a + t + 64 * r);
    };
    auto load_b = [&](long long cc, long long jj) {
        const float* b = x + cc * x_stride + jj * LOUT - LE + LOUT;
#pragma unroll
        for (int r = 0; r < G::P; ++r) xb[r] = b[t + 64 * r];   // overlaps the next pair's block a: cached
    };
    // Edge pairs (pair index < qf: the span starts before sample 0; >= ql: it
    // reaches past n) take bounds-checked loads (history prefix or zeros before
    // 0, zeros past n) and predicated stores in the same launch -- a wave-
    // uniform branch, so the bulk pairs pay two scalar compares.
    // An edge pair is loaded at the top of its own iteration (nothing else live
    // then); a bulk pair is prefetched during the previous pair's stores.
    auto is_edge = [&](long long jj) { return (jj >> 1) < qf || (jj >> 1) >= ql; };
    if (p < p_end && !is_edge(j)) {
        load_a(c, j);
        load_b(c, j);
    }
    for (; p < p_end; p += p_step) {
        if constexpr (DYN) p_step = band_pair(__builtin_amdgcn_readfirstlane(rk)) - p;
        const bool more = p + p_step < p_end;
        long long cn = c, jn = j;
        if (more) locate(p + p_step, &cn, &jn);
        if (is_edge(j)) {
            // staged through the (idle) exchange buffer with a rolled loop, so the
            // bounds checks need no per-register address state
            const float* xs = x + c * x_stride;
            const float* pre = prefix ? prefix + c * lm1 : nullptr;
            float* sf = reinterpret_cast<float*>(my);
            auto stage = [&](long long s0, float* dst) {
#pragma unroll 1
                for (int k = t; k < N; k += 64) {
                    const long long i = s0 + k;
                    float v = 0.0f;
                    if (i < 0) {
                        if (pre && i >= -lm1) v = pre[lm1 + i];
                    } else if (i < n) {
                        v = xs[i];
                    }
                    sf[k] = v;
                }
                xsync<64>();
#pragma unroll
                for (int r = 0; r < G::P; ++r) dst[r] = sf[t + 64 * r];
                xsync<64>();
            };
            stage(j * LOUT - LE, xa);
            stage((j + 1) * LOUT - LE, xb);
        }
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = make_float2(xa[r], xb[r]);
        tw.opaque();
        fft_regs<N, true, false, true, TwLastReg<N>, false, false>(v, t, my, tw);
        float2 u[G::P];
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const int m = q / RL + G::NPT * (q % RL);   // out_pos<N>(t, q) = t + 64*m
            if (m < G::P / 2) u[m] = cmul(v[q], lH[t + 64 * m]);
            else u[m] = cmul(v[q], cconj(lH[N - t - 64 * m]));
        }
        tw.opaque();
        fft_regs<N, false, false, true, TwLastReg<N>, false, false>(u, t, my, tw);
        if (more && !is_edge(jn)) {   // ahead of this pair's stores: in flight across them
            load_a(cn, jn);
            load_b(cn, jn);
        }
        if constexpr (DYN) {
            if (more && t == 0) rk = atomicAdd(ctr, 1u);   // -> the pair after cn/jn
        }
        float* ya = y + c * y_stride + j * LOUT - LE;   // + e: block j output (e >= LE)
        if (is_edge(j)) {   // outputs past n are not stored
            long long rem = n - (j * LOUT - LE + t);   // this lane's outputs below n: e < rem
            const int rm = (int)(rem < (1 << 30) ? rem : (1 << 30));
#pragma unroll
            for (int q = 0; q < G::P; ++q) {
                const int m = q / RL + G::NPT * (q % RL);
                if (q % RL != 0) {
                    if (64 * m < rm) ya[t + 64 * m] = u[q].x;
                    if (64 * m + LOUT < rm) ya[LOUT + t + 64 * m] = u[q].y;
                }
            }
            c = cn;
            j = jn;
            continue;
        }
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            if (q % RL != 0) {   // e = t + 64 m >= LE exactly for these registers
                const int m = q / RL + G::NPT * (q % RL);
                __builtin_nontemporal_store(u[q].x, ya + t + 64 * m);
                __builtin_nontemporal_store(u[q].y, ya + LOUT + t + 64 * m);
            }
        }
        c = cn;
        j = jn;
    }
    if constexpr (DYN) {   // the XCD group's last wave out resets its counters for the next launch
        if (t == 0) {
            const unsigned nw = (unsigned)((gridDim.x - (blockIdx.x & 7) + 7) / 8);
            if (atomicAdd(ctr + 16, 1u) == nw - 1) {
                atomicExch(ctr, 0u);
                atomicExch(ctr + 16, 0u);
            }
        }
    }
}

// ------------------------------------------------------------------------
// k_fir_r32: config 4's overlap-save (N = 1024, LE = 256, LOUT = 768) with the
// 1024-point transforms split 32 x 32 instead of 16 x 16 x 4, so each FFT
// crosses LDS ONCE (a 32 x 32 transpose) instead of twice.  The FFTs of
// k_fir_bulk_reg are LDS-bound (each exchange moves 8 KB through a ~80 B/clk
// write path per CU; four exchanges per pair): this halves the exchanges.
//
// A transform lives on 32 lanes (32 points per lane), so a wave runs two pairs
// at once, one per half.  Forward, for z[n] = a[n] + i b[n], n = 32 m1 + m2:
//   lane m2: DFT_32 over m1 (registers) -> k1, times W_1024^(m2 k1)
//   transpose through LDS (row k1, column m2; rows padded to 33: conflict-free)
//   lane k1: DFT_32 over m2 -> X[k1 + 32 k2] in register k2.
// The product with H (f < 512: H[f], else conj H[1024 - f]) keeps that
// layout, and the inverse runs the same two steps mirrored:
//   lane k1: IDFT_32 over k2 -> a, times conj W_1024^(k1 a)
//   transpose; lane a: IDFT_32 over k1 -> b:  y[a + 32 b] in register b,
// so the 768 outputs of a block (e = a + 32 b >= 256, b >= 8) leave as 24
// lane-contiguous dword stores per block.  Each lane keeps its 31 twiddles
// W_1024^(m r) come from an LDS table [r][m] (consecutive lanes, consecutive
// words) and the next pair's 64 samples are loaded during the current pair's
// transforms: two waves per SIMD (launch bounds 256, 2); exchange buffers
// 66 KB + H 4 KB + twiddles 8 KB per workgroup, two workgroups per CU.
// Edge pairs (span before sample 0 or past n) load through the prefix / zero
// rule and store predicated, in the same loop (a wave-uniform branch).
// Walk: each XCD group takes one contiguous eighth of the couples (xcd_walk), so
// neighbouring blocks' overlap comes from that XCD's L2 (a grid-wide front
// measured 0.2517 vs 0.2019 ms, profiles/r04_kbench_fir_walk.jsonl).
// PAIRED (the launcher's choice for 8 B aligned channels): bulk samples move as 8 B per lane -- a block's 1024 inputs as 16
// dwordx2 loads (rows 0..7 of block b are rows 24..31 of block a: 12 more), its
// 768 outputs as 12 dwordx2 stores -- each pair of dwords re-laid by one
// v_permlane16_swap (r32_pairswap): lane l of a half works on residue
// 2 (l & 15) + (l >> 4) instead of l, which only moves its forward-twiddle column
// and the rows the transposes use.  Needs 8 B aligned channels (x, y and
// their strides even).
// ------------------------------------------------------------------------
template <bool PAIRED>
__global__ void __launch_bounds__(256, 2)
k_fir_r32(const float2* Hg, const float* x, float* y, long long nch, long long x_stride, long long y_stride,
          long long ppc, const float2* tw1024, long long n, const float* prefix, long long lm1, long long qf,
          long long ql) {
    constexpr int N = 1024, LE = 256, LOUT = N - LE, F = 4;
    __shared__ __attribute__((aligned(16))) float2 xch[F * 2 * R32_BUF];
    __shared__ float2 lH[N / 2 + 1];
    __shared__ float2 ltw[32 * 32];   // [r][m] = W_1024^(m r) (row 0 unused)
    for (int i = threadIdx.x; i <= N / 2; i += 256) lH[i] = Hg[i];
    for (int i = threadIdx.x; i < 32 * 32; i += 256) ltw[i] = tw1024[((i & 31) * (i >> 5)) & (N - 1)];
    const int lt = threadIdx.x, slot = lt >> 6, lane = lt & 63, half = lane >> 5, m = lane & 31;
    float2* buf = xch + (2 * slot + half) * R32_BUF;
    // the lane's residue: input / output samples 32 r + mr in register r
    const int mr = PAIRED ? 2 * (m & 15) + (m >> 4) : m;
    const float2* atwf = ltw + mr;      // + 32 r: W_1024^(mr r), forward (lane = input residue)
    const float2* atw = ltw + m;        // + 32 r: W_1024^(m r), inverse (lane = bin residue)
    const float2* ahl = lH + m;         // + 32 k2: H[m + 32 k2], k2 < 16
    const float2* ahh = lH + 32 - m;    // + 32 (31 - k2): H[1024 - m - 32 k2]
    __syncthreads();
    const long long pairs = nch * ppc, couples = (pairs + 1) / 2;
    long long it, it_end, it_step;
    xcd_walk(couples, F, slot, &it, &it_end, &it_step);
    it = uni<64>(it);
    it_end = uni<64>(it_end);
    it_step = uni<64>(it_step);
    if (it < it_end) {
    // couple k: pairs 2k (lanes 0..31) and 2k+1 (lanes 32..63); a missing
    // second pair (odd total) computes pair 2k again and stores nothing.
    // Pair 2k = (channel c0, pair q0 of it), kept incrementally for the static
    // walk (one division per wave, not three per couple).
    long long c0 = 0, q0 = 0, dc = 0, dq = 0;
    auto seek = [&](long long k) {
        c0 = (2 * k) / ppc;
        q0 = 2 * k - c0 * ppc;
    };
    auto locate = [&](long long k, long long* c, long long* j, bool* valid, bool* edge_any) {
        const bool two = 2 * k + 1 < pairs;
        const bool wrap = q0 + 1 == ppc;
        const long long c1 = two ? c0 + (wrap ? 1 : 0) : c0, q1 = two ? (wrap ? 0 : q0 + 1) : q0;
        *valid = !half || two;
        *c = half ? c1 : c0;
        *j = 2 * (half ? q1 : q0);
        *edge_any = q0 < qf || q0 >= ql || q1 < qf || q1 >= ql;
    };
    auto advance = [&]() {   // (c0, q0) of couple k + it_step from those of k
        q0 += dq;
        c0 += dc;
        if (q0 >= ppc) {
            q0 -= ppc;
            ++c0;
        }
    };
    dc = (2 * it_step) / ppc;
    dq = 2 * it_step - dc * ppc;
    seek(it);
    float xa[32], xb[32];
    auto load_bulk = [&](long long c, long long j) {
        if constexpr (PAIRED) {
            // 8 B pairs (samples 64 i + 2m, +1), swapped into the residue layout at use
            const float2* a = reinterpret_cast<const float2*>(x + c * x_stride + j * LOUT - LE) + m;
            const float2* b = a + LOUT / 2;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float2 u = ld_nt(a + 32 * i);
                xa[2 * i] = u.x;
                xa[2 * i + 1] = u.y;
            }
#pragma unroll
            for (int i = 4; i < 16; ++i) {   // rows 0..7 of block b = rows 24..31 of block a
                const float2 u = b[32 * i];    // overlaps the next pair's block a: cached
                xb[2 * i] = u.x;
                xb[2 * i + 1] = u.y;
            }
        } else {
            const float* a = x + c * x_stride + j * LOUT - LE + m;
            const float* b = a + LOUT;
#pragma unroll
            for (int r = 0; r < 32; ++r) xa[r] = __builtin_nontemporal_load(a + 32 * r);
#pragma unroll
            for (int r = 0; r < 32; ++r) xb[r] = b[32 * r];   // overlaps the next pair's block a: cached
        }
    };
    // edge couples: staged through the (idle) exchange buffer with rolled loops
    // (the prefix / zero rule per sample), then read back -- no register
    // array is indexed by a loop variable, and nothing else is live here
    auto load_edge = [&](long long c, long long j) {
        const float* xs = x + c * x_stride;
        const float* pre = prefix ? prefix + c * lm1 : nullptr;
        float* sf = reinterpret_cast<float*>(buf);
        const long long s0 = j * LOUT - LE;
#pragma unroll 1
        for (int k = m; k < 2 * N; k += 32) {
            const long long i = s0 + (k < N ? k : k - N + LOUT);
            float v = 0.0f;
            if (i < 0) {
                if (pre && i >= -lm1) v = pre[lm1 + i];
            } else if (i < n) {
                v = xs[i];
            }
            sf[k] = v;
        }
        xsync<64>();
#pragma unroll
        for (int r = 0; r < 32; ++r) xa[r] = sf[mr + 32 * r];
#pragma unroll
        for (int r = 0; r < 32; ++r) xb[r] = sf[N + mr + 32 * r];
        xsync<64>();
    };
    long long c, j;
    bool valid, edge;
    locate(it, &c, &j, &valid, &edge);
    if (!edge) load_bulk(c, j);
    for (; it < it_end; it += it_step) {
        if (edge) {
            load_edge(c, j);   // at the top of its own iteration (a bulk couple was prefetched)
        } else if constexpr (PAIRED) {
#pragma unroll
            for (int i = 0; i < 16; ++i) r32_pairswap(xa[2 * i], xa[2 * i + 1]);
#pragma unroll
            for (int i = 4; i < 16; ++i) r32_pairswap(xb[2 * i], xb[2 * i + 1]);
        }
        float2 v[32];
        if constexpr (PAIRED) {
            // v[r] = (block a row r, block b row r); block b's rows 0..7 are block a's
            // rows 24..31 (edge couples too: the same sample indices)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const vf2_t A = {xa[2 * i], xa[2 * i + 1]};
                const vf2_t B = i < 4 ? vf2_t{xa[24 + 2 * i], xa[25 + 2 * i]} : vf2_t{xb[2 * i], xb[2 * i + 1]};
                v[2 * i] = upk(pk_pair<0>(A, B));
                v[2 * i + 1] = upk(pk_pair<1>(A, B));
            }
        } else {
#pragma unroll
            for (int r = 0; r < 32; ++r) v[r] = make_float2(xa[r], xb[r]);
        }
        const long long itn = it + it_step;
        long long cn = c, jn = j;
        bool validn = valid, edgen = edge;
        if (itn < it_end) {   // the next couple's loads, in flight across this one's transforms
            advance();
            locate(itn, &cn, &jn, &validn, &edgen);
            if (!edgen) load_bulk(cn, jn);
        }
        {
            // forward: DFT over m1, twiddle, transpose, DFT over m2 -> X[m + 32 k2] in v[k2]
            dft32<true>(v);
            r32_twiddle<true>(v, atwf);
            r32_transpose(v, buf, mr, m);
            dft32<true>(v);
            // times H: bin f = m + 32 k2 (H[f] for f < 512, conj H[1024 - f] above)
            {
                float2 h[16];
                lds_rd64x16<0, 256>(ahl, h);   // H[m + 32 k2], k2 < 16
#pragma unroll
                for (int k2 = 0; k2 < 16; ++k2) v[k2] = cmul(v[k2], h[k2]);
                lds_rd64x16<15 * 256, -256>(ahh, h);   // h[i] = H[1024 - m - 32 (16 + i)]
#pragma unroll
                for (int i = 0; i < 16; ++i) v[16 + i] = cmulc(v[16 + i], h[i]);
            }
            // inverse: IDFT over k2, conj twiddle, transpose, IDFT over k1 -> y[m + 32 b] in v[b]
            dft32<false>(v);
            r32_twiddle<false>(v, atw);
            r32_transpose(v, buf, m, mr);
            dft32<false>(v);
        }
        {
            float* ya = y + c * y_stride + j * LOUT - LE + mr;   // + 32 b: block j's output (b >= 8)
            if (!edge) {
                if constexpr (PAIRED) {
                    // rows b, b + 1 -> 8 B pairs: lane l < 16 stores samples 32 b + 2l, +1,
                    // lane l + 16 samples 32 (b + 1) + 2l, +1
                    float2 oa[12], ob[12];   // (row b, row b + 1) of block a / block b
#pragma unroll
                    for (int i = 0; i < 12; ++i) {
                        oa[i] = upk(pk_pair<0>(pk(v[8 + 2 * i]), pk(v[9 + 2 * i])));
                        ob[i] = upk(pk_pair<1>(pk(v[8 + 2 * i]), pk(v[9 + 2 * i])));
                        r32_pairswap(oa[i].x, oa[i].y);
                        r32_pairswap(ob[i].x, ob[i].y);
                    }
                    float2* yp = reinterpret_cast<float2*>(y + c * y_stride + j * LOUT - LE) + (m & 15) + 16 * (m >> 4);
                    if (valid) {
#pragma unroll
                        for (int i = 0; i < 12; ++i) st_nt(oa[i], yp + 16 * (8 + 2 * i));
#pragma unroll
                        for (int i = 0; i < 12; ++i) st_nt(ob[i], yp + LOUT / 2 + 16 * (8 + 2 * i));
                    }
                } else if (valid) {
#pragma unroll
                    for (int b = 8; b < 32; ++b) __builtin_nontemporal_store(v[b].x, ya + 32 * b);
#pragma unroll
                    for (int b = 8; b < 32; ++b) __builtin_nontemporal_store(v[b].y, ya + LOUT + 32 * b);
                }
            } else if (valid) {   // outputs past n are not stored
                const long long rem = n - (j * LOUT - LE + mr);
                const int rm = (int)(rem < (1 << 30) ? rem : (1 << 30));
#pragma unroll
                for (int b = 8; b < 32; ++b) {
                    if (32 * b < rm) ya[32 * b] = v[b].x;
                    if (32 * b + LOUT < rm) ya[LOUT + 32 * b] = v[b].y;
                }
            }
        }
        c = cn;
        j = jn;
        valid = validn;
        edge = edgen;
    }
    }
}

// Effective history of the block geometry (see the header comment).
long long fir_effective_history(long long nfft, long long taps) {
    long long le = taps - 1;
    if (le < nfft / 4) le = nfft / 4;
    return (le + 3) & ~3LL;
}

// LDS-DMA bulk variant: one wave per transform, where span + exchange + H +
// twiddles (80 KB per 4 transforms) still leave two workgroups per CU
template <int N>
constexpr bool FIR_BULK = Geo<N>::T == 64;

template <int N>
static hipError_t run_fir(long long taps, const float2* H, const float* x, float* y, long long n,
                          long long nch, long long x_stride, long long y_stride, const float* prefix,
                          hipStream_t s) {
    const long long lm1 = taps - 1, le = fir_effective_history(N, taps), lout = N - le;
    if (lout < N / 4) return hipErrorInvalidValue;
    const long long nblk = (n + lout - 1) / lout, ppc = (nblk + 1) / 2;
    const float2* tN = twiddle_table(N);
    const float2* pN = pass_twiddles(N);
    float* sink = store_sink();
    if (!tN || !pN || !sink) return hipErrorOutOfMemory;
    constexpr int WG = Wg<N>::value, F = Wg<N>::F;
    // bulk pairs [qf, ql): span start (2q*lout - le) >= 0 and both blocks'
    // outputs (2q+2)*lout <= n; aligned channels only
    long long qf = ppc, ql = ppc;
    if constexpr (FIR_BULK<N>) {
        const bool aligned = ((uintptr_t)x & 15) == 0 && (x_stride & 3) == 0;
        if (aligned) {
            qf = (le + 2 * lout - 1) / (2 * lout);
            ql = n / (2 * lout);   // (2q+2)*lout <= n  <=>  q < n/(2 lout)
            if (ql > ppc) ql = ppc;
            if (qf >= ql) qf = ql = ppc;
        }
    }
    // the bulk kernel reads spans [2q*lout - le, (2q+2)*lout) and writes outputs
    // below (2q+2)*lout without bounds checks: verify the range on the host
    if (ql > qf && (2 * qf * lout < le || 2 * ql * lout > n || N + lout > N + (3 * N) / 4))
        return hipErrorInvalidValue;
    static std::atomic<int> capc_b, capc_e;
    const bool old = knob(KNOB_FIR_OLD, 0) == 1;   // A/B knob (scripts/kbench.py)
    // le == N/4 holds for every filter fir_block gives N = 1024 (taps <= 257)
    if constexpr (N == 1024) {
        // the 32 x 32 transform split (k_fir_r32): one LDS transpose per FFT instead
        // of two; every pair, edges included, in one launch.  Knob FIR_R32 = 0: the
        // 16 x 16 x 4 kernels below (A/B)
        if (le == N / 4 && knob(KNOB_FIR_R32, 1) != 0) {
            // bulk pairs need no alignment here (dword loads): [qf, ql) from the geometry alone
            long long qf32 = (le + 2 * lout - 1) / (2 * lout), ql32 = n / (2 * lout);
            if (ql32 > ppc) ql32 = ppc;
            if (qf32 >= ql32) qf32 = ql32 = ppc;
            qf = qf32;
            ql = ql32;
            // 8 B pairs (PAIRED) for 8 B aligned channels; dword loads and stores otherwise
            const bool paired = ((uintptr_t)x & 7) == 0 && ((uintptr_t)y & 7) == 0 && (x_stride & 1) == 0 &&
                                (y_stride & 1) == 0;
            static std::atomic<int> capc_32;
            const int cap = cached_grid(capc_32, (const void*)k_fir_r32<true>, 256, 0, 1LL << 40);
            const long long couples = (nch * ppc + 1) / 2, need = (couples + 3) / 4;
            const int grid = (int)(need < cap ? need : cap);
            const float2* t1024 = twiddle_table(1024);
            if (!t1024) return hipErrorOutOfMemory;
            if (grid < 1) return hipSuccess;
            stat_inc(STAT_FIR_R32);
            if (paired)
                hipLaunchKernelGGL((k_fir_r32<true>), dim3(grid), dim3(256), 0, s, H, x, y, nch, x_stride, y_stride,
                                   ppc, t1024, n, prefix, lm1, qf, ql);
            else
                hipLaunchKernelGGL((k_fir_r32<false>), dim3(grid), dim3(256), 0, s, H, x, y, nch, x_stride, y_stride,
                                   ppc, t1024, n, prefix, lm1, qf, ql);
            return hipGetLastError();
        }
    }
    if (ql > qf && le == N / 4 && !old) {
        // every pair of every channel in one launch: the edge pairs [0, qf) and
        // [ql, ppc) take the kernel's bounds-checked branch (round 2 ran them as a
        // second, latency-bound launch: 11 us of config 4's 237)
        if constexpr (FIR_BULK<N>) {
            static std::atomic<int> capc_r, capc_rd;
            // the dynamic band walk (k_fir_bulk_reg<N, true>): 0.2385 -> 0.2323 ms
            // for config 4, same buffers, bit-identical (profiles/r03_kbench_fir_dyn.jsonl);
            // knob FIR_DYN = 0 keeps the static XCD walk (A/B)
            // Small jobs (< 8 pairs per wave slot of the persistent grid), a grid
            // too small for 8 XCD groups, or no counter block (pool exhausted, a
            // first use inside a graph capture) take the static walk below.
            if (knob(KNOB_FIR_DYN, -1) != 0) {
                const int cap_d = cached_grid(capc_rd, (const void*)k_fir_bulk_reg<N, true>, 256, 0, 1LL << 40);
                unsigned* ctrs = (cap_d >= 8 && nch * ppc >= 8LL * 4 * cap_d) ? stream_counters(s) : nullptr;
                if (ctrs) {
                    stat_inc(STAT_FIR_DYN);
                    hipLaunchKernelGGL((k_fir_bulk_reg<N, true>), dim3(cap_d / 8 * 8), dim3(256), 0, s, H, x, y, nch,
                                       x_stride, y_stride, ppc, 0LL, pN, n, prefix, lm1, qf, ql, ctrs);
                    return hipGetLastError();
                }
            }
            const int cap_r = cached_grid(capc_r, (const void*)k_fir_bulk_reg<N>, 256, 0, 1LL << 40);
            const long long need = (nch * ppc + 3) / 4;
            const int grid = (int)(need < cap_r ? need : cap_r);
            stat_inc(STAT_FIR_STATIC);
            hipLaunchKernelGGL((k_fir_bulk_reg<N>), dim3(grid), dim3(256), 0, s, H, x, y, nch, x_stride, y_stride, ppc,
                               0LL, pN, n, prefix, lm1, qf, ql, (unsigned*)nullptr);
        }
        return hipGetLastError();
    } else if (ql > qf) {
        if constexpr (FIR_BULK<N>) {
            const int cap_b = cached_grid(capc_b, (const void*)k_fir_pair<N, true>, WG, 0, 1LL << 40);
            const long long cnt = ql - qf, need = (nch * cnt + F - 1) / F;
            const int grid = (int)(need < cap_b ? need : cap_b);   // persistent (chunked launches measured slower)
            hipLaunchKernelGGL((k_fir_pair<N, true>), dim3(grid), dim3(WG), 0, s, lm1, le, H, x, y, n, nch,
                               x_stride, y_stride, prefix, cnt, 0LL, qf, pN, tN, sink, 0LL);
        }
    }
    const long long ecnt = qf + (ppc - ql);   // edge pairs per channel: [0, qf) and [ql, ppc)
    if (ecnt > 0) {
        const int cap_e = cached_grid(capc_e, (const void*)k_fir_pair<N, false>, WG, 0, 1LL << 40);
        const long long need = (nch * ecnt + F - 1) / F;
        const int grid = (int)(need < cap_e ? need : cap_e);
        hipLaunchKernelGGL((k_fir_pair<N, false>), dim3(grid), dim3(WG), 0, s, lm1, le, H, x, y, n, nch,
                           x_stride, y_stride, prefix, ecnt, qf, ql, pN, tN, sink, 0LL);
    }
    return hipGetLastError();
}

bool fir_ols_supported(long long nfft) { return nfft >= 64 && nfft <= 8192 && (nfft & (nfft - 1)) == 0; }

// H: N complex bins of FFT(h zero-padded to N) / N
hipError_t launch_fir_ols(long long nfft, long long taps, const float2* H, const float* x, float* y,
                          long long n, long long nch, long long x_stride, long long y_stride,
                          const float* prefix, hipStream_t s) {
#define CALL(NN) run_fir<NN>(taps, H, x, y, n, nch, x_stride, y_stride, prefix, s)
    switch (nfft) {
        case 64: return CALL(64); case 128: return CALL(128); case 256: return CALL(256);
        case 512: return CALL(512); case 1024: return CALL(1024); case 2048: return CALL(2048);
        case 4096: return CALL(4096); case 8192: return CALL(8192);
        default: return hipErrorInvalidValue;
    }
#undef CALL
}

// ------------------------------------------------------------------------
// Direct form, bit-identical to vv_dsp_fir_apply (fir.c:170-186):
//   acc = 0; acc += h[0]*x[i]; acc += h[t]*x[i-t] for t = 1..L-1 (newest first)
// with every product and sum rounded separately (no FMA contraction), so the
// f32 result equals the reference's.  Samples before x[0] come from `prefix`.
// A block owns DIRECT_TILE outputs; the taps go through LDS in tiles of
// DIRECT_TAPS (with the matching input window, DIRECT_TILE + DIRECT_TAPS - 1
// samples), the accumulators stay in registers across tiles, so any filter
// length keeps the reference's summation order in 37 KB of LDS.
// ------------------------------------------------------------------------
constexpr int DIRECT_TILE = 1024;
constexpr int DIRECT_TAPS = 4096;
constexpr int DIRECT_OPT = DIRECT_TILE / 256;   // outputs per thread

// SRC 0: x[i] for 0 <= i < n, samples before x[0] from `prefix` (taps-1 per
//        channel, prefix_stride apart; NULL: zeros), zero past n.
// SRC 1: the reflect-padded input of vv_dsp_filtfilt_fir (common.c:6-21):
//        output i is sample pad + i of ext = [reflection | x | reflection] with
//        pad = taps - 1, so every tap lands inside ext; `xn` is x's length.
// REV:   output i is stored at y[n - 1 - i] (the filtfilt reversals).
template <int SRC, bool REV>
__global__ void __launch_bounds__(256)
k_fir_direct(const float* __restrict__ h, long long taps, const float* __restrict__ x,
             float* __restrict__ y, long long n, long long x_stride, long long y_stride,
             const float* __restrict__ prefix, long long prefix_stride, long long xn, long long tiles_per_ch) {
    __shared__ float hs[DIRECT_TAPS];
    __shared__ float xs[DIRECT_TILE + DIRECT_TAPS];
    const long long c = blockIdx.x / tiles_per_ch;
    const long long i0 = (blockIdx.x % tiles_per_ch) * DIRECT_TILE;
    const long long lm1 = taps - 1;
    const float* xc = x + c * x_stride;
    const float* pc = prefix ? prefix + c * prefix_stride : nullptr;
    float acc[DIRECT_OPT];
#pragma unroll
    for (int j = 0; j < DIRECT_OPT; ++j) acc[j] = 0.0f;
    for (long long t0 = 0; t0 < taps; t0 += DIRECT_TAPS) {
        const int tt = (int)(taps - t0 < DIRECT_TAPS ? taps - t0 : DIRECT_TAPS);
        __syncthreads();   // the previous tile's reads are done
        for (int u = threadIdx.x; u < tt; u += 256) hs[u] = h[t0 + u];
        // xs[e] = x[i0 - t0 - (tt - 1) + e], e < DIRECT_TILE + tt - 1
        const long long base = i0 - t0 - (tt - 1);
        for (int e = threadIdx.x; e < DIRECT_TILE + tt - 1; e += 256) {
            const long long idx = base + e;   // >= -lm1
            float v;
            if constexpr (SRC == 0) {
                if (idx < 0) v = pc ? pc[lm1 + idx] : 0.0f;
                else v = (idx < n) ? xc[idx] : 0.0f;
            } else {
                // ext[pad + idx]: left pad ext[pad-1-i] = x[min(i+1, xn) - 1],
                // right pad ext[pad+xn+i] = x[i + 1 <= xn ? xn-1-i : 0]
                long long src;
                if (idx < 0) src = (-idx < xn ? -idx : xn) - 1;
                else if (idx < xn) src = idx;
                else src = (idx - xn + 1 <= xn) ? 2 * xn - 1 - idx : 0;
                v = (idx < n) ? xc[src] : 0.0f;
            }
            xs[e] = v;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < DIRECT_OPT; ++j) {
            const int o = threadIdx.x + 256 * j;
            const float* xi = xs + (tt - 1) + o;   // xi[-u] = x[i0 + o - (t0 + u)]
            float a = acc[j];
            // hipcc contracts a*b+c into v_fma regardless of pragmas; an empty asm on
            // the product keeps the multiply and the add separately rounded.
            for (int u = 0; u < tt; ++u) {
                float pt = hs[u] * xi[-u];
                asm volatile("" : "+v"(pt));
                a = a + pt;
            }
            acc[j] = a;
        }
    }
    float* yc = y + c * y_stride;
#pragma unroll
    for (int j = 0; j < DIRECT_OPT; ++j) {
        const long long i = i0 + threadIdx.x + 256 * j;
        if (i < n) yc[REV ? n - 1 - i : i] = acc[j];
    }
}

// ------------------------------------------------------------------------
// Direct form from registers (k_fir_reg): the same sums in the same order,
// without LDS.  A thread owns 16 consecutive outputs o0..o0+15 (a workgroup
// 4096) and runs the taps in tiles of 16.  For tile u0 its window is
// E[j] = s[o0 - u0 - 16 + j], j < 32, held as 24 register pairs
// Q[j] = (E[j], E[j+8]), so that the products for outputs (r, r+8) at tap
// u0+k are ONE packed multiply Q[16+r-k] * h[u0+k] (v_pk_mul_f32 with the tap
// broadcast by op_sel) and the sums one packed add: 16 VALU per 16 MACs, every
// product and sum separately rounded (the multiply is an asm statement, so no
// FMA can form).  The next tile's window is the previous one shifted by 16:
// eight pairs carry over, sixteen new samples come in (dwordx4 loads, L1/L2
// hits).  Tiles touching the signal's edges load element by element through
// the kernel's source rule (prefix / zeros / reflection), so results equal
// k_fir_direct's bit for bit.
// ------------------------------------------------------------------------
constexpr int REG_OPT = 16;                 // outputs per thread
constexpr int REG_TILE = 256 * REG_OPT;     // outputs per workgroup

template <int SRC>
__device__ __forceinline__ float fir_fetch(const float* xc, const float* pc, long long idx, long long n, long long lm1,
                                           long long xn) {
    if constexpr (SRC == 0) {
        // the last tap tile's window reaches up to 15 samples before -lm1: those
        // are never multiplied by a tap, and must not be read past the prefix
        if (idx < 0) return (pc && idx >= -lm1) ? pc[lm1 + idx] : 0.0f;
        return idx < n ? xc[idx] : 0.0f;
    } else {
        if (idx >= n) return 0.0f;
        long long src;
        if (idx < 0) src = (-idx < xn ? -idx : xn) - 1;
        else if (idx < xn) src = idx;
        else src = (idx - xn + 1 <= xn) ? 2 * xn - 1 - idx : 0;
        return xc[src];
    }
}

template <int SRC, bool REV>
__global__ void __launch_bounds__(256)
k_fir_reg(const float* __restrict__ h, long long taps, const float* __restrict__ x, float* __restrict__ y, long long n,
          long long x_stride, long long y_stride, const float* __restrict__ prefix, long long prefix_stride,
          long long xn, long long tiles_per_ch, int aligned) {
    const long long c = blockIdx.x / tiles_per_ch;
    const long long ob = (blockIdx.x % tiles_per_ch) * REG_TILE;
    const long long o0 = ob + (long long)threadIdx.x * REG_OPT;
    const long long lm1 = taps - 1;
    const long long hi_ok = SRC == 1 ? (xn < n ? xn : n) : n;   // [0, hi_ok): plain loads
    const float* xc = x + c * x_stride;
    const float* pc = prefix ? prefix + c * prefix_stride : nullptr;
    vf2_t acc[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = vf2_t{0.0f, 0.0f};
    vf2_t Q[24];
    // tile 0 window: E[j] = s[o0 - 16 + j], j < 32
    {
        float E[32];
        const bool fast = aligned && ob - 16 >= 0 && ob + REG_TILE <= hi_ok;
        if (fast) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const vf4_t v = *reinterpret_cast<const vf4_t*>(xc + o0 - 16 + 4 * q);
                E[4 * q] = v.x; E[4 * q + 1] = v.y; E[4 * q + 2] = v.z; E[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 32; ++j) E[j] = fir_fetch<SRC>(xc, pc, o0 - 16 + j, n, lm1, xn);
        }
#pragma unroll
        for (int j = 0; j < 24; ++j) Q[j] = vf2_t{E[j], E[j + 8]};
    }
    const long long full = taps / 16;
    for (long long t = 0;; ++t) {
        const long long u0 = 16 * t;
        const int kn = t < full ? 16 : (int)(taps - u0);   // taps in this tile
        vf2_t H[8];
        if (kn == 16) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const vf4_t v = *reinterpret_cast<const vf4_t*>(h + u0 + 4 * q);
                H[2 * q] = vf2_t{v.x, v.y};
                H[2 * q + 1] = vf2_t{v.z, v.w};
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) {
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const vf2_t p = (k & 1) ? pk_mul_bcast<1>(Q[16 + r - k], H[k >> 1])
                                            : pk_mul_bcast<0>(Q[16 + r - k], H[k >> 1]);
                    acc[r] = acc[r] + p;
                }
            }
        } else {   // the last, partial tile: exactly the remaining taps
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (k < kn) {
                    const float hk = h[u0 + k];
                    const vf2_t hh = vf2_t{hk, hk};
#pragma unroll
                    for (int r = 0; r < 8; ++r) acc[r] = acc[r] + pk_mul_bcast<0>(Q[16 + r - k], hh);
                }
            }
        }
        if (u0 + 16 >= taps) break;
        // next window: E'[j] = s[o0 - u0 - 32 + j]; Q'[16+j] = Q[j], Q'[8+j] = (N[8+j], E[j]), Q'[j] = (N[j], N[j+8])
        float N[16];
        const long long lo = ob - u0 - 32;
        const bool fast = aligned && lo >= 0 && ob + REG_TILE - u0 - 16 <= hi_ok;
        if (fast) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const vf4_t v = *reinterpret_cast<const vf4_t*>(xc + o0 - u0 - 32 + 4 * q);
                N[4 * q] = v.x; N[4 * q + 1] = v.y; N[4 * q + 2] = v.z; N[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) N[j] = fir_fetch<SRC>(xc, pc, o0 - u0 - 32 + j, n, lm1, xn);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) Q[16 + j] = Q[j];
#pragma unroll
        for (int j = 0; j < 8; ++j) Q[8 + j] = vf2_t{N[8 + j], Q[16 + j].x};
#pragma unroll
        for (int j = 0; j < 8; ++j) Q[j] = vf2_t{N[j], N[j + 8]};
    }
    float* yc = y + c * y_stride;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const long long ia = o0 + r, ib = o0 + r + 8;
        if (ia < n) yc[REV ? n - 1 - ia : ia] = acc[r].x;
        if (ib < n) yc[REV ? n - 1 - ib : ib] = acc[r].y;
    }
}

template <int SRC, bool REV>
static hipError_t run_fir_reg(const float* h, long long taps, const float* x, float* y, long long n, long long nch,
                              long long x_stride, long long y_stride, const float* prefix, long long prefix_stride,
                              long long xn, hipStream_t s) {
    const long long tiles = (n + REG_TILE - 1) / REG_TILE;
    if (tiles * nch <= 0) return hipSuccess;
    if (taps < 1 || tiles * nch > 0x7fffffffLL) return hipErrorInvalidValue;
    // the 16 B tap loads need 16 B aligned taps; the fast sample loads 16 B
    // aligned rows (a 4-float multiple stride)
    if ((uintptr_t)h & 15) return hipErrorInvalidValue;
    const int aligned = ((uintptr_t)x & 15) == 0 && (x_stride & 3) == 0;
    hipLaunchKernelGGL((k_fir_reg<SRC, REV>), dim3((unsigned)(tiles * nch)), dim3(256), 0, s, h, taps, x, y, n,
                       x_stride, y_stride, prefix, prefix_stride, xn, tiles, aligned);
    return hipGetLastError();
}

static bool fir_reg_enabled() { return knob(KNOB_FIR_DIRECT_LDS, 0) != 1; }   // A/B: 1 = the LDS kernel

hipError_t launch_fir_direct(const float* h, long long taps, const float* x, float* y, long long n,
                             long long nch, long long x_stride, long long y_stride,
                             const float* prefix, hipStream_t s) {
    const long long tiles = (n + DIRECT_TILE - 1) / DIRECT_TILE;
    if (tiles * nch <= 0) return hipSuccess;
    if (taps < 1 || tiles * nch > 0x7fffffffLL) return hipErrorInvalidValue;
    if (fir_reg_enabled() && ((uintptr_t)h & 15) == 0)
        return run_fir_reg<0, false>(h, taps, x, y, n, nch, x_stride, y_stride, prefix, taps - 1, n, s);
    hipLaunchKernelGGL((k_fir_direct<0, false>), dim3((unsigned)(tiles * nch)), dim3(256), 0, s, h, taps, x, y, n,
                       x_stride, y_stride, prefix, taps - 1, n, tiles);
    return hipGetLastError();
}

// vv_dsp_filtfilt_fir (common.c:23-80) over nch rows of n samples: the forward
// pass writes the n + pad outputs of ext that the backward pass reads, already
// reversed (tmp_rev[j] = tmp[ext_n - 1 - j]); the backward pass is then a plain
// direct form over tmp_rev whose first pad samples are its history, and its n
// outputs are stored reversed into y.  Both passes keep the reference's
// summation order (acc = 0, += h[k] * s[i-k], k ascending, no FMA); every
// output needed has all its taps inside ext, so the reference's maxk bound
// never cuts a sum short and the results are bit-identical.
hipError_t launch_filtfilt(const float* h, long long taps, const float* x, float* y, long long n, long long nch,
                           long long x_stride, long long y_stride, float* tmp, hipStream_t s) {
    const long long pad = taps - 1, m = n + pad;
    const long long t1 = (m + DIRECT_TILE - 1) / DIRECT_TILE, t2 = (n + DIRECT_TILE - 1) / DIRECT_TILE;
    if (n <= 0 || nch <= 0) return hipSuccess;
    if (taps < 1 || t1 * nch > 0x7fffffffLL) return hipErrorInvalidValue;
    if (fir_reg_enabled() && ((uintptr_t)h & 15) == 0) {
        hipError_t e = run_fir_reg<1, true>(h, taps, x, tmp, m, nch, x_stride, m, nullptr, 0, n, s);
        if (e != hipSuccess) return e;
        return run_fir_reg<0, true>(h, taps, tmp + pad, y, n, nch, m, y_stride, tmp, m, n, s);
    }
    hipLaunchKernelGGL((k_fir_direct<1, true>), dim3((unsigned)(t1 * nch)), dim3(256), 0, s, h, taps, x, tmp, m,
                       x_stride, m, (const float*)nullptr, 0LL, n, t1);
    hipLaunchKernelGGL((k_fir_direct<0, true>), dim3((unsigned)(t2 * nch)), dim3(256), 0, s, h, taps,
                       (const float*)(tmp + pad), y, n, m, y_stride, (const float*)tmp, m, n, t2);
    return hipGetLastError();
}

// ------------------------------------------------------------------------
// Overlap-save for filters longer than the fused kernels take (N > 8192):
// blocks j (2 per complex row: z = a + i b, as k_fir_pair) gathered into rows
// of an N-point batch, FFT, x H (FFT(h) unscaled; the inverse applies 1/N),
// inverse FFT, and the block outputs LE..N-1 scattered back.  The FFTs are the
// four-step kernels (large_fft.hip); these three kernels are the glue.
// Row q of a chunk is pair p = p0 + q over (channel, pair) items.
// ------------------------------------------------------------------------
__global__ void k_fir_long_gather(const float* x, long long n, long long x_stride, long long nfft, long long le,
                                  long long lout, long long ppc, long long p0, long long rows, float2* z) {
    const long long total = rows * nfft;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long q = i / nfft, e = i - q * nfft, p = p0 + q;
        const long long c = p / ppc, j = 2 * (p - c * ppc);
        const float* xc = x + c * x_stride;
        const long long ia = j * lout - le + e, ib = ia + lout;
        const float a = (ia >= 0 && ia < n) ? xc[ia] : 0.0f;
        const float b = (ib >= 0 && ib < n) ? xc[ib] : 0.0f;
        z[i] = make_float2(a, b);
    }
}

__global__ void k_fir_long_mul(float2* Z, const float2* H, long long nfft, long long total) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x)
        Z[i] = cmul(Z[i], H[i % nfft]);
}

__global__ void k_fir_long_scatter(const float2* z, float* y, long long n, long long y_stride, long long nfft,
                                   long long le, long long lout, long long ppc, long long p0, long long rows) {
    const long long total = rows * lout;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long q = i / lout, k = i - q * lout, p = p0 + q;
        const long long c = p / ppc, j = 2 * (p - c * ppc);
        const float2 v = z[q * nfft + le + k];
        float* yc = y + c * y_stride;
        const long long oa = j * lout + k, ob = oa + lout;
        if (oa < n) yc[oa] = v.x;
        if (ob < n) yc[ob] = v.y;
    }
}

static unsigned glue_grid(long long total) {
    long long b = (total + 255) / 256;
    return (unsigned)(b < 1 ? 1 : (b > 65536 ? 65536 : b));
}

hipError_t launch_fir_long_gather(const float* x, long long n, long long x_stride, long long nfft, long long le,
                                  long long lout, long long ppc, long long p0, long long rows, float2* z,
                                  hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fir_long_gather, dim3(glue_grid(rows * nfft)), dim3(256), 0, s, x, n, x_stride, nfft, le,
                       lout, ppc, p0, rows, z);
    return hipGetLastError();
}

hipError_t launch_fir_long_mul(float2* Z, const float2* H, long long nfft, long long rows, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fir_long_mul, dim3(glue_grid(rows * nfft)), dim3(256), 0, s, Z, H, nfft, rows * nfft);
    return hipGetLastError();
}

hipError_t launch_fir_long_scatter(const float2* z, float* y, long long n, long long y_stride, long long nfft,
                                   long long le, long long lout, long long ppc, long long p0, long long rows,
                                   hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fir_long_scatter, dim3(glue_grid(rows * lout)), dim3(256), 0, s, z, y, n, y_stride, nfft,
                       le, lout, ppc, p0, rows);
    return hipGetLastError();
}

}  // namespace vvh
