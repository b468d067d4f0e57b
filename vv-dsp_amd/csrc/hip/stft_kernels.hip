// stft_kernels.hip -- fused STFT analysis for gfx950.
//
// For every (channel, frame) of the reference's spectrogram (stft.c:112-144):
// gather the frame (zero past the end of the signal, stft.c:124-130), apply the
// window (vectorized_math_fallback.c:13-29), FFT, and write either magnitudes
// sqrtf(re^2+im^2) for all nfft bins (stft.c:133-139) or the full complex
// spectrum (stft_process semantics, stft.c:74-92).
//
// k_stft_pair<N>: TWO real frames a, b share one complex N-point FFT of
// z = w*a + i*w*b.  With the mirror-paired last pass each thread holds Z[k]
// and Z[N-k], so Xa[k] = (Z[k] + conj Z[N-k])/2 and Xb[k] = (Z[k] - conj Z[N-k])/2i
// come straight from registers -- no split twiddles, no LDS post pass -- and
// every bin 0..N-1 of both rows is produced in place (Hermitian symmetry is
// automatic).  Used when Geo<N>::CAN_PAIR.
// k_stft_pair_lds<N>: the same frame pairs where the last pass cannot be
// mirror-paired (nfft = 256 and 4096): the mirror bins are read back through LDS.
//
// Scheduling: the bulk variant (VAR 0) is launched non-persistently, one
// workgroup per 16 consecutive frame pairs per transform slot, the slots of a
// workgroup interleaved, so the nfft-hop overlap of neighbouring frames is
// re-read from the same CU's L1/L2 and the dispatcher balances the CUs (no
// straggler tail).  VAR 1 (unaligned hops / channel strides) and VAR 2 (the
// zero-padded tail frames) are persistent and walk XCD-aware shares
// (xcd_walk).  VAR 0 streams each pair's input span (N + hop samples) into LDS
// with global_load_lds_dwordx4 one pair ahead and waits on hand-counted
// vmcnt.  For N = 1024 (one wave per transform) the magnitudes go straight
// from registers as full-line dword streaming stores and the FFT exchanges
// through a half-size real/imaginary buffer (3 workgroups per CU); other N
// stage the rows through LDS for 16-byte stores.  Window values are
// per-thread constants in registers; twiddles live in LDS.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"

#include <cstdint>
#include <cstdlib>

// N = 2048 magnitude rows (R2048): both last-pass butterflies' twiddles in
// registers (TwLastRegA, 166 VGPRs, three waves per SIMD as before) instead of
// TwLastRegP's mirror half read from LDS: -1.5 %, bit-identical
// (profiles/r06_ab_twregs_mfcc_windows.jsonl); 0 restores TwLastRegP (A/B)
#ifndef VVH_R2048_RA
#define VVH_R2048_RA 1
#endif

namespace vvh {

// samples e = t + r*T of one frame (zero outside [0, n); all zero when !valid).
// `s` must point at a real channel.  The tail path clamps the index and selects
// instead of branching per element, so the loads stay branch-free.
template <int N>
__device__ __forceinline__ void frame_load(float* x, const float* s, long long start, long long n, int t,
                                           bool valid) {
    using G = Geo<N>;
    if (start + N <= n) {
#pragma unroll
        for (int r = 0; r < G::P; ++r) x[r] = s[start + t + r * G::T];
    } else {
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            const long long e = start + t + r * G::T;
            const float val = s[e < n ? e : n - 1];
            x[r] = e < n ? val : 0.0f;
        }
    }
    if (!valid) {
#pragma unroll
        for (int r = 0; r < G::P; ++r) x[r] = 0.0f;
    }
}

// |re + i im| with the hardware v_sqrt_f32 (<=1 ulp).  sqrtf's correctly
// rounded IEEE expansion costs ~10 VALU per bin; the magnitude is compared at
// the reference's float tolerance, never bit-exactly.
__device__ __forceinline__ float cmag(float re, float im) {
    return __builtin_amdgcn_sqrtf(__builtin_fmaf(re, re, im * im));
}

// Spectra of the two frames at bin k from Z = FFT(w/2 * (a + i b)):
//   Xa[k] = Z[k] + conj Z[N-k],  Xb[k] = -i (Z[k] - conj Z[N-k]).
// The 1/2 rides in the window (a power-of-two scale commutes with every
// rounding, so this is bit-identical to halving at the end).  Packed f32 math.
// MODE 0: A.x = |Xa[k]|, B.x = |Xb[k]|;  MODE 1: A = Xa[k], B = Xb[k];
// MODE 2: A.x = |Xa[k]|^2, B.x = |Xb[k]|^2 (power, bins 0..N/2 stored).
template <int MODE>
__device__ __forceinline__ void pair_post(float2 Z, float2 Zm, float2* A, float2* B) {
    const vf2_t z = {Z.x, Z.y}, zm = {Zm.x, Zm.y};
    const vf2_t s = z + zm;   // (Re Xa, Re Xb)
    const vf2_t d = z - zm;   // (-Im Xb, Im Xa)
    if constexpr (MODE == 0 || MODE == 2) {
        const vf2_t dd = d * d;
        // an explicit fused multiply-add: every call site rounds the same way, so
        // bins k and N-k (the same conjugate pair) get bit-identical values
        // wherever they are computed (lane 0's partner bins, tail pairs) -- the
        // half-spectrum gather relies on it (vv_dsp_spectrogram_unpack_half_device)
        const vf2_t m2 = __builtin_elementwise_fma(s, s, dd.yx);   // (|Xa|^2, |Xb|^2)
        A->x = MODE == 0 ? __builtin_amdgcn_sqrtf(m2.x) : m2.x;
        B->x = MODE == 0 ? __builtin_amdgcn_sqrtf(m2.y) : m2.y;
        A->y = B->y = 0.0f;
    } else {
        *A = make_float2(s.x, d.y);
        *B = make_float2(s.y, -d.x);
    }
}

// bin k of an output row (MODE 0: float magnitudes, MODE 1: float2 spectrum,
// MODE 2: float power of the half spectrum -- bins above N/2 are not stored)
template <int MODE, int N>
__device__ __forceinline__ void put_bin(char* row, int k, float2 X) {
    if constexpr (MODE == 0) *(reinterpret_cast<float*>(row) + k) = X.x;
    else if constexpr (MODE == 2) {
        if (k <= N / 2) *(reinterpret_cast<float*>(row) + k) = X.x;
    } else *(reinterpret_cast<float2*>(row) + k) = X;
}

// Rows of one frame pair straight from the FFT registers (N = 1024: one wave
// per transform, mirror-paired last pass; see k_stft_pair).  Issues exactly
// the kernel's NST stores per pair (rows of a missing second frame go to the
// sink), so the caller's hand-counted vmcnt stays exact.
template <int N, int MODE>
__device__ __forceinline__ void direct_rows(const float2* v, int t, char* rowa, char* rowb, bool has_b,
                                            float* sink) {
    using G = Geo<N>;
    using Mi = Mirror<N>;
    constexpr int R = G::RL;
    if constexpr (MODE == 1) {
        // as the DIRECT block below, with complex bins: a mirror block holds
        // conj(X[k]) (real frames), lane 0's rotated partner conj of its own
        // bin in slot j + 1, or in the last slot its self-mirrored bin as is.
        // Byte offsets reach 8 KB: blocks past 4 KB use the base + 4096.
        constexpr int J = G::NPT / 2, NB = G::NB, T = G::T;
        const unsigned ve = 8u * (unsigned)t;
        const unsigned vo = 8u * (unsigned)(t == 0 ? 0 : T - t);
        const char* ra = rowa;
        const char* rb = has_b ? rowb : reinterpret_cast<const char*>(sink);   // counted stores must all issue
        const char* ra2 = ra + 4096;
        const char* rb2 = rb + 4096;
        auto st = [&](auto imm, unsigned off, float2 val, const char* b1, const char* b2) {
            constexpr int I = decltype(imm)::value;
            if constexpr (I < 4096) st8_nt_sbase<I>(off, val, b1);
            else st8_nt_sbase<I - 4096>(off, val, b2);
        };
        float2 nxa[R], nxb[R];   // lane 0's partner values for slot j: conj of slot j+1's own bins
        static_for<0, J>([&](auto jc) {
            constexpr int j = J - 1 - decltype(jc)::value;   // last slot first: its partners are the specials
            static_for<0, R>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                constexpr int q = 2 * j * R + r;
                float2 A, B;
                pair_post<1>(v[q], mirror_of<N, true>(v, t, q), &A, &B);
                float2 pa, pb;
                if constexpr (j == J - 1) {
                    const int qm = Mi::normal(r);
                    pair_post<1>(v[qm], v[Mi::special(qm)], &pa, &pb);
                } else {
                    pa = nxa[r];
                    pb = nxb[r];
                }
                const float2 oa = select2(t == 0, pa, cconj(A)), ob = select2(t == 0, pb, cconj(B));
                nxa[r] = cconj(A);
                nxb[r] = cconj(B);
                constexpr int IE = 8 * (T * j + r * NB), IO = 8 * ((R - 1 - r) * NB - T * j + NB - T);
                st(std::integral_constant<int, IE>{}, ve, A, ra, ra2);
                st(std::integral_constant<int, IE>{}, ve, B, rb, rb2);
                st(std::integral_constant<int, IO>{}, vo, oa, ra, ra2);
                st(std::integral_constant<int, IO>{}, vo, ob, rb, rb2);
            });
        });
    } else {
        // Even slot j holds bins k = t + T j + r NB (lane-contiguous, 256 B
        // aligned per store); its partner slot holds N - k, which for lanes
        // t >= 1 covers N - k of the same magnitude.  Lane 0's partner bins
        // are shifted by one slot (lane 0 writes the mirror of its own bin in
        // slot j + 1, or its self-mirrored bin NB/2 + .. in the last slot), so
        // that every store instruction covers one aligned 256 B block: full
        // 128 B lines for the streaming stores, no LDS staging.
        constexpr int J = G::NPT / 2, NB = G::NB, T = G::T;
        constexpr int PM = MODE == 2 ? 2 : 0;   // magnitude or power post
        float ea[J][R], eb[J][R], sa[R], sb[R];
#pragma unroll
        for (int j = 0; j < J; ++j) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int q = 2 * j * R + r;
                float2 A, B;
                pair_post<PM>(v[q], mirror_of<N, true>(v, t, q), &A, &B);
                ea[j][r] = A.x;
                eb[j][r] = B.x;
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {   // lane 0's odd slot 1: bins NB/2 + (R-1-r) NB, their own mirrors
            const int qm = Mi::normal(r);
            float2 A2, B2;
            pair_post<PM>(v[qm], v[Mi::special(qm)], &A2, &B2);
            sa[r] = A2.x;
            sb[r] = B2.x;
        }
        const unsigned ve = 4u * (unsigned)t;
        const unsigned vo = 4u * (unsigned)(t == 0 ? NB - T : NB - t);
        const void* ra = rowa;
        const void* rb = has_b ? rowb : (void*)sink;   // counted stores must all issue
        // Power rows (n/2+1 floats, so not line-aligned): a block is stored
        // only if it lies below N/2, with plain stores (partial lines merge
        // in L2; streaming stores of partial lines measured 1.65x slower)
        auto st = [&](auto imm, unsigned off, float val, const void* base) {
            constexpr int I = decltype(imm)::value;
            if constexpr (MODE == 2) {
                if constexpr (I < 4 * (N / 2)) st4_sbase<I>(off, val, base);
            } else {
                // streaming stores with sc0 sc1 (write-through, not kept in L2):
                // 0.6 % faster than nt alone on the config-5 shard (same-box A/B,
                // six alternating runs each)
                st4_pol_sbase<I, 2>(off, val, base);
            }
        };
        // The N/T blocks of a row in ascending address order, row a then
        // row b (measured 0.5 % faster than interleaving the rows).  Block
        // m is an even block (slot j = m % (NB/T) < J, r = m / (NB/T)) or
        // the mirror block of (j, r) with (N/T - 1) - m = r (NB/T) + j.
        auto val = [&](auto mc, const float (&e)[J][R], const float (&sp)[R]) -> float {
            constexpr int m = decltype(mc)::value;
            constexpr int je = m % (NB / T), re = m / (NB / T);
            if constexpr (je < J) {
                return e[je][re];
            } else {
                constexpr int mm = (N / T - 1) - m, rm = mm / (NB / T), jm = mm % (NB / T);
                if constexpr (jm + 1 < J) return t == 0 ? e[jm + 1][rm] : e[jm][rm];
                else return t == 0 ? sp[rm] : e[jm][rm];
            }
        };
        auto row = [&](const float (&e)[J][R], const float (&sp)[R], const void* base) {
            static_for<0, N / T>([&](auto mc) {
                constexpr int m = decltype(mc)::value;
                if constexpr (m % (NB / T) < J) st(std::integral_constant<int, 4 * T * m>{}, ve, val(mc, e, sp), base);
                else st(std::integral_constant<int, 4 * T * m>{}, vo - 4u * (NB - T), val(mc, e, sp), base);
            });
        };
        row(ea, sa, ra);
        row(eb, sb, rb);
        if constexpr (MODE == 2) {
            // bin N/2 = NB * (R/2): even slot j = 0, r = R/2, lane 0 (one
            // lane-0 store per row, counted; rb is the sink for a missing frame)
            static_assert(N / 2 == NB * (R / 2), "Nyquist bin in lane 0 of an even block");
            st4_lane0_counted((float*)ra + N / 2, ea[0][R / 2]);
            st4_lane0_counted((float*)rb + N / 2, eb[0][R / 2]);
        }
    }
}

// Log-mel (MODE 3) or MFCC (MODE 4) rows of one frame pair from the FFT
// registers (N = 1024, one wave per transform).  The power of bins 0..N/2 of
// both frames (pair_post<2>: the power rows' arithmetic) goes to the
// transform's idle exchange buffer P, the two rows interleaved bin by bin; then k_mel_grp's steps
// with FR = 2 frames: chunk partials (FMA in bin order; lane c % 64 holds chunk
// c in round c / 64), per-filter sums of the partials in chunk order (fetched
// across lanes by ds_bpermute), logf(e + eps), and for MODE 4 the DCT-II and
// lifter over the log-mel rows (kept in P's spare tail) -- the same operations
// in the same order, so the rows equal launch_stft mode 2 followed by
// launch_mel_grp bit for bit.  The plan's tables sit in dynamic LDS (about
// 4-8 KB), paid for by spans of N + 256 floats (hop <= 256), so 3 workgroups
// per CU still fit; no compiler-generated global load enters the hand-counted
// pipeline.  Stores: MODE 3 four counted dword stores (rows a, b x filters
// t, t + 64; M <= 128), MODE 4 two ((frame, coefficient) pairs t, t + 64;
// C <= 64); lanes without a row element write to the sink.
constexpr int MEL_MAX_ROUNDS = 4;   // chunks <= 256
constexpr int MEL_LM_OFF = 1028;    // MODE 4: log-mel rows in P past the two power rows (16 B aligned)
template <int MODE, bool COUNTED>
__device__ __forceinline__ void mel_tail(int t, float* P, float* fa, float* fb, bool has_b, float* sink,
                                         const float* sW, const int* sCh, const int* sCb, const float* sD,
                                         const float* sL, const MelArgs& mel);
template <int N, int MODE>
__device__ __forceinline__ void mel_rows(const float2* v, int t, float* fa, float* fb, bool has_b, float* sink,
                                         float* P, const float* sW, const int* sCh, const int* sCb,
                                         const float* sD, const float* sL, const MelArgs& mel) {
    using G = Geo<N>;
    using Mi = Mirror<N>;
    constexpr int R = G::RL, J = G::NPT / 2, NB = G::NB, T = G::T, RW = N / 2 + 1;
    static_assert(T == 64, "one wave per transform");
    static_assert(2 * RW <= MEL_LM_OFF, "log-mel rows past the (interleaved) power rows");
    float ea[J][R], eb[J][R], sa[R], sb[R];
#pragma unroll
    for (int j = 0; j < J; ++j) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int q = 2 * j * R + r;
            float2 A, B;
            pair_post<2>(v[q], mirror_of<N, true>(v, t, q), &A, &B);
            ea[j][r] = A.x;
            eb[j][r] = B.x;
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int qm = Mi::normal(r);
        float2 A2, B2;
        pair_post<2>(v[qm], v[Mi::special(qm)], &A2, &B2);
        sa[r] = A2.x;
        sb[r] = B2.x;
    }
    // block m of 64 bins: an even block (lane t: bin 64 m + t) or the mirror
    // block of slot (jm, rm) (lane t: bin 64 m + (64 - t) % 64), as direct_rows.
    // The two rows go to P interleaved, P[2k] = |Xa[k]|^2, P[2k + 1] = |Xb[k]|^2:
    // one ds_write_b64 per bin here and one ds_read_b64 per bin in the chunk sums
    // below, the pair landing in one register pair for a packed FMA (two rows
    // RW floats apart took two b32 accesses and v_movs to re-pair them)
    auto put = [&](int bin, float va, float vb) { *reinterpret_cast<vf2_t*>(P + 2 * bin) = vf2_t{va, vb}; };
    static_for<0, N / T>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        if constexpr (T * m < N / 2) {
            constexpr int je = m % (NB / T), re = m / (NB / T);
            if constexpr (je < J) {
                put(T * m + t, ea[je][re], eb[je][re]);
            } else {
                constexpr int mm = (N / T - 1) - m, rm = mm / (NB / T), jm = mm % (NB / T);
                float va, vb;
                if constexpr (jm + 1 < J) {
                    va = t == 0 ? ea[jm + 1][rm] : ea[jm][rm];
                    vb = t == 0 ? eb[jm + 1][rm] : eb[jm][rm];
                } else {
                    va = t == 0 ? sa[rm] : ea[jm][rm];
                    vb = t == 0 ? sb[rm] : eb[jm][rm];
                }
                put(T * m + (t == 0 ? 0 : T - t), va, vb);
            }
        }
    });
    if (t == 0) {
        put(N / 2, ea[0][R / 2], eb[0][R / 2]);
        if constexpr (MelArgs::W2) {   // bins N/2 + 1 .. N/2 + 3: zeros under the last windows' tails
            put(N / 2 + 1, 0.0f, 0.0f);
            put(N / 2 + 2, 0.0f, 0.0f);
            put(N / 2 + 3, 0.0f, 0.0f);
        }
    }
    xsync<T>();
    mel_tail<MODE, true>(t, P, fa, fb, has_b, sink, sW, sCh, sCb, sD, sL, mel);
}

// The mel stage of one frame pair (MODE 3 log-mel, MODE 4 MFCC) over the 64
// lanes of a wave, from the pair's power rows in LDS interleaved bin by bin,
// P[2k] = |Xa[k]|^2, P[2k + 1] = |Xb[k]|^2 (k <= N/2): k_mel_grp's steps with
// FR = 2 frames -- chunk partials (FMA in bin order; lane c % 64 holds chunk c
// in round c / 64), per-filter sums of the partials in chunk order (fetched
// across lanes by ds_bpermute), logf(e + eps), and for MODE 4 the DCT-II and
// lifter over the log-mel rows (kept at P + MEL_LM_OFF) -- the same operations
// in the same order, so the rows equal the power rows followed by
// launch_mel_grp bit for bit.  Stores: MODE 3 rows a, b x filters t, t + 64
// (M <= 128), MODE 4 (frame, coefficient) pairs t, t + 64 (C <= 64).
template <int MODE, bool COUNTED>
__device__ __forceinline__ void mel_tail(int t, float* P, float* fa, float* fb, bool has_b, float* sink,
                                         const float* sW, const int* sCh, const int* sCb, const float* sD,
                                         const float* sL, const MelArgs& mel) {
    constexpr int T = 64;
    const int nc = mel.nc, M = mel.M, C = mel.C, lc = mel.lc, lcs = mel.lcs;
    float pa[MEL_MAX_ROUNDS], pb[MEL_MAX_ROUNDS];
    int dc[MEL_MAX_ROUNDS];   // the chunk a slot computes (windows: the host's bank-aware order)
#pragma unroll
    for (int u = 0; u < MEL_MAX_ROUNDS; ++u) {
        pa[u] = pb[u] = 0.0f;
        const int c = t + T * u;
        dc[u] = c;
        if (MODE == 3 || mel.cw == 0) {   // the chunk windows (log-mel; MFCC where the table fits three workgroups per CU)
            if (c >= nc) continue;
            // log-mel: the chunk's window of lc bins, the same lc for every lane (a
            // uniform loop: scalar trip count, immediate offsets); its zero weights
            // add exact zeros to the (row a, row b) partials, so the sums equal the
            // non-zero range's FMAs in bin order (3.053 -> 2.990 ms, 32 ch x 10 min).
            // Rows lcs = window_stride(lc) floats apart (16 B aligned, lcs / 4 odd: a
            // lane's four weights are one ds_read_b128 and the lanes' reads cover
            // distinct bank blocks; the host deals the chunks to lanes so that the
            // power reads' start banks collide least).  MFCC takes them where the windows' larger table
            // still leaves three workgroups per CU (with the register last-pass
            // twiddles, 6 KB less static LDS: the 40-mel / 13-coefficient plan);
            // otherwise the packed table (a workgroup per CU fewer: +17 %)
            const float* wr = sW + c * lcs;
            const int bits = __float_as_int(wr[lc]);   // window start | chunk << 16
            dc[u] = bits >> 16;
            const vf2_t* pp = reinterpret_cast<const vf2_t*>(P) + (bits & 0xffff);
            vf2_t ab = {0.0f, 0.0f};
            if constexpr (MelArgs::W2) {   // even starts: two bins' (row a, row b) pairs per 16 B read
                const vf4_t* p4 = reinterpret_cast<const vf4_t*>(pp);
                for (int j = 0; j < lc; j += 4) {
                    const vf4_t wq = *reinterpret_cast<const vf4_t*>(wr + j);
                    const vf4_t q0 = p4[j / 2], q1 = p4[j / 2 + 1];
                    ab = __builtin_elementwise_fma(vf2_t{q0[0], q0[1]}, vf2_t{wq[0], wq[0]}, ab);
                    ab = __builtin_elementwise_fma(vf2_t{q0[2], q0[3]}, vf2_t{wq[1], wq[1]}, ab);
                    ab = __builtin_elementwise_fma(vf2_t{q1[0], q1[1]}, vf2_t{wq[2], wq[2]}, ab);
                    ab = __builtin_elementwise_fma(vf2_t{q1[2], q1[3]}, vf2_t{wq[3], wq[3]}, ab);
                }
            } else {
                for (int j = 0; j < lc; j += 4) {
                    const vf4_t wq = *reinterpret_cast<const vf4_t*>(wr + j);   // rows 16 B aligned (lcs % 4 == 0)
#pragma unroll
                    for (int i = 0; i < 4; ++i) ab = __builtin_elementwise_fma(pp[j + i], vf2_t{wq[i], wq[i]}, ab);
                }
            }
            pa[u] = ab.x;
            pb[u] = ab.y;
        } else if (c < nc) {   // the packed layout, each chunk's own length
            const int lo = sCh[3 * c], len = sCh[3 * c + 1], off = sCh[3 * c + 2];
            vf2_t ab = {0.0f, 0.0f};   // (row a, row b) partials: fma per element, bin order
            const vf2_t* pp = reinterpret_cast<const vf2_t*>(P) + lo;
#pragma unroll 4
            for (int j = 0; j < len; ++j) {
                const float w = sW[off + j];
                ab = __builtin_elementwise_fma(pp[j], vf2_t{w, w}, ab);
            }
            pa[u] = ab.x;
            pb[u] = ab.y;
        }
    }
    // the chunk partials go to LDS over P (every lane has read its power bins
    // above), pair c at P[2c], P[2c + 1]; then lane m adds its filter's chunks
    // in chunk order -- independent ds_read_b64s instead of a chain of
    // cross-lane permutes (2 per round per chunk), the same sums bit for bit
    xsync<T>();
#pragma unroll
    for (int u = 0; u < MEL_MAX_ROUNDS; ++u) {
        const int c = t + T * u;
        if (c < nc) *reinterpret_cast<vf2_t*>(P + 2 * dc[u]) = vf2_t{pa[u], pb[u]};
    }
    xsync<T>();
    const vf2_t* part = reinterpret_cast<const vf2_t*>(P);
    float la[2] = {0.0f, 0.0f}, lb[2] = {0.0f, 0.0f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        if (T * u >= M) break;   // no filter in this round (M <= 64): skip its sums and logf
        const int m = t + T * u;
        const bool on = m < M;
        const int cb = on ? sCb[m] : 0, ce = on ? sCb[m + 1] : 0;
        float e0 = 0.0f, e1 = 0.0f;
#pragma unroll 4
        for (int c = cb; c < ce; ++c) {   // this lane's filter's chunks, in order
            const vf2_t q = part[c];
            e0 += q.x;
            e1 += q.y;
        }
        la[u] = on ? logf(e0 + mel.eps) : 0.0f;
        lb[u] = on ? logf(e1 + mel.eps) : 0.0f;
    }
    float* const snk = COUNTED ? sink + t : nullptr;
    // COUNTED: every lane issues each store (the sink when it has no element) so
    // k_stft_pair's hand-counted vmcnt stays exact; otherwise predicated stores
    auto put_out = [&](bool on, float* dst, float v) {
        if constexpr (COUNTED) st4_counted(on ? dst : snk, v);
        else if (on) *dst = v;
    };
    if constexpr (MODE == 3) {
        put_out(t < M, fa + t, la[0]);
        put_out(t + T < M, fa + t + T, la[1]);
        put_out(has_b && t < M, fb + t, lb[0]);
        put_out(has_b && t + T < M, fb + t + T, lb[1]);
    } else {
        float* const lm = P + MEL_LM_OFF;   // [2][M], M <= (ri_floats - MEL_LM_OFF) / 2
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int m = t + T * u;
            if (m < M) {
                lm[m] = la[u];
                lm[M + m] = lb[u];
            }
        }
        xsync<T>();
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int idx = t + T * u;
            float res = 0.0f;
            float* dst = snk;   // COUNTED: the sink; otherwise nullptr (no store)
            if (idx < 2 * C) {
                const int f = idx >= C ? 1 : 0, i = idx - f * C;
                const float* l = lm + f * M;
                const float* d = sD + i * M;
                float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f, c3 = 0.0f;
                int m = 0;
                if ((M & 3) == 0) {   // as k_mel_grp: four partial sums
#pragma unroll 5
                    for (; m < M; m += 4) {
                        const vf4_t a = *reinterpret_cast<const vf4_t*>(l + m);
                        const vf4_t b = *reinterpret_cast<const vf4_t*>(d + m);   // 16 B aligned: M % 4 == 0
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
                res = ((c0 + c1) + (c2 + c3)) * sL[i];
                if (f == 0) dst = fa + i;
                else if (has_b) dst = fb + i;
            }
            if constexpr (COUNTED) st4_counted(dst, res);
            else if (dst) *dst = res;
        }
    }
}

// Frame pairs (2j, 2j+1) of one channel, j in [pair0, pair0 + ppc): pairs never
// span channels, so a channel's rows do not depend on how channels are grouped
// into calls or shards.
//   VAR 0: bulk (both frames inside the signal), input spans by LDS-DMA,
//          magnitude rows as full-line streaming stores (16 B aligned rows)
//   VAR 1: bulk, stores straight from registers
//   VAR 2: tail -- the last few pairs, zero-padded past the end / odd last frame
// N = 1024 bulk: 3 waves per SIMD (<= 168 VGPRs) -- the LDS budget allows 3 workgroups per CU
template <int N, int MODE, int VAR>
__global__ void __launch_bounds__(Wg<N>::value, ((N == 1024 && (VAR == 0 || VAR == 3 || VAR == 4 || VAR == 5)) ||
                                                 (N == 2048 && MODE == 0 && VAR == 0))
                                                    ? 3
                                                    : 1)
k_stft_pair(const float* sig, long long n, long long nch, long long ch_stride, long long frames,
            long long hop, long long pair0, long long ppc, const float* win, void* out,
            long long out_ch_stride, long long row_pitch, const float2* gpass, const float2* gtab, long long chunk,
            float* sink, unsigned* ctrs, MelArgs mel) {
    using G = Geo<N>;
    using Mi = Mirror<N>;
    // MODE 3 / 4: log-mel / MFCC rows from the power rows, which stay in LDS
    // (launch_stft_mel; the tables of the MFCC plan in dynamic LDS)
    constexpr bool MEL = MODE == 3 || MODE == 4;
    constexpr bool TAIL = VAR == 2;
    constexpr bool BULK = VAR == 0 || VAR == 3 || VAR == 4 || VAR == 5;
    // VAR 3: VAR 0 with each wave walking a contiguous run of pairs and its
    // span kept as a ring of 256-float chunks (hop % 256 == 0): a pair DMAs only
    // its 2*hop new samples instead of the whole N + hop span
    // VAR 5: the dynamic walk below handing out runs of `rl` consecutive pairs
    // per counter value, each run walked with VAR 3's ring
    constexpr bool DRING = VAR == 5;
    constexpr bool RING = VAR == 3 || DRING;
    // VAR 4 / 5: the dynamic band walk -- each wave takes its next pair (run) from
    // a counter of its (XCD group, slot) stream, so the chip works on one moving
    // band and neighbouring pairs share an L2 while waves balance dynamically;
    // a persistent grid, counters from stream_counters().  The counter atomics
    // are hand-counted VMEM ops like the spans and stores.
    constexpr bool DYN = VAR == 4 || DRING;
    constexpr bool STAGE = BULK && MODE == 0 && G::NPASS > 1 && G::T > 1;
    // power rows (N = 1024): the DIRECT stores below, keeping only the
    // 64-bin blocks under N/2 plus one lane for bin N/2
    constexpr bool POWD = BULK && (MODE == 2 || MEL) && G::T == 64 && G::NPASS > 1;
    static_assert(!MEL || POWD, "log-mel / MFCC rows: the one-wave-per-transform bulk kernel (N = 1024)");
    // complex rows (N = 1024): DIRECT with 8 B/lane stores, conj() for the mirror blocks
    constexpr bool CPXD = BULK && MODE == 1 && G::T == 64 && G::NPASS > 1;
    constexpr bool GLDS = (STAGE || POWD || CPXD) && G::T >= 64;   // input spans by LDS-DMA (launcher checks hop/alignment)
    // floats per transform: hop <= N/2 (MEL: hop <= 256)
    // (MEL: hop <= 256; the ring walks VAR 3 / VAR 5: hop == 256 -- so N + 256
    // floats per span; for the ring walks that makes 40.8 KB of LDS per workgroup
    // with the register last-pass twiddles: four per CU, -2.5 % for power rows,
    // -2..-3 % for the headline's magnitude rows)
    constexpr int SPAN = GLDS ? ((MEL || VAR == 3 || VAR == 5) ? N + 256 : N + N / 2) : 1;
    // T == 64 (one wave per transform): magnitudes go straight from registers as
    // full-line dword stores (DIRECT); otherwise they are staged through LDS and
    // written as 16 B/lane stores
    constexpr bool DIRECT = GLDS && G::T == 64;
    static_assert(!RING || DIRECT, "ring spans: one wave per transform on the LDS-DMA path");
    // stores per pair (both rows): power rows keep half the blocks + bin N/2
    constexpr int NST = MEL ? (MODE == 3 ? 4 : 2)
                            : DIRECT ? (MODE == 2 ? G::P + 2 : 2 * G::P)
                                                                  : 2 * (G::P / 4);
    constexpr int WG = Wg<N>::value, F = Wg<N>::F, R = G::RL;
    // N = 2048 magnitude rows (two waves per transform, LDS-DMA spans, rows
    // staged for 16 B stores): the same half-size exchange, the last pass'
    // twiddles of each thread's first butterfly held in registers (TwLastRegP:
    // 1136 table entries in LDS instead of 2032) and the two rows staged one
    // after the other through the half-size buffer -- 51 KB of LDS per
    // workgroup instead of 75.6 KB, so 3 workgroups (3 waves per SIMD) fit per
    // CU instead of 2
    constexpr bool R2048 = N == 2048 && STAGE && GLDS;
    // DIRECT needs no staging buffer: the exchange goes through a half-size
    // (real, then imaginary) buffer, so 3 workgroups fit per CU instead of 2
    constexpr bool RI = DIRECT || R2048;
    constexpr int XF = RI ? (ri_floats<N>() + 3) / 4 * 2 : G::LDS;   // float2 per transform (16 B multiple)
    constexpr int LDSN = G::NPASS > 1 ? F * XF : 1;
    __shared__ __attribute__((aligned(16))) float2 lds[LDSN];   // 16 B: pass_exchange_ri's b128 writes
    // N = 1024 one-wave transforms (DIRECT): every last-pass twiddle of a
    // thread in registers (TwLastRegA: 24 VGPRs), only the first two passes'
    // 240 entries in LDS -- 6 KB less LDS per workgroup, 12 fewer LDS reads per
    // pair, the table's own values (bit-identical)
    // (Not for magnitude rows' VAR 0, the launch of small jobs: config 3's single
    // 60 s call measured +2 % with the per-workgroup twiddle loads.)
    constexpr bool RA = (DIRECT && N == 1024 && !(MODE == 0 && VAR == 0)) || (R2048 && VVH_R2048_RA);
    constexpr int TWE = RA       ? G::tw_off(G::NPASS - 1)
                        : R2048 ? G::tw_off(G::NPASS - 1) + (G::RL - 1) * (G::ns(G::NPASS - 1) / 2)   // TwLastRegP's
                                : TwLayout<N>::ENTRIES;
    __shared__ float2 ltab[TWE];
    __shared__ float span_all[GLDS ? F * SPAN : 1];
    const TwTab<N> tw{ltab};
    using TwL = std::conditional_t<RA, TwLastRegA<N, true>, std::conditional_t<R2048, TwLastRegP<N>, TwTab<N>>>;
    TwL twl{};
    if constexpr (RA) {
        twl.tab = ltab;
        twl.load(gpass, (int)threadIdx.x % Geo<N>::T);
    } else if constexpr (R2048) {
        twl.tab = ltab;
        twl.hi = ltab + Geo<N>::tw_off(Geo<N>::NPASS - 1);
        twl.load(gpass, (int)threadIdx.x % Geo<N>::T);
    }
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T;
    float2* my = lds + (G::NPASS > 1 ? slot * XF : 0);
    // window values 0.5 w[t + r T], packed two per VGPR pair (pk_mul_bcast)
    vf2_t wp[(G::P + 1) / 2];
#pragma unroll
    for (int r = 0; r < G::P; ++r) {
        const float wr = 0.5f * win[t + r * G::T];
        if (r & 1) wp[r / 2].y = wr;
        else wp[r / 2] = vf2_t{wr, 0.0f};
    }

    int kb[G::NPT];   // last-pass butterfly of each slot (loop invariant)
#pragma unroll
    for (int i = 0; i < G::NPT; ++i) kb[i] = bfly<N, G::NPASS - 1, true>(t, i);
    constexpr long long ES = MODE == 1 ? 8 : 4;            // bytes per bin
    constexpr long long ROW = MODE == 2 ? N / 2 + 1 : N;   // bins per row
    // floats (MODE 1: complex values) from one row's start to the next: power rows
    // may sit `row_pitch` floats apart (>= N/2 + 1, e.g. 544 = 17 whole lines)
    const long long ROWR = MODE == 3 ? (long long)mel.M : MODE == 4 ? (long long)mel.C : MODE == 2 ? row_pitch : ROW;
    // MEL: the plan's tables in dynamic LDS: W [nnz], chunks [3 nc], cbeg [M + 1], then (MODE 4) D [C M], lift [C]
    extern __shared__ __attribute__((aligned(16))) float mel_lds[];
    const int mel_dpos = MEL ? (mel.nnz + mel.cw * mel.nc + mel.M + 1 + 3) & ~3 : 0;
    // rows of one pair from the registers, plain stores (unaligned / tail pairs)
    auto store_generic = [&](float2* v, char* rowa, char* rowb, bool has_b) {
        if constexpr (G::T == 1) {
#pragma unroll
            for (int q = 0; q < G::P; ++q) {
                float2 A, B;
                pair_post<MODE>(v[q], mirror_of<N, true>(v, t, q), &A, &B);
                put_bin<MODE, N>(rowa, q, A);
                if (has_b) put_bin<MODE, N>(rowb, q, B);
            }
        } else {
            // even slots hold bins k, their partner slots hold N-k: one post
            // per (k, N-k) pair, stored at both (real input -> mirror = conj)
#pragma unroll
            for (int i = 0; i < G::NPT; i += 2) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int q = i * R + r, qm = Mi::normal(q);
                    float2 A, B;
                    pair_post<MODE>(v[q], mirror_of<N, true>(v, t, q), &A, &B);
                    float2 Am = MODE == 0 ? A : cconj(A), Bm = MODE == 0 ? B : cconj(B);
                    if (i == 0) {   // thread 0: slot 1 is butterfly NB/2, its own mirror
                        float2 A2, B2;
                        pair_post<MODE>(v[qm], v[Mi::special(qm)], &A2, &B2);
                        Am = select2(t == 0, A2, Am);
                        Bm = select2(t == 0, B2, Bm);
                    }
                    const int k = kb[i] + r * G::NB, km = kb[i + 1] + (R - 1 - r) * G::NB;
                    put_bin<MODE, N>(rowa, k, A);
                    put_bin<MODE, N>(rowa, km, Am);
                    if (has_b) {
                        put_bin<MODE, N>(rowb, k, B);
                        put_bin<MODE, N>(rowb, km, Bm);
                    }
                }
            }
        }
    };
    const long long pairs = nch * ppc;
    long long p, p_end, p_step;
    // RING: block b owns items [b*chunk, (b+1)*chunk) (chunk = the low 40 bits),
    // cut into groups of F runs of `rl` consecutive pairs (rl = the high bits);
    // slot s walks run s of every group
    const long long rl = RING ? (chunk >> 40) : 1;
    long long kk = 0;   // items this slot has done
    if constexpr (RING && !DRING) {
        const long long ch = chunk & ((1LL << 40) - 1);
        p = (long long)blockIdx.x * ch + slot * rl;
        p_end = (long long)(blockIdx.x + 1) * ch < pairs ? (long long)(blockIdx.x + 1) * ch : pairs;
        p_step = 1;
    } else if constexpr (DYN) {
        p = 0;   // set below from the XCD's counter
        p_end = pairs;
        p_step = 1;
    } else {
        work_walk(pairs, F, slot, chunk, &p, &p_end, &p_step);
    }
    p = uni<G::T>(p);
    p_end = uni<G::T>(p_end);
    p_step = uni<G::T>(p_step);
    // one counter per (XCD, slot): 32 streams, so no address takes more than one
    // atomic per workgroup of its XCD per pair
    const int stream = __builtin_amdgcn_readfirstlane((int)(blockIdx.x & 7) * F + slot);
    unsigned* const ctr = DYN ? ctrs + 32 * stream : nullptr;
    // DB = 2^dbs consecutive items per stream and band (VAR 5: log2 in chunk's low bits)
    const int dbs = DRING ? (int)(chunk & 15) : 6;
    // Each XCD group walks its own contiguous eighth of the runs (its F slot
    // streams banded inside it) -- the write probe's best layout (scripts/
    // membench.hip k_wprobe BAND 1: 0.896 of peak for pure writes against 0.840
    // for 2 MB chunks dealt round robin); a stream past its eighth is done.
    // 3.2967 -> 3.2556 ms for the config-5 shard, same buffers, bit-identical
    // (profiles/r04_kbench_xcd_eighths.jsonl).
    const long long nrun = DYN ? (pairs + rl - 1) / rl : 0, r8 = (nrun + 7) / 8;
    auto band_pair = [&](unsigned k) -> long long {
        const long long DB = 1LL << dbs;
        const long long g = stream / F, sl = stream % F;   // wave-uniform (stream is readfirstlane'd)
        const long long it = g * r8 + (long long)(k >> dbs) * (F * DB) + sl * DB + (long long)(k & (DB - 1));
        const long long ge = (g + 1) * r8 < nrun ? (g + 1) * r8 : nrun;
        return it < ge ? it : pairs;
    };
    unsigned rr = 0;   // lane 0: an issued counter atomic's result (valid after a vmcnt wait)
    auto grab = [&]() {
        if (t == 0) asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(rr) : "v"(ctr), "v"(1u) : "memory");
    };
    long long pn = 0;   // DYN: the pair after p
    if constexpr (DYN) {
        unsigned r0 = 0;
        if (t == 0)
            asm volatile("global_atomic_add %0, %1, %2, off sc0\n\ts_waitcnt vmcnt(0)" : "=v"(r0) : "v"(ctr), "v"(1u) : "memory");
        if constexpr (DRING) {   // counter value k -> the run of pairs [rl b(k), rl b(k) + rl)
            p = rl * band_pair(__builtin_amdgcn_readfirstlane(r0));
        } else {
            grab();
            unsigned k1;
            asm volatile("s_waitcnt vmcnt(0)\n\tv_readfirstlane_b32 %0, %1" : "=s"(k1) : "v"(rr) : "memory");
            p = band_pair(__builtin_amdgcn_readfirstlane(r0));
            pn = band_pair(k1);
        }
    }
    const bool any = p < p_end;   // uniform per transform
    // (channel, first frame) of a pair; this launch covers frames
    // [2*pair0, 2*(pair0 + ppc)) of every channel
    auto locate = [&](long long q, long long* cc, long long* ff) {
        *cc = q / ppc;
        *ff = 2 * (pair0 + q - *cc * ppc);
    };
    long long c = 0, fa = 0;
    if (any) locate(p, &c, &fa);
    float xa[G::P], xb[G::P];
    // GLDS: the pair's span [fa*hop, fa*hop + hop + N) goes HBM/L2 -> LDS by
    // 16 B/lane LDS-DMA, issued right after the previous span was read, so it
    // lands while that pair is transformed -- no VGPRs held across iterations.
    float* span = span_all + (GLDS ? slot * SPAN : 0);
    // Pairs that reach past the end of the signal (the zero-padded tail, at
    // most a few per channel) fill the span with ordinary bounds-checked loads
    // and LDS stores instead: the compiler waits on those itself, and being
    // younger than every hand-counted operation they keep the counts valid.
    auto issue_span = [&](long long cc, long long ff) {
        const float* s0 = sig + cc * ch_stride + ff * hop;
        const int len = (int)(N + hop), lane = t & 63;
        if (ff * hop + len <= n) {
            for (int u = t >> 6; u * 256 < len; u += G::T / 64) {
                const int e = u * 256 + lane * 4;
                glds16(s0 + (e < len ? e : 0), span + u * 256);
            }
        } else {
            const long long left = n - ff * hop;   // samples of this span inside the signal
            for (int u = t >> 6; u * 256 < len; u += G::T / 64) {
                const int e = u * 256 + lane * 4;
                vf4_t q;
#pragma unroll
                for (int k = 0; k < 4; ++k) q[k] = e + k < left ? s0[e + k] : 0.0f;
                *reinterpret_cast<vf4_t*>(span + u * 256 + lane * 4) = q;
            }
        }
    };
    // ring (VAR 3): chunk k of the current pair's span [fa*hop, fa*hop + N + hop)
    // sits in ring slot (rs + k) mod rc; the next pair of the same channel
    // reuses chunks h2.. and DMAs its last h2 into the slots of chunks 0..h2-1,
    // which this pair has read (into registers) before the DMA is issued
    const int rc = RING ? (int)((N + hop) >> 8) : 1, h2 = RING ? (int)((2 * hop) >> 8) : 0,
              hb = RING ? (int)(hop >> 8) : 0;
    int rs = 0, rsn = 0;
    auto issue_new = [&](long long cc, long long ff) {
        const float* s0 = sig + cc * ch_stride + ff * hop;
        rsn = rs + h2 >= rc ? rs + h2 - rc : rs + h2;
        for (int k = rc - h2; k < rc; ++k) {
            const int sl = rsn + k >= rc ? rsn + k - rc : rsn + k;
            glds16(s0 + k * 256 + (t & 63) * 4, span + sl * 256);
        }
    };
    auto load_pair = [&](long long cc, long long ff) {
        if constexpr (RING) rsn = 0;   // whole span, chunk k in slot k
        if constexpr (GLDS) {
            issue_span(cc, ff);
        } else if constexpr (TAIL) {
            const float* s = sig + cc * ch_stride;
            frame_load<N>(xa, s, ff * hop, n, t, true);
            frame_load<N>(xb, s, (ff + 1 < frames ? ff + 1 : ff) * hop, n, t, ff + 1 < frames);
        } else {   // both frames lie inside the signal: wave-uniform bases, plain loads
            const float* sa = sig + cc * ch_stride + ff * hop;
            const float* sb = sa + hop;
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                xa[r] = sa[t + r * G::T];
                xb[r] = sb[t + r * G::T];
            }
        }
    };
    // the first span's DMA is in flight while the block stages its twiddles
    if (any) load_pair(c, fa);
    if constexpr (DYN) {
        if constexpr (DRING) {
            if (any) grab();   // -> the next run
        } else {
            if (any && pn < pairs) grab();   // -> the pair after pn
        }
    }
    if constexpr (RA) {   // the passes before the last
        TwLastRegA<N, true>::template stage<WG>(ltab, gpass);
    } else if constexpr (R2048) {   // the passes before the last, and the last pass' upper half
        TwLastRegP<N>::template stage<WG>(ltab, ltab + Geo<N>::tw_off(Geo<N>::NPASS - 1), gpass);
    } else {
        stage_twiddles<N, WG>(ltab, gpass, gtab);
    }
    if constexpr (MEL) {
        int* const mi = reinterpret_cast<int*>(mel_lds);
        for (int i = threadIdx.x; i < mel.nnz; i += WG) mel_lds[i] = mel.W[i];
        for (int i = threadIdx.x; i < mel.cw * mel.nc; i += WG) mi[mel.nnz + i] = mel.chunks[i];
        for (int i = threadIdx.x; i <= mel.M; i += WG) mi[mel.nnz + mel.cw * mel.nc + i] = mel.cbeg[i];
        if constexpr (MODE == 4) {
            for (int i = threadIdx.x; i < mel.C * mel.M; i += WG) mel_lds[mel_dpos + i] = mel.D[i];
            for (int i = threadIdx.x; i < mel.C; i += WG) mel_lds[mel_dpos + mel.C * mel.M + i] = mel.lift[i];
        }
    }
    __syncthreads();
    if (!any && !DYN) return;
    if constexpr (GLDS) vm_wait<0>();
    if constexpr (RING) rs = rsn;
    for (; p < p_end; p += p_step) {
        if constexpr (DRING) {
            // the last grabbed run: its atomic is older than the previous pair's
            // NST stores (issued with the DMA of its run's first pair)
            unsigned kq;
            asm volatile("s_waitcnt vmcnt(%1)\n\tv_readfirstlane_b32 %0, %2" : "=s"(kq) : "n"(NST), "v"(rr) : "memory");
            const long long pq = p + 1 >= pairs ? pairs : kk + 1 < rl ? p + 1 : rl * band_pair(kq);
            p_step = uni<G::T>(pq - p);
        } else if constexpr (RING) {
            p_step = ((kk + 1) % rl) ? 1 : (long long)F * rl - rl + 1;
        }
        if constexpr (DYN && !DRING) p_step = pn - p;
        const bool more = p + p_step < p_end;
        long long cn = c, fn = fa;
        if constexpr (RING) {   // within a run: the next pair, or frame 2*pair0 of the next channel
            if (p_step == 1) {
                fn = fa + 2;
                if (fn >= 2 * (pair0 + ppc)) {
                    cn = c + 1;
                    fn = 2 * pair0;
                }
            } else if (more) {
                locate(p + p_step, &cn, &fn);
            }
        } else {
            if (more) locate(p + p_step, &cn, &fn);
        }
        if constexpr (RING) {
            if constexpr (!DRING) vm_wait<NST>();
            // chunk slots of frame a (chunks 0..3) and frame b (chunks hb..hb+3)
            int ca[4], cbk[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int a = rs + k, b = rs + k + hb;
                ca[k] = __builtin_amdgcn_readfirstlane(a >= rc ? a - rc : a) * 256;
                cbk[k] = __builtin_amdgcn_readfirstlane(b >= rc ? b - rc : b) * 256;
            }
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                xa[r] = span[ca[r / 4] + t + 64 * (r % 4)];
                xb[r] = span[cbk[r / 4] + t + 64 * (r % 4)];
            }
            lgkm_wait0();   // span read before it is refilled
            if (more) {
                if (p_step == 1 && cn == c && fn * hop + (N + hop) <= n) issue_new(cn, fn);
                else load_pair(cn, fn);
                if constexpr (DRING) {
                    if (kk + 1 == rl) grab();   // the next pair starts a run: fetch the one after it
                }
            }
        } else if constexpr (DYN) {
            // this span's DMA and the counter atomic issued after it are older
            // than the previous pair's NST stores
            unsigned knn;
            asm volatile("s_waitcnt vmcnt(%1)\n\tv_readfirstlane_b32 %0, %2" : "=s"(knn) : "n"(NST), "v"(rr) : "memory");
            const long long pnn = more ? band_pair(knn) : pairs;
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                xa[r] = span[t + r * G::T];
                xb[r] = span[hop + t + r * G::T];
            }
            lgkm_wait0();   // span read before it is refilled
            if (more) {
                load_pair(cn, fn);
                if (pnn < pairs) grab();
            }
            pn = pnn;
        } else if constexpr (GLDS) {
            // younger than this span's DMA: only the previous pair's NST stores
            vm_wait<NST>();
            if constexpr (G::T > 64) lds_barrier();   // the other waves' pieces
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                xa[r] = span[t + r * G::T];
                xb[r] = span[hop + t + r * G::T];
            }
            lgkm_wait0();   // span read before it is refilled
            if constexpr (G::T > 64) lds_barrier();
            if (more) load_pair(cn, fn);
        }
        float2 v[G::P];
        if constexpr (BULK && G::T == 64) {
            // the span reads come in pairs (r, r + 1) of one frame (ds_read2st64: adjacent
            // registers); one v_pk_mov_b32 per (frame a, frame b) register pair instead of
            // two v_mov_b32.  With the exchange reads as single ds_read_b32 (RIV 1) the
            // loop's v_movs drop from 87 to 27 (power rows; VALU 419 -> 370 per pair),
            // bit-identical, 2.766 -> 2.741 ms power / 3.410 -> 3.399 ms magnitude
            // (profiles/r04_kbench_stft_movefree.jsonl).
#pragma unroll
            for (int i = 0; i < G::P / 2; ++i) {
                const vf2_t A = {xa[2 * i], xa[2 * i + 1]}, B = {xb[2 * i], xb[2 * i + 1]};
                v[2 * i] = upk(pk_mul_bcast<0>(pk_pair<0>(A, B), wp[i]));
                v[2 * i + 1] = upk(pk_mul_bcast<1>(pk_pair<1>(A, B), wp[i]));
            }
        } else {
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                const vf2_t x = {xa[r], xb[r]};
                v[r] = upk((r & 1) ? pk_mul_bcast<1>(x, wp[r / 2]) : pk_mul_bcast<0>(x, wp[r / 2]));
            }
        }
        if constexpr (GLDS) {
        } else if constexpr (TAIL) {
            if (more) load_pair(cn, fn);
        } else {
            load_pair(more ? cn : c, more ? fn : fa);   // last step re-reads its own pair
        }
        if constexpr (R2048 || RA) {
            twl.opaque();
            fft_regs<N, true, true, RI, TwL, false, false, 1>(v, t, my, twl);
        } else {
            fft_regs<N, true, true, RI, TwTab<N>, false, false, 1>(v, t, my, tw);
        }
        char* rowa = reinterpret_cast<char*>(out) + (c * out_ch_stride + fa * ROWR) * ES;
        char* rowb = rowa + ROWR * ES;
        const bool has_b = (TAIL || GLDS) ? fa + 1 < frames : true;
        if constexpr (MEL) {
            const int* mi = reinterpret_cast<const int*>(mel_lds);
            mel_rows<N, MODE>(v, t, reinterpret_cast<float*>(rowa), reinterpret_cast<float*>(rowb), has_b, sink,
                              reinterpret_cast<float*>(my), mel_lds, mi + mel.nnz, mi + mel.nnz + mel.cw * mel.nc,
                              mel_lds + mel_dpos, mel_lds + mel_dpos + mel.C * mel.M, mel);
        } else if constexpr (DIRECT) {
            direct_rows<N, MODE>(v, t, rowa, rowb, has_b, sink);
        } else if constexpr (R2048) {
            // row a, then row b, through the (now idle) half-size exchange buffer
            // (N floats each), each as full-line 16 B/lane streaming stores
            float* sf = reinterpret_cast<float*>(my);
            float bq[G::P];   // row b's magnitudes, staged after row a's stores
#pragma unroll
            for (int i = 0; i < G::NPT; i += 2) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int q = i * R + r, qm = Mi::normal(q);
                    float2 A, B;
                    pair_post<0>(v[q], mirror_of<N, true>(v, t, q), &A, &B);
                    float am = A.x, bm = B.x;
                    if (i == 0) {
                        float2 A2, B2;
                        pair_post<0>(v[qm], v[Mi::special(qm)], &A2, &B2);
                        am = t == 0 ? A2.x : am;
                        bm = t == 0 ? B2.x : bm;
                    }
                    const int k = kb[i] + r * G::NB, km = kb[i + 1] + (R - 1 - r) * G::NB;
                    sf[k] = A.x;
                    sf[km] = am;
                    bq[2 * (i / 2 * R + r)] = B.x;
                    bq[2 * (i / 2 * R + r) + 1] = bm;
                }
            }
            char* rb = has_b ? rowb : reinterpret_cast<char*>(sink);
            xsync<G::T>();
#pragma unroll
            for (int j = 0; j < G::P / 4; ++j) {   // N / (4 T) = P / 4 stores per row
                const int e = 4 * (t + G::T * j);
                st16_nt_counted(reinterpret_cast<vf4_t*>(rowa) + (t + G::T * j),
                                *reinterpret_cast<const vf4_t*>(sf + e));
            }
            xsync<G::T>();
#pragma unroll
            for (int i = 0; i < G::NPT; i += 2) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int k = kb[i] + r * G::NB, km = kb[i + 1] + (R - 1 - r) * G::NB;
                    sf[k] = bq[2 * (i / 2 * R + r)];
                    sf[km] = bq[2 * (i / 2 * R + r) + 1];
                }
            }
            xsync<G::T>();
#pragma unroll
            for (int j = 0; j < G::P / 4; ++j) {
                const int e = 4 * (t + G::T * j);
                st16_nt_counted(reinterpret_cast<vf4_t*>(rb) + (t + G::T * j), *reinterpret_cast<const vf4_t*>(sf + e));
            }
            xsync<G::T>();   // the next transform's first exchange reuses `my`
        } else if constexpr (STAGE) {
            // both magnitude rows through the (now idle) exchange buffer, then
            // full-line 16 B/lane streaming stores: 2N/(4T) instead of 2P per lane
            float* sf = reinterpret_cast<float*>(my);
#pragma unroll
            for (int i = 0; i < G::NPT; i += 2) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int q = i * R + r, qm = Mi::normal(q);
                    float2 A, B;
                    pair_post<0>(v[q], mirror_of<N, true>(v, t, q), &A, &B);
                    float am = A.x, bm = B.x;
                    if (i == 0) {
                        float2 A2, B2;
                        pair_post<0>(v[qm], v[Mi::special(qm)], &A2, &B2);
                        am = t == 0 ? A2.x : am;
                        bm = t == 0 ? B2.x : bm;
                    }
                    const int k = kb[i] + r * G::NB, km = kb[i + 1] + (R - 1 - r) * G::NB;
                    sf[k] = A.x;
                    sf[km] = am;
                    sf[N + k] = B.x;
                    sf[N + km] = bm;
                }
            }
            xsync<G::T>();
#pragma unroll
            for (int j = 0; j < G::P / 4; ++j) {
                const int e = 4 * (t + G::T * j);
                const vf4_t a = *reinterpret_cast<const vf4_t*>(sf + e);
                const vf4_t b = *reinterpret_cast<const vf4_t*>(sf + N + e);
                if constexpr (GLDS) {   // counted by the vm_wait<NST> above: exactly NST per pair
                    char* rb = has_b ? rowb : reinterpret_cast<char*>(sink);
                    st16_nt_counted(reinterpret_cast<vf4_t*>(rowa) + (t + G::T * j), a);
                    st16_nt_counted(reinterpret_cast<vf4_t*>(rb) + (t + G::T * j), b);
                } else {
                    __builtin_nontemporal_store(a, reinterpret_cast<vf4_t*>(rowa) + (t + G::T * j));
                    __builtin_nontemporal_store(b, reinterpret_cast<vf4_t*>(rowb) + (t + G::T * j));
                }
            }
            xsync<G::T>();   // the next transform's first exchange reuses `my`
        } else {
            store_generic(v, rowa, rowb, has_b);
        }
        c = cn;
        fa = fn;
        if constexpr (RING) {
            rs = rsn;
            if constexpr (DRING) kk = kk + 1 == rl ? 0 : kk + 1;
            else ++kk;
        }
    }
    if constexpr (DYN) {   // the XCD's last wave out resets its counters for the next launch
        vm_wait<0>();
        if (t == 0) {
            const unsigned nw = (unsigned)((gridDim.x - (blockIdx.x & 7) + 7) / 8);
            if (atomicAdd(ctr + 16, 1u) == nw - 1) {
                atomicExch(ctr, 0u);
                atomicExch(ctr + 16, 0u);
            }
        }
    }
}

// Frame pairs for the lengths whose last FFT pass cannot be mirror-paired in
// registers (N = 256 = 16 x 16, 4096 = 16^3: one last-pass butterfly per
// thread): two windowed real frames per complex FFT as k_stft_pair, then the
// spectrum goes through the (idle) LDS exchange buffer in natural order, and
// each thread reads Z[k], Z[N-k] for bins k = t + T j -- so both rows leave
// as lane-contiguous, full-line stores.  Persistent XCD walk with the next
// pair's samples loaded into registers while this pair is transformed.
// (Bounded to three waves per SIMD at N = 256 -- 168 VGPRs, no spills -- its
// magnitude rows ran 4 % slower: profiles/r06_ab_stft_sizes_stage.jsonl; they
// now run in k_stft_stage.)
template <int N, int MODE>
__global__ void __launch_bounds__(Wg<N>::value)
k_stft_pair_lds(const float* sig, long long n, long long nch, long long ch_stride, long long frames,
                long long hop, const float* win, void* out, long long out_ch_stride, long long row_pitch,
                const float2* gpass, const float2* gtab) {
    using G = Geo<N>;
    constexpr int WG = Wg<N>::value, F = Wg<N>::F;
    __shared__ float2 lds[F * G::LDS];
    __shared__ float2 ltab[TwLayout<N>::ENTRIES];
    stage_twiddles<N, WG>(ltab, gpass, gtab);
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T;
    float2* my = lds + slot * G::LDS;
    float w[G::P];   // 0.5 w: Xa = Z[k] + conj Z[N-k] needs no further scaling (pair_post)
#pragma unroll
    for (int r = 0; r < G::P; ++r) w[r] = 0.5f * win[t + r * G::T];
    __syncthreads();
    const TwTab<N> tw{ltab};
    constexpr long long ES = MODE == 1 ? 8 : 4;
    constexpr long long ROW = MODE == 2 ? N / 2 + 1 : N;
    const long long ppc = (frames + 1) / 2, pairs = nch * ppc;
    long long p, p_end, p_step;
    xcd_walk(pairs, F, slot, &p, &p_end, &p_step);
    p = uni<G::T>(p);
    p_end = uni<G::T>(p_end);
    p_step = uni<G::T>(p_step);
    float xa[G::P], xb[G::P];
    auto load = [&](long long q) {
        const long long c = q / ppc, fa = 2 * (q - c * ppc);
        const float* s = sig + c * ch_stride;
        const long long sa = fa * hop, sb = sa + hop;
        const bool hb = fa + 1 < frames;
        if (sb + N <= n) {   // both frames inside the signal
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                xa[r] = s[sa + t + r * G::T];
                xb[r] = s[sb + t + r * G::T];
            }
        } else {
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                const long long i = t + r * G::T;
                xa[r] = sa + i < n ? s[sa + i] : 0.0f;
                xb[r] = hb && sb + i < n ? s[sb + i] : 0.0f;
            }
        }
    };
    if (p < p_end) load(p);
    for (; p < p_end; p += p_step) {
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = make_float2(xa[r] * w[r], xb[r] * w[r]);
        const long long c = p / ppc, fa = 2 * (p - c * ppc);
        const bool hb = fa + 1 < frames;
        if (p + p_step < p_end) load(p + p_step);   // in flight across this pair's FFT and stores
        fft_regs<N, true>(v, t, my, tw);
#pragma unroll
        for (int q = 0; q < G::P; ++q) my[G::pad(out_pos<N>(t, q))] = v[q];
        xsync<G::T>();
        const long long rp = MODE == 2 ? row_pitch : ROW;   // power rows: row_pitch floats apart
        char* rowa = reinterpret_cast<char*>(out) + (c * out_ch_stride + fa * rp) * ES;
        char* rowb = rowa + rp * ES;
        if constexpr (N == 4096 && MODE == 0) {
            // bins k = t + T j <= N/2 only: bin N - k of a real frame is the
            // conjugate of bin k, bit for bit (pair_post with Z[k], Z[N-k] swapped
            // gives conj(A), conj(B) exactly: the sums commute and negation is
            // exact), so each post serves both bins -- half the posts and LDS
            // reads: 5.48 -> 5.17 ms for 32 ch x 10 min.  (At N = 256 the mirror
            // halves are 16-lane, one-float-misaligned 64 B segments whose
            // streaming stores leave partial lines: 2x slower there, and complex
            // rows at 4096 +16 %: not used; profiles/r06_ab_fir_run_stft_sizes.jsonl.)
#pragma unroll
            for (int j = 0; j <= G::P / 2; ++j) {
                const int k = t + G::T * j;
                if (j == G::P / 2 && t != 0) continue;   // bin N/2 (its own mirror): thread 0
                float2 A, B;
                pair_post<MODE>(my[G::pad(k)], my[G::pad((N - k) & (N - 1))], &A, &B);
                const bool mir = MODE != 2 && k != 0 && k != N / 2;   // bin N - k is another bin
                // bases at bins t and N - t: bin k = t + T j and N - k at -T j
                if constexpr (MODE == 1) {
                    float2* ra = reinterpret_cast<float2*>(rowa) + t;
                    float2* rm = reinterpret_cast<float2*>(rowa) + (N - t);
                    st_nt(A, ra + G::T * j);
                    if (mir) st_nt(cconj(A), rm - G::T * j);
                    if (hb) {
                        st_nt(B, ra + (rowb - rowa) / 8 + G::T * j);
                        if (mir) st_nt(cconj(B), rm + (rowb - rowa) / 8 - G::T * j);
                    }
                } else {
                    float* ra = reinterpret_cast<float*>(rowa) + t;
                    float* rm = reinterpret_cast<float*>(rowa) + (N - t);
                    __builtin_nontemporal_store(A.x, ra + G::T * j);
                    if (mir) __builtin_nontemporal_store(A.x, rm - G::T * j);
                    if (hb) {
                        __builtin_nontemporal_store(B.x, ra + rp + G::T * j);
                        if (mir) __builtin_nontemporal_store(B.x, rm + rp - G::T * j);
                    }
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < G::P; ++j) {
                const int k = t + G::T * j;
                if (MODE == 2 && k > N / 2) continue;
                float2 A, B;
                pair_post<MODE>(my[G::pad(k)], my[G::pad((N - k) & (N - 1))], &A, &B);
                if constexpr (MODE == 1) {
                    st_nt(A, reinterpret_cast<float2*>(rowa) + k);
                    if (hb) st_nt(B, reinterpret_cast<float2*>(rowb) + k);
                } else {
                    __builtin_nontemporal_store(A.x, reinterpret_cast<float*>(rowa) + k);
                    if (hb) __builtin_nontemporal_store(B.x, reinterpret_cast<float*>(rowb) + k);
                }
            }
        }
        xsync<G::T>();   // the next pair's FFT exchange reuses `my`
    }
}

// ------------------------------------------------------------------------
// k_stft_one<N>: magnitude rows with ONE frame pair per transform slot and no
// loop (N = 4096) -- no prefetch registers, no persistent walk: the occupancy
// hides the latency and the dispatcher balances the CUs (k_c2c ONE's shape,
// which took c2c 4096 from 0.72 to 0.775).  Slot s of block b takes pair
// (b % 8) per8 + (b / 8) F + s: each XCD (block b runs on XCD b % 8) walks its
// own contiguous eighth of the pairs, so the N + hop - 2 hop overlap of
// neighbouring spans comes from that XCD's L2.  The frames are windowed on load
// (zero past the end of the signal), two per complex FFT; the spectrum goes to
// LDS in natural order and each post serves bin k and its mirror N - k (bit for
// bit the same magnitude), as k_stft_pair_lds<4096>.
// ------------------------------------------------------------------------
// Twiddles of a one-transform kernel whose threads own one last-pass butterfly
// each (T = N/16, e.g. N = 4096): the passes before the last read the LDS
// pass-major table (its first tw_off(LAST) entries: 240 at 4096); the last
// pass' W_N^{t r} (j = t) are powers of W = W_N^t -- one L2 load per thread,
// each power a product of W, W^2, W^4, W^8 (at most four roundings deep) --
// instead of the two-level table's two LDS reads, index arithmetic and complex
// multiply per twiddle.
template <int N>
struct TwPow {
    using G = Geo<N>;
    static constexpr int LAST = G::NPASS - 1, RL = G::RL, NS = G::ns(LAST);
    static_assert(G::T == NS && G::P == RL, "one last-pass butterfly per thread, j = t");
    const float2* tab;
    float2 w[RL - 1];   // w[r - 1] = W^r
    template <int p>
    __device__ __forceinline__ float2 at(int j, int r, int /*i*/ = 0) const {
        if constexpr (p == LAST) return w[r - 1];
        else return tab[G::tw_off(p) + (r - 1) * G::ns(p) + j];
    }
    __device__ __forceinline__ void init(float2 W) {
        w[0] = W;
#pragma unroll
        for (int r = 2; r < RL; ++r) {
            const int hp = 1 << (31 - __builtin_clz(r));   // the highest power of two <= r
            w[r - 1] = r == hp ? cmul(w[hp / 2 - 1], w[hp / 2 - 1]) : cmul(w[hp - 1], w[r - hp - 1]);
        }
    }
};

template <int N, int VAR>
__global__ void __launch_bounds__(Wg<N>::value)
k_stft_one(const float* sig, long long n, long long nch, long long ch_stride, long long frames, long long hop,
           const float* win, float* out, long long out_ch_stride, const float2* gpass, const float2* gtab,
           long long per8) {
    // VAR bits: 1 the samples loaded before the twiddles are staged; 2 the
    // half-size real/imaginary exchange (and spectrum pass), half the LDS per
    // transform; 4 the last pass' twiddles as powers in registers (TwPow)
    // instead of the two-level lo * hi table
    using G = Geo<N>;
    static_assert(G::T >= 64 && G::T % 64 == 0, "whole waves per transform");
    constexpr bool EARLY = VAR & 1, RI = VAR & 2, TLR = VAR & 4;
    constexpr int WG = Wg<N>::value, F = Wg<N>::F, JH = G::P / 2;
    constexpr int XF = RI ? (ri_floats<N>() + 3) / 4 * 2 : G::LDS;   // float2 per transform
    __shared__ __attribute__((aligned(16))) float2 lds[F * XF];
    using TW = std::conditional_t<TLR, TwPow<N>, TwTab<N>>;
    __shared__ float2 ltab[TLR ? G::tw_off(G::NPASS - 1) : TwLayout<N>::ENTRIES];
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T;
    float2* my = lds + slot * XF;
    const long long b = blockIdx.x;
    const long long ppc = (frames + 1) / 2, pairs = nch * ppc;
    const long long p = uni<G::T>((b & 7) * per8 + (b >> 3) * F + slot);
    const bool act = p < pairs;   // uniform per transform
    const long long pc = act ? p : 0;   // an idle slot (F > 1) transforms pair 0 and stores nothing
    // (channel, first frame): 32-bit division (the launcher keeps pairs < 2^31)
    const unsigned cu = (unsigned)pc / (unsigned)ppc;
    const long long c = cu, fa = 2 * (pc - (long long)cu * ppc);
    const float* s = sig + c * ch_stride;
    const long long sa = fa * hop, sb = sa + hop;
    const bool hb = fa + 1 < frames;
    float2 v[G::P];
    auto load = [&]() {
        if (sb + N <= n) {   // both frames inside the signal
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                const float w = 0.5f * win[t + r * G::T];
                v[r] = make_float2(s[sa + t + r * G::T] * w, s[sb + t + r * G::T] * w);
            }
        } else {
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                const long long i = t + r * G::T;
                const float w = 0.5f * win[i];
                const float xa = sa + i < n ? s[sa + i] : 0.0f;
                const float xb = hb && sb + i < n ? s[sb + i] : 0.0f;
                v[r] = make_float2(xa * w, xb * w);
            }
        }
    };
    if constexpr (EARLY) load();
    TW tw{ltab};
    float2 w1 = make_float2(1.0f, 0.0f);
    if constexpr (TLR) {
        w1 = gtab[t];   // W_N^t
        for (int i = threadIdx.x; i < G::tw_off(G::NPASS - 1); i += WG) ltab[i] = gpass[i];
    } else {
        stage_twiddles<N, WG>(ltab, gpass, gtab);
    }
    __syncthreads();
    if constexpr (F == 1) {
        if (!act) return;
    }
    if constexpr (!EARLY) load();
    if constexpr (TLR) tw.init(w1);
    fft_regs<N, true, false, RI, TW>(v, t, my, tw);
    float* ra = out + c * out_ch_stride + fa * N;
    float* rb = ra + N;
    // each post stores bin k and its mirror N - k at once (k <= N/2; the
    // mirror blocks one float off the 256 B grid)
    auto post = [&](const float2* z, const float2* zm) {
#pragma unroll
        for (int j = 0; j <= JH; ++j) {
            const int k = t + G::T * j;
            if (j == JH && t != 0) continue;   // bin N/2 (its own mirror): thread 0
            float2 A, B;
            pair_post<0>(z[j], zm[j], &A, &B);
            const bool mir = k != 0 && k != N / 2;   // bin N - k is another bin
            __builtin_nontemporal_store(A.x, ra + k);
            if (mir) __builtin_nontemporal_store(A.x, ra + N - k);
            if (hb) {
                __builtin_nontemporal_store(B.x, rb + k);
                if (mir) __builtin_nontemporal_store(B.x, rb + N - k);
            }
        }
    };
    float2 z[JH + 1], zm[JH + 1];
    if constexpr (RI) {
        // the spectrum in natural order through the half-size buffer: real
        // parts, then imaginary parts, of bins k and N - k
        float* lf = reinterpret_cast<float*>(my);
#pragma unroll
        for (int q = 0; q < G::P; ++q) lf[G::pad(out_pos<N>(t, q))] = v[q].x;
        xsync<G::T>();
#pragma unroll
        for (int j = 0; j <= JH; ++j) {
            const int k = j < JH ? t + G::T * j : N / 2;
            z[j].x = lf[G::pad(k)];
            zm[j].x = lf[G::pad((N - k) & (N - 1))];
        }
        xsync<G::T>();
#pragma unroll
        for (int q = 0; q < G::P; ++q) lf[G::pad(out_pos<N>(t, q))] = v[q].y;
        xsync<G::T>();
#pragma unroll
        for (int j = 0; j <= JH; ++j) {
            const int k = j < JH ? t + G::T * j : N / 2;
            z[j].y = lf[G::pad(k)];
            zm[j].y = lf[G::pad((N - k) & (N - 1))];
        }
    } else {
#pragma unroll
        for (int q = 0; q < G::P; ++q) my[G::pad(out_pos<N>(t, q))] = v[q];
        xsync<G::T>();
#pragma unroll
        for (int j = 0; j <= JH; ++j) {
            const int k = j < JH ? t + G::T * j : N / 2;
            z[j] = my[G::pad(k)];
            zm[j] = my[G::pad((N - k) & (N - 1))];
        }
    }
    if (!act) return;   // after the last barrier
    post(z, zm);
}

// ------------------------------------------------------------------------
// k_stft_stage<N>: magnitude rows for N = 256 (T = 16 threads per transform,
// four transforms per wave) with every global access a coalesced 16 B per
// lane.  k_stft_pair_lds reads each frame as 16 dword loads of 64 B per slot
// (four frames of four pairs per instruction) and writes each row the same
// way.  Here the four slots of a wave take four consecutive frame pairs of one
// channel (xcd_walk gives a wave's slots consecutive pairs), so the wave's
// eight frames are ONE span of 7 hop + N samples: it comes in as <= 3
// dwordx4 per lane (issued one step ahead, 12 VGPRs instead of 32), is laid
// into the wave's idle exchange buffers, and each slot reads its two frames
// from there.  After the transforms and the mirror-bin posts (bins k <= N/2,
// bin N - k its mirror) the wave's eight rows -- 2048 contiguous floats --
// go back through the same buffers and leave as eight dwordx4 streaming
// stores per lane.  Steps whose four pairs cross a channel, reach past the
// end of the signal (zero padding) or would need an unaligned span take the
// per-slot path with the padding rule, in the same loop (a wave-uniform
// branch).  Bit-identical to k_stft_pair_lds<N, 0> (same transform, same posts).
// ------------------------------------------------------------------------
template <int N>
__global__ void __launch_bounds__(256, 3)
k_stft_stage(const float* sig, long long n, long long nch, long long ch_stride, long long frames, long long hop,
             const float* win, float* out, long long out_ch_stride, const float2* gpass, const float2* gtab) {
    using G = Geo<N>;
    constexpr int T = G::T, NT = 64 / T, F = 256 / T;
    constexpr int WF = NT * G::LDS * 2;        // floats of one wave's exchange buffers
    constexpr int ROWS = 2 * NT * N;           // floats of the wave's eight rows
    constexpr int U = 3;                       // span pieces of 256 floats: 7 hop + N <= 768
    static_assert(T == 16 && ROWS <= WF && U * 256 <= WF, "N = 256: four transforms per wave");
    __shared__ __attribute__((aligned(16))) float2 lds[F * G::LDS];
    __shared__ float2 ltab[TwLayout<N>::ENTRIES];
    stage_twiddles<N, 256>(ltab, gpass, gtab);
    const int lt = threadIdx.x, slot = lt / T, t = lt % T, lane = lt & 63, ws = slot % NT;
    float2* my = lds + slot * G::LDS;
    float* wb = reinterpret_cast<float*>(lds + (slot - ws) * G::LDS);   // the wave's buffers (16 B aligned)
    float w[G::P];   // 0.5 w (pair_post)
#pragma unroll
    for (int r = 0; r < G::P; ++r) w[r] = 0.5f * win[t + r * T];
    __syncthreads();
    const TwTab<N> tw{ltab};
    const long long ppc = (frames + 1) / 2, pairs = nch * ppc;
    long long p, p_end, p_step;
    xcd_walk(pairs, F, slot, &p, &p_end, &p_step);
    long long p0 = uni<64>(p - ws);   // the wave's first pair (its slots hold p0 .. p0 + NT - 1)
    p_end = uni<64>(p_end);
    p_step = uni<64>(p_step);
    const int span = (int)(2 * NT - 1) * (int)hop + N;   // the launcher keeps it <= U * 256
    // wave-uniform: the NT pairs from q0 lie in one channel, all 2 NT frames
    // inside the signal, and their span starts 16 B aligned
    auto staged_ok = [&](long long q0) -> bool {
        if (q0 + NT > p_end) return false;
        const long long c = q0 / ppc, q = q0 - c * ppc;
        if (q + NT > ppc) return false;
        const long long f0 = 2 * q;
        if (f0 + 2 * NT > frames || (f0 + 2 * NT - 1) * hop + N > n) return false;
        return ((c * ch_stride + f0 * hop) & 3) == 0;
    };
    vf4_t pre[U];
    auto issue = [&](long long q0) {
        const long long c = q0 / ppc, f0 = 2 * (q0 - c * ppc);
        const vf4_t* s = reinterpret_cast<const vf4_t*>(sig + c * ch_stride + f0 * hop);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = 4 * lane + 256 * u;
            pre[u] = e < span ? s[e >> 2] : vf4_t{0.0f, 0.0f, 0.0f, 0.0f};   // plain loads: the span overlaps the next wave's (L2)
        }
    };
    bool stg = p0 < p_end && staged_ok(p0);
    if (stg) issue(p0);
    for (; p0 < p_end; p0 += p_step) {
        const long long qq = p0 + ws, q = qq < p_end ? qq : p_end - 1;   // invalid slots redo a valid pair
        const bool qv = qq < p_end;
        const long long c = q / ppc, fa = 2 * (q - c * ppc);
        const bool hb = fa + 1 < frames;
        float xa[G::P], xb[G::P];
        const bool stg0 = stg;
        if (stg0 && hop == 64) {
            // hop 64 (nfft / 4): the span laid out with 16 floats of pad per 128, so
            // the four slots' frames (128 floats apart) read from four distinct bank
            // quarters: unpadded, slots ws and ws + 1 of a 32-lane group hit the
            // same 16 banks on every frame read (a 2-way conflict per instruction)
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (4 * lane + 256 * u < span)
                    *reinterpret_cast<vf4_t*>(wb + 4 * lane + 256 * u + 16 * (lane >> 5) + 32 * u) = pre[u];
            xsync<64>();
            const float* fsa = wb + 144 * ws + t;   // element e at e + 16 (e >> 7)
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                xa[r] = fsa[T * r + 16 * (r >> 3)];
                xb[r] = fsa[64 + T * r + 16 * ((r + 4) >> 3)];
            }
            xsync<64>();
        } else if (stg0) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (4 * lane + 256 * u < span) *reinterpret_cast<vf4_t*>(wb + 4 * lane + 256 * u) = pre[u];
            xsync<64>();
            const float* fsa = wb + 2 * ws * hop + t;
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                xa[r] = fsa[T * r];
                xb[r] = fsa[hop + T * r];
            }
            xsync<64>();
        } else {
            const float* sg = sig + c * ch_stride;
            const long long sa = fa * hop, sb = sa + hop;
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                const long long i = t + r * T;
                xa[r] = sa + i < n ? sg[sa + i] : 0.0f;
                xb[r] = hb && sb + i < n ? sg[sb + i] : 0.0f;
            }
        }
        // the next step's span, in flight across this step's transforms and stores
        stg = p0 + p_step < p_end && staged_ok(p0 + p_step);
        if (stg) issue(p0 + p_step);
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = make_float2(xa[r] * w[r], xb[r] * w[r]);
        fft_regs<N, true>(v, t, my, tw);
#pragma unroll
        for (int k = 0; k < G::P; ++k) my[G::pad(out_pos<N>(t, k))] = v[k];
        xsync<T>();
        float A[G::P / 2 + 1], B[G::P / 2 + 1];
#pragma unroll
        for (int j = 0; j <= G::P / 2; ++j) {
            const int k = t + T * j;
            float2 a, b;
            pair_post<0>(my[G::pad(k & (N - 1))], my[G::pad((N - k) & (N - 1))], &a, &b);
            A[j] = a.x;
            B[j] = b.x;
        }
        xsync<64>();   // every slot of the wave has read its spectrum: the buffers take the rows
        if (stg0) {
            float* ra = wb + 2 * ws * N;
#pragma unroll
            for (int j = 0; j <= G::P / 2; ++j) {
                const int k = t + T * j;
                if (j == G::P / 2 && t != 0) continue;   // bin N/2: thread 0
                ra[k] = A[j];
                ra[N + k] = B[j];
                if (k != 0 && k != N / 2) {
                    ra[N - k] = A[j];
                    ra[2 * N - k] = B[j];
                }
            }
            xsync<64>();
            const long long cw = p0 / ppc, f0 = 2 * (p0 - cw * ppc);
            vf4_t* dst = reinterpret_cast<vf4_t*>(out + cw * out_ch_stride + f0 * N);
#pragma unroll
            for (int u = 0; u < ROWS / 256; ++u)
                __builtin_nontemporal_store(*reinterpret_cast<const vf4_t*>(wb + 4 * lane + 256 * u), dst + lane + 64 * u);
        } else if (qv) {
            float* rowa = out + c * out_ch_stride + fa * N;
            float* r0 = rowa + t;
            float* rm = rowa + (N - t);
#pragma unroll
            for (int j = 0; j <= G::P / 2; ++j) {
                const int k = t + T * j;
                if (j == G::P / 2 && t != 0) continue;
                const bool mir = k != 0 && k != N / 2;
                __builtin_nontemporal_store(A[j], r0 + T * j);
                if (mir) __builtin_nontemporal_store(A[j], rm - T * j);
                if (hb) {
                    __builtin_nontemporal_store(B[j], r0 + N + T * j);
                    if (mir) __builtin_nontemporal_store(B[j], rm + N - T * j);
                }
            }
        }
        xsync<64>();   // the next step's span / exchange reuses the buffers
    }
}

// ------------------------------------------------------------------------
// k_stft_r32<MODE>: power rows (MODE 2) of nfft = 1024, hop = 256 frames with
// the transform split 32 x 32 on half-waves, as k_fir_r32: two frames per
// complex FFT (z = w/2 (a + i b)), two frame pairs per wave (one per half),
// ONE padded LDS transpose per FFT instead of k_stft_pair's two exchanges.
//   lane m2 (residue 2 (m & 15) + (m >> 4), the PAIRED layout): the pair's
//   1280-sample span as 20 dwordx2 loads re-laid by v_permlane16_swap -- frame
//   a = span rows 0..31, frame b = span rows 8..39 (hop = 8 rows) -- times the
//   window, DFT_32 over m1, twiddle W_1024^(m2 k1), transpose, DFT_32 over m2
//   -> Z[m + 32 k2] in register k2 of lane m.
// The mirror bins Z[N - k] (lane 32 - m, register 31 - k2; lane 0: register
// 32 - k2) come back through the same LDS buffer (16 writes, 16 reads), then
// pair_post<2> gives |Xa[k]|^2, |Xb[k]|^2 for bins 0..512 and each half stores
// its pair's two rows, 128 B per instruction.  Spans that reach past the end
// of the signal (the zero-padded tail) are staged through LDS with the zero
// rule, in the same loop.  Persistent grid, static XCD walk over frame-pair
// couples.
// ------------------------------------------------------------------------
// MODE 3 / 4 (log-mel / MFCC rows, launch_stft_mel): the power rows of each
// half's pair go to that half's (now idle) transpose buffer, interleaved bin by
// bin, and the wave runs mel_tail over its two pairs in turn -- the rows equal
// MODE 2's power rows followed by launch_mel_grp, bit for bit.  The plan's
// tables ride in dynamic LDS, so these modes take 8 transform slots per
// workgroup (512 threads, one workgroup and two waves per SIMD per CU) instead of
// two workgroups of 4: the same occupancy with one copy of the tables.
// 33 rows: the mirror read of lane 0 touches row 32; + 1 keeps every buffer 16 B
// aligned (the mel tail's 16 B reads of the power pairs in it)
constexpr int R33_BUF = 33 * R32_ROW + 1;
template <int MODE>
__global__ void __launch_bounds__(MODE >= 3 ? 512 : 256, MODE >= 3 ? 1 : 2)
k_stft_r32(const float* sig, long long n, long long nch, long long ch_stride, long long frames, const float* win,
           float* out, long long out_ch_stride, long long row_pitch, const float2* tw1024, MelArgs mel) {
    static_assert(MODE == 0 || MODE >= 2, "magnitude, power, log-mel or MFCC rows");
    constexpr bool MEL = MODE >= 3;
    constexpr int N = 1024, HOP = 256, F = MEL ? 8 : 4, WG = 64 * F, RW = MODE == 0 ? N : N / 2 + 1, SPAN = N + HOP;
    // floats from one output row's start to the next
    const long long RP = MODE == 2 ? row_pitch : MODE == 3 ? (long long)mel.M : MODE == 4 ? (long long)mel.C : RW;
    __shared__ __attribute__((aligned(16))) float2 xch[F * 2 * R33_BUF];
    __shared__ float2 ltw[32 * 32];   // [r][m] = W_1024^(m r)
    for (int i = threadIdx.x; i < 32 * 32; i += WG) ltw[i] = tw1024[((i & 31) * (i >> 5)) & (N - 1)];
    // MEL: the plan's tables in dynamic LDS: W [nnz], chunks [3 nc], cbeg [M + 1], then (MODE 4) D [C M], lift [C]
    extern __shared__ __attribute__((aligned(16))) float mel_lds[];
    const int mel_dpos = MEL ? (mel.nnz + mel.cw * mel.nc + mel.M + 1 + 3) & ~3 : 0;
    if constexpr (MEL) {
        int* const mi = reinterpret_cast<int*>(mel_lds);
        for (int i = threadIdx.x; i < mel.nnz; i += WG) mel_lds[i] = mel.W[i];
        for (int i = threadIdx.x; i < mel.cw * mel.nc; i += WG) mi[mel.nnz + i] = mel.chunks[i];
        for (int i = threadIdx.x; i <= mel.M; i += WG) mi[mel.nnz + mel.cw * mel.nc + i] = mel.cbeg[i];
        if constexpr (MODE == 4) {
            for (int i = threadIdx.x; i < mel.C * mel.M; i += WG) mel_lds[mel_dpos + i] = mel.D[i];
            for (int i = threadIdx.x; i < mel.C; i += WG) mel_lds[mel_dpos + mel.C * mel.M + i] = mel.lift[i];
        }
    }
    const int lt = threadIdx.x, slot = lt >> 6, lane = lt & 63, half = lane >> 5, m = lane & 31;
    const int mr = 2 * (m & 15) + (m >> 4);   // this lane's input residue
    float2* buf = xch + (2 * slot + half) * R33_BUF;
    // 0.5 w[32 r + mr], two rows per register pair (the 1/2 of the two-frame split rides in the window)
    vf2_t wp[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) wp[i] = vf2_t{0.5f * win[64 * i + mr], 0.5f * win[64 * i + 32 + mr]};
    __syncthreads();
    const long long ppc = (frames + 1) / 2, pairs = nch * ppc, couples = (pairs + 1) / 2;
    long long it, it_end, it_step;
    xcd_walk(couples, F, slot, &it, &it_end, &it_step);
    it = uni<64>(it);
    it_end = uni<64>(it_end);
    it_step = uni<64>(it_step);
    if (it >= it_end) return;
    // pair 2k = (channel c0, pair q0 of it), advanced incrementally (one division per wave)
    long long c0 = (2 * it) / ppc, q0 = 2 * it - c0 * ppc;
    const long long dc = (2 * it_step) / ppc, dq = 2 * it_step - dc * ppc;
    // a couple's rows as the stores see them: both pairs' row offsets (every lane
    // stores 256 B runs of ONE pair per instruction, see below), whether the second
    // pair exists, and whether each pair has its second frame
    struct Rows {
        long long oa, ob;
        bool two, ha, hb;
    };
    auto locate = [&](long long k, long long* c, long long* q, bool* valid, bool* edge_any, Rows* rw) {
        const bool two = 2 * k + 1 < pairs;
        const bool wrap = q0 + 1 == ppc;
        const long long c1 = two ? c0 + (wrap ? 1 : 0) : c0, q1 = two ? (wrap ? 0 : q0 + 1) : q0;
        *valid = !half || two;
        *c = half ? c1 : c0;
        *q = half ? q1 : q0;
        *edge_any = 2 * q0 * HOP + SPAN > n || 2 * q1 * HOP + SPAN > n;
        rw->oa = c0 * out_ch_stride + 2 * q0 * RP;
        rw->ob = c1 * out_ch_stride + 2 * q1 * RP;
        rw->two = two;
        rw->ha = 2 * q0 + 1 < frames;
        rw->hb = 2 * q1 + 1 < frames;
    };
    float xa[32], xt[8];   // span rows 0..31 (frame a) and 32..39 (frame b's rows 24..31)
    auto load_bulk = [&](long long c, long long q) {
        const float2* a = reinterpret_cast<const float2*>(sig + c * ch_stride + 2 * q * HOP) + m;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float2 u = ld_nt(a + 32 * i);
            xa[2 * i] = u.x;
            xa[2 * i + 1] = u.y;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float2 u = a[32 * (16 + i)];   // the next pair's span starts here: cached
            xt[2 * i] = u.x;
            xt[2 * i + 1] = u.y;
        }
    };
    // edge couples: the span through LDS with the zero rule (rolled loop), then the
    // residue layout directly (no swap)
    auto load_edge = [&](long long c, long long q) {
        const float* xs = sig + c * ch_stride;
        float* sf = reinterpret_cast<float*>(buf);
        const long long s0 = 2 * q * HOP;
#pragma unroll 1
        for (int k = m; k < SPAN; k += 32) sf[k] = s0 + k < n ? xs[s0 + k] : 0.0f;
        xsync<64>();
#pragma unroll
        for (int r = 0; r < 32; ++r) xa[r] = sf[32 * r + mr];
#pragma unroll
        for (int r = 0; r < 8; ++r) xt[r] = sf[N + 32 * r + mr];
        xsync<64>();
    };
    long long c, q;
    bool valid, edge;
    Rows rw;
    locate(it, &c, &q, &valid, &edge, &rw);
    if (!edge) load_bulk(c, q);
    for (; it < it_end; it += it_step) {
        if (edge) {
            load_edge(c, q);
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) r32_pairswap(xa[2 * i], xa[2 * i + 1]);
#pragma unroll
            for (int i = 0; i < 4; ++i) r32_pairswap(xt[2 * i], xt[2 * i + 1]);
        }
        // v[r] = 0.5 w_r (a_r, b_r), b_r = span row r + 8
        float2 v[32];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const vf2_t A = {xa[2 * i], xa[2 * i + 1]};
            const vf2_t B = i < 12 ? vf2_t{xa[2 * i + 8], xa[2 * i + 9]} : vf2_t{xt[2 * i - 24], xt[2 * i - 23]};
            v[2 * i] = upk(pk_mul_bcast<0>(pk_pair<0>(A, B), wp[i]));
            v[2 * i + 1] = upk(pk_mul_bcast<1>(pk_pair<1>(A, B), wp[i]));
        }
        const long long itn = it + it_step;
        long long cn = c, qn = q;
        bool validn = valid, edgen = edge;
        Rows rwn = rw;
        if (itn < it_end) {   // the next couple's span, in flight across this one's transform
            q0 += dq;
            c0 += dc;
            if (q0 >= ppc) {
                q0 -= ppc;
                ++c0;
            }
            locate(itn, &cn, &qn, &validn, &edgen, &rwn);
            if (!edgen) load_bulk(cn, qn);
        }
        dft32<true>(v);
        r32_twiddle<true>(v, ltw + mr);
        r32_transpose(v, buf, mr, m);
        dft32<true>(v);
        // Z[N - k] (lane 32 - m, register 31 - r; lane 0: register 32 - r) through the
        // buffer: registers 16..31 for the power rows' bins 0..512, all 32 for the
        // magnitude rows, whose upper half each lane computes from its own
        // registers 16..31 (the same roundings as the mirror's: |X[N - k]| = |X[k]|
        // bit for bit), so every store has the lanes in address order
#pragma unroll
        for (int r = MODE == 0 ? 0 : 16; r < 32; ++r) buf[R32_ROW * r + m] = v[r];
        xsync<64>();
        float2 zm[16];   // zm[15 - k2] = Z[N - (m + 32 k2)], k2 < 16
        lds_rd64x16<0, 8 * R32_ROW>(buf + R32_ROW * (m == 0 ? 17 : 16) + ((32 - m) & 31), zm);
        float2 zu[16];   // MODE 0: zu[31 - r] = Z[N - (m + 32 r)], r >= 16 (lane 0, r = 16: Z[512] itself)
        if constexpr (MODE == 0) lds_rd64x16<0, 8 * R32_ROW>(buf + R32_ROW * (m == 0 ? 1 : 0) + ((32 - m) & 31), zu);
        xsync<64>();   // the next couple's transpose writes stay behind these reads
        if constexpr (MODE == 0) {
            // magnitude rows, all N bins: lane m holds bin m + 32 r of its pair's two
            // rows, r < 32.  Blocks 2j, 2j + 1 of one row are an aligned 256 B run: one
            // v_permlane32_swap per register pair moves half 0's block 2j + 1 up and half
            // 1's block 2j down, so each store writes 256 B of ONE pair's row (the first
            // pair's, then the second's) -- the 64-lane width of k_stft_pair's stores.
            float A[32], B[32];
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                float2 pa, pb;
                pair_post<0>(v[r], r < 16 ? ((r == 0 && m == 0) ? v[0] : zm[15 - r]) : zu[31 - r], &pa, &pb);
                A[r] = pa.x;
                B[r] = pb.x;
            }
            const int lo = half * 32 + m;   // this lane's float in a 256 B run
            float* ra = out + rw.oa + lo;
            float* rb = out + rw.ob + lo;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                r32_halfswap(A[2 * j], A[2 * j + 1]);
                r32_halfswap(B[2 * j], B[2 * j + 1]);
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) __builtin_nontemporal_store(A[2 * j], ra + 64 * j);
            if (rw.two) {
#pragma unroll
                for (int j = 0; j < 16; ++j) __builtin_nontemporal_store(A[2 * j + 1], rb + 64 * j);
            }
            if (rw.ha) {
#pragma unroll
                for (int j = 0; j < 16; ++j) __builtin_nontemporal_store(B[2 * j], ra + RW + 64 * j);
            }
            if (rw.two && rw.hb) {
#pragma unroll
                for (int j = 0; j < 16; ++j) __builtin_nontemporal_store(B[2 * j + 1], rb + RW + 64 * j);
            }
        }
        if constexpr (MODE == 2) {
            const long long fa = 2 * q;
            float* rowa = out + c * out_ch_stride + fa * RP + m;
            float* rowb = rowa + RP;
            const bool hb = fa + 1 < frames;
            float A[16], B[16];
#pragma unroll
            for (int k2 = 0; k2 < 16; ++k2) {
                float2 pa, pb;
                pair_post<2>(v[k2], (k2 == 0 && m == 0) ? v[0] : zm[15 - k2], &pa, &pb);
                A[k2] = pa.x;
                B[k2] = pb.x;
            }
            float2 na, nb;   // bin 512: Z[512] is its own mirror (lane 0, register 16)
            pair_post<2>(v[16], v[16], &na, &nb);
            if (valid && m == 0) {   // each half's lane 0: its own pair's bin 512
                rowa[512] = na.x;
                if (hb) rowb[512] = nb.x;
            }
            // bins 0..511 as 256 B runs of one pair's row per store (v_permlane32_swap,
            // as the magnitude rows)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                r32_halfswap(A[2 * j], A[2 * j + 1]);
                r32_halfswap(B[2 * j], B[2 * j + 1]);
            }
            const int lo = half * 32 + m;
            float* pa = out + rw.oa + lo;
            float* pb = out + rw.ob + lo;
#pragma unroll
            for (int j = 0; j < 8; ++j) pa[64 * j] = A[2 * j];
            if (rw.two) {
#pragma unroll
                for (int j = 0; j < 8; ++j) pb[64 * j] = A[2 * j + 1];
            }
            if (rw.ha) {
#pragma unroll
                for (int j = 0; j < 8; ++j) pa[RP + 64 * j] = B[2 * j];
            }
            if (rw.two && rw.hb) {
#pragma unroll
                for (int j = 0; j < 8; ++j) pb[RP + 64 * j] = B[2 * j + 1];
            }
        }
        if constexpr (MEL) {
            // this half's pair: power of bins m + 32 k2 (k2 < 16) and bin 512 (lane
            // 0) into its buffer as P[2k] = |Xa[k]|^2, P[2k + 1] = |Xb[k]|^2
            float* P = reinterpret_cast<float*>(buf);
#pragma unroll
            for (int k2 = 0; k2 < 16; ++k2) {
                float2 pa, pb;
                pair_post<2>(v[k2], (k2 == 0 && m == 0) ? v[0] : zm[15 - k2], &pa, &pb);
                *reinterpret_cast<vf2_t*>(P + 2 * (m + 32 * k2)) = vf2_t{pa.x, pb.x};
            }
            float2 na, nb;   // bin 512: Z[512] is its own mirror (lane 0, register 16)
            pair_post<2>(v[16], v[16], &na, &nb);
            if (m == 0) {
                *reinterpret_cast<vf2_t*>(P + 2 * (N / 2)) = vf2_t{na.x, nb.x};
                if constexpr (MelArgs::W2) {   // zeros under the last windows' tails (as mel_rows)
#pragma unroll
                    for (int z = 1; z <= 3; ++z) *reinterpret_cast<vf2_t*>(P + 2 * (N / 2 + z)) = vf2_t{0.0f, 0.0f};
                }
            }
            xsync<64>();
            const int* mi = reinterpret_cast<const int*>(mel_lds);
            for (int h = 0; h < 2; ++h) {   // the two pairs in turn, each over the whole wave
                if (h == 1 && !rw.two) break;
                float* Ph = reinterpret_cast<float*>(xch + (2 * slot + h) * R33_BUF);
                float* fa_row = out + (h ? rw.ob : rw.oa);
                mel_tail<MODE, false>(lane, Ph, fa_row, fa_row + RP, h ? rw.hb : rw.ha, nullptr, mel_lds,
                                      mi + mel.nnz, mi + mel.nnz + mel.cw * mel.nc, mel_lds + mel_dpos,
                                      mel_lds + mel_dpos + mel.C * mel.M, mel);
            }
            xsync<64>();   // the next couple's transpose writes stay behind the tails' reads
        }
        c = cn;
        q = qn;
        valid = validn;
        edge = edgen;
        rw = rwn;
    }
}

// The 32 x 32 kernels' shape (k_stft_r32): hop 256, 8 B aligned channel starts.
// Power rows and the fused log-mel / MFCC rows share this rule, so the fused
// rows always come from the same FFT as the power rows they must equal.
static bool stft_r32_ok(long long hop, const float* sig, long long nch, long long ch_stride) {
    return hop == 256 && ((uintptr_t)sig & 7) == 0 && (nch == 1 || (ch_stride & 1) == 0);
}

template <int N, int MODE>
static hipError_t run_stft(const float* sig, long long n, long long nch, long long ch_stride,
                           long long frames, long long hop, const float* win, void* out,
                           long long out_ch_stride, hipStream_t s, long long row_pitch) {
    if (MODE != 2 || row_pitch <= 0) row_pitch = MODE == 2 ? N / 2 + 1 : N;   // packed rows
    if constexpr (MODE == 0 && N == 4096) {
        // one frame pair per transform slot, no loop (k_stft_one VAR 5: the loads
        // before the twiddle staging, the last pass' twiddles as powers in
        // registers): 5.07 -> 4.13 ms for 32 ch x 10 min against k_stft_pair_lds
        // (0.454 -> 0.558 of HBM; profiles/r06_ab_stft4096_one.jsonl: the
        // half-size exchange at five workgroups per CU, the lane-0 trade for
        // aligned mirror blocks and the two-level twiddle table were slower).
        // Knob STFT_ONE = 0 keeps k_stft_pair_lds (A/B)
        if (knob(KNOB_STFT_ONE, 1) != 0 && nch * ((frames + 1) / 2) < (1LL << 31)) {
            const float2* tN = twiddle_table(N);
            const float2* pN = pass_twiddles(N);
            if (!tN || !pN) return hipErrorOutOfMemory;
            constexpr int F = Wg<N>::F;
            const long long pairs = nch * ((frames + 1) / 2);
            const long long per8 = ((pairs + 8 * F - 1) / (8 * F)) * F;   // pairs per XCD, whole blocks
            const long long grid = 8 * (per8 / F);
            if (pairs < 1) return hipSuccess;
            hipLaunchKernelGGL((k_stft_one<N, 5>), dim3((unsigned)grid), dim3(Wg<N>::value), 0, s, sig, n, nch,
                               ch_stride, frames, hop, win, (float*)out, out_ch_stride, pN, tN, per8);
            return hipGetLastError();
        }
    }
    if constexpr (Geo<N>::CAN_PAIR) {
        const float2* tN = twiddle_table(N);
        const float2* pN = pass_twiddles(N);
        if (!tN || !pN) return hipErrorOutOfMemory;
        constexpr int WG = Wg<N>::value, F = Wg<N>::F;
        // pairs whose two frames lie inside the signal, then the zero-padded tail
        const long long nfull = n >= N ? (n - N) / hop + 1 : 0;
        const long long ppc = (frames + 1) / 2;
        long long mpc = (nfull < frames ? nfull : frames) / 2;
        if (mpc > ppc) mpc = ppc;
        const long long tpc = ppc - mpc;
        static std::atomic<int> capc[7];   // zero-initialised (static storage)
        // The bulk launch is NOT persistent: one workgroup per `cps` pairs per
        // transform slot, so the hardware dispatcher balances the CUs and the
        // launch has no straggler tail (measured 8-13 % faster than the
        // persistent walk at 16-64 pairs per slot; profiles/r01_kbench_chunk.jsonl).
        // Small jobs use fewer pairs per slot: just enough that the grid fits the
        // resident workgroup slots once (one round, every wave pipelining its
        // pairs) instead of a few long chains or several short rounds.
        const long long bulk_pairs = nch * ppc;
        const int cap0 = cached_grid(capc[0], (const void*)k_stft_pair<N, MODE, 0>, WG, 0, 1LL << 40);
        long long cps = (bulk_pairs + (long long)F * cap0 - 1) / ((long long)F * cap0);
        cps = cps < 1 ? 1 : (cps > 16 ? 16 : cps);
        {   // A/B knob (scripts/kbench.py stftcps*): an upper bound on the pairs per slot
            const long long cmax = knob(KNOB_STFT_CPS, 0);
            if (cmax > 0 && cps > cmax) cps = cmax;
        }
        float* sink = store_sink();
        if (!sink) return hipErrorOutOfMemory;
        unsigned* ctrs = nullptr;
        auto launch = [&](auto kern, int var, long long pair0, long long cnt) {
            const int capv = cached_grid(capc[var], (const void*)kern, WG, 0, 1LL << 40);
            const long long need = (nch * cnt + F - 1) / F;
            long long grid = need < capv ? need : capv;
            long long chunk = 0;
            if (var == 0 || var == 3) {
                chunk = cps * F;
                grid = (nch * cnt + chunk - 1) / chunk;
            }
            if (var == 4 || var == 5) grid = capv / 8 * 8;   // persistent, the same number of blocks per XCD group
            if (var == 5) {   // pairs per counter value; knob STFT_RUN overrides (A/B)
                long long rl = knob(KNOB_STFT_RUN, 2);
                if (rl < 1 || rl > 64) rl = 2;
                long long dbs = knob(KNOB_STFT_DBS, 6);   // band: 2^dbs runs per (XCD group, slot) stream (A/B)
                if (dbs < 0 || dbs > 12) dbs = 6;
                chunk = (rl << 40) | dbs;
            }
            if (var == 3) {   // run length (pairs), a divisor of cps; knob STFT_RUN overrides (A/B)
                long long rl = knob(KNOB_STFT_RUN, cps);
                if (rl < 1 || cps % rl) rl = cps;
                chunk |= rl << 40;
            }
            hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(WG), 0, s, sig, n, nch, ch_stride, frames, hop, pair0,
                               cnt, win, out, out_ch_stride, row_pitch, pN, tN, chunk, sink, ctrs, MelArgs{});
        };
        // 16 B aligned output rows allow the staged 16 B/lane stores
        // (power rows are n/2+1 floats: their direct stores are dwords, 4 B suffice;
        // complex rows are stored 8 B per lane)
        bool aligned = MODE == 2   ? ((uintptr_t)out & 3) == 0
                       : MODE == 1 ? ((uintptr_t)out & 7) == 0
                                   : ((uintptr_t)out & 15) == 0 && (out_ch_stride & 3) == 0 && N >= 4;
        // T >= 64: VAR 0 also reads its input spans by 16 B LDS-DMA
        if (Geo<N>::T >= 64)
            aligned = aligned && hop % 4 == 0 && hop <= N / 2 && ((uintptr_t)sig & 15) == 0 && (ch_stride & 3) == 0;
        if (MODE != 0 && knob(KNOB_POW_OLD, 0) == 1) aligned = false;   // A/B: register loads, per-bin stores
        // the VAR 0 kernels that read spans by LDS-DMA run the tail pairs too:
        // one launch for the whole job
        constexpr bool FUSE_TAIL = (MODE == 0 || Geo<N>::T == 64) && Geo<N>::NPASS > 1 && Geo<N>::T >= 64;
        // ring spans (VAR 3) when the span is whole 256-float chunks: power rows only
        // (2.74 vs 2.84 ms for 32 ch x 10 min; magnitude and complex rows measured
        // 1-2 % slower than with VAR 0's interleaved walk, profiles/r02_kbench_ring.jsonl).
        // knob STFT_RING = 0 / 1 forces VAR 0 / VAR 3 (A/B)
        const long long kring = knob(KNOB_STFT_RING, -1);
        const bool ring = Geo<N>::T == 64 && hop == 256 && (kring >= 0 ? kring == 1 : MODE == 2);
        // Magnitude and complex rows of large jobs: the persistent dynamic walk (VAR 4) --
        // each wave takes its next pair from a per-(XCD group, slot) counter, so
        // the chip sweeps one moving band of pairs with the load balanced on the
        // fly (-1.6 % against the chunked launch in two same-buffer measurements,
        // profiles/r03_kbench_ablation_samebuf.jsonl lab8192; bit-identical rows).
        // Knob STFT_DYN = 0 keeps the chunked VAR 0 (A/B).
        // Complex rows take it too (1.629 -> 1.579 ms for 8 ch x 10 min, -3.1 %);
        // power rows keep the ring walk below (2.689 ring vs 2.730 dynamic vs
        // 2.760 chunked, profiles/r03_kbench_dyn_modes.jsonl).  Knob STFT_DYN =
        // 1 forces it for every row kind (A/B).
        // power rows, nfft 1024 / hop 256, 8 B aligned channels: the 32 x 32 split
        // (k_stft_r32) on knob POW_R32 = 1 (A/B; round 5, same buffers: 3.02 ms
        // against the ring walk's 2.70 for 32 ch x 10 min -- its 128 B half-wave
        // stores leave in a burst at two waves per SIMD)
        if constexpr (N == 1024 && MODE == 2) {
            if (stft_r32_ok(hop, sig, nch, ch_stride) && knob(KNOB_POW_R32, 0) == 1) {
                static std::atomic<int> capr;
                const int cap = cached_grid(capr, (const void*)k_stft_r32<2>, 256, 0, 1LL << 40);
                const long long couples = (nch * ppc + 1) / 2, need = (couples + 3) / 4;
                const int grid = (int)(need < cap ? need : cap);
                if (grid < 1) return hipSuccess;
                stat_inc(STAT_POW_R32);
                hipLaunchKernelGGL((k_stft_r32<2>), dim3(grid), dim3(256), 0, s, sig, n, nch, ch_stride, frames, win,
                                   (float*)out, out_ch_stride, row_pitch, tN, MelArgs{});
                return hipGetLastError();
            }
        }
        if constexpr (N == 1024 && MODE == 0) {   // magnitude rows: the same split on knob MAG_R32 = 1 (A/B)
            if (hop == 256 && knob(KNOB_MAG_R32, 0) == 1 && ((uintptr_t)sig & 7) == 0 &&
                (nch == 1 || (ch_stride & 1) == 0) && ((uintptr_t)out & 127) == 0 && (out_ch_stride & 31) == 0) {
                static std::atomic<int> capm;
                const int cap = cached_grid(capm, (const void*)k_stft_r32<0>, 256, 0, 1LL << 40);
                const long long couples = (nch * ppc + 1) / 2, need = (couples + 3) / 4;
                const int grid = (int)(need < cap ? need : cap);
                if (grid < 1) return hipSuccess;
                stat_inc(STAT_MAG_R32);
                hipLaunchKernelGGL((k_stft_r32<0>), dim3(grid), dim3(256), 0, s, sig, n, nch, ch_stride, frames, win,
                                   (float*)out, out_ch_stride, row_pitch, tN, MelArgs{});
                return hipGetLastError();
            }
        }
        const long long kdyn = knob(KNOB_STFT_DYN, -1);
        bool dyn = false;
        if constexpr (Geo<N>::T == 64) {
            const int capd = cached_grid(capc[4], (const void*)k_stft_pair<N, MODE, 4>, WG, 0, 1LL << 40);
            const bool want = kdyn >= 0 ? kdyn != 0 : (MODE == 0 || MODE == 1);
            dyn = aligned && FUSE_TAIL && want && capd >= 8 &&
                  bulk_pairs >= 16LL * F * capd;   // >= 16 pairs per wave: the band walk pays off
            if (dyn) {   // no counter block (pool exhausted, or first use inside a capture): static walk
                ctrs = stream_counters(s);
                dyn = ctrs != nullptr;
            }
        }
        // Magnitude rows with whole-chunk hops: the dynamic walk in runs of 2
        // pairs on a ring (VAR 5): 3.357 vs 3.440 ms (VAR 4) vs 3.501 ms (chunked)
        // for 32 ch x 10 min, runs of 1 / 3 / 4 / 8 / 16 slower; power and complex
        // rows measured 1-4 % slower with it (profiles/r03_kbench_dynring.jsonl).
        // knob STFT_DYN = 1 / 2 forces VAR 4 / VAR 5 (A/B)
        const bool dring = kdyn >= 0 ? kdyn == 2 : MODE == 0;
        if (dyn) stat_inc(STAT_STFT_DYN);
        if (dyn && dring && hop == 256) {
            if constexpr (Geo<N>::T == 64) launch(k_stft_pair<N, MODE, 5>, 5, 0LL, ppc);
        } else if (dyn) {
            if constexpr (Geo<N>::T == 64) launch(k_stft_pair<N, MODE, 4>, 4, 0LL, ppc);
        } else if (aligned && FUSE_TAIL && ring) {
            if constexpr (Geo<N>::T == 64) launch(k_stft_pair<N, MODE, 3>, 3, 0LL, ppc);
        } else if (aligned && FUSE_TAIL) {
            launch(k_stft_pair<N, MODE, 0>, 0, 0LL, ppc);
        } else {
            if (mpc > 0) {
                if (aligned) launch(k_stft_pair<N, MODE, 0>, 0, 0LL, mpc);
                else launch(k_stft_pair<N, MODE, 1>, 1, 0LL, mpc);
            }
            if (tpc > 0) launch(k_stft_pair<N, MODE, 2>, 2, mpc, tpc);
        }
    } else {
        // frame pairs with the mirror bins read back through LDS (k_stft_pair_lds;
        // it replaced round 1's one-frame-per-half-length-FFT kernel, now gone)
        const float2* tN = twiddle_table(N);
        const float2* pN = pass_twiddles(N);
        if (!tN || !pN) return hipErrorOutOfMemory;
        constexpr int WG = Wg<N>::value, F = Wg<N>::F;
        if constexpr (N == 256 && MODE == 0) {
            // magnitude rows with every global access 16 B per lane (k_stft_stage);
            // knob STFT_STAGE = 0 keeps k_stft_pair_lds (A/B)
            if (7 * hop + N <= 768 && hop % 4 == 0 && ((uintptr_t)sig & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
                (out_ch_stride & 3) == 0 && knob(KNOB_STFT_STAGE, 1) != 0) {
                static std::atomic<int> caps;
                const int cap = cached_grid(caps, (const void*)k_stft_stage<N>, 256, 0, 1LL << 40);
                const long long need = (nch * ((frames + 1) / 2) + F - 1) / F;
                const int grid = (int)(need < cap ? need : cap);
                if (grid < 1) return hipSuccess;
                hipLaunchKernelGGL((k_stft_stage<N>), dim3(grid), dim3(256), 0, s, sig, n, nch, ch_stride, frames, hop,
                                   win, (float*)out, out_ch_stride, pN, tN);
                return hipGetLastError();
            }
        }
        static std::atomic<int> capl;
        const int cap = cached_grid(capl, (const void*)k_stft_pair_lds<N, MODE>, WG, 0, 1LL << 40);
        const long long need = (nch * ((frames + 1) / 2) + F - 1) / F;
        const int grid = (int)(need < cap ? need : cap);
        if (grid < 1) return hipSuccess;
        hipLaunchKernelGGL((k_stft_pair_lds<N, MODE>), dim3(grid), dim3(WG), 0, s, sig, n, nch, ch_stride, frames,
                           hop, win, out, out_ch_stride, row_pitch, pN, tN);
    }
    return hipGetLastError();
}

bool stft_fused_supported(long long nfft) {
    return nfft >= 2 && nfft <= 8192 && (nfft & (nfft - 1)) == 0;
}

// Signal -> log-mel (kind 0) / MFCC (kind 1) rows in one launch (k_stft_pair
// MODE 3 / 4, N = 1024).  The launch follows run_stft's bulk path: the chunked
// non-persistent grid, or the dynamic walk for large jobs; the plan's tables
// ride in dynamic LDS, so the occupancy is computed per call.
template <int MODE>
static hipError_t run_stft_mel(const float* sig, long long n, long long nch, long long ch_stride, long long frames,
                               long long hop, const float* win, const MelArgs& mel_in, float* out,
                               long long out_ch_stride, hipStream_t s) {
    constexpr int N = 1024, WG = Wg<N>::value, F = Wg<N>::F;
    const float2* tN = twiddle_table(N);
    const float2* pN = pass_twiddles(N);
    float* sink = store_sink();
    if (!tN || !pN || !sink) return hipErrorOutOfMemory;
    const long long ppc = (frames + 1) / 2, pairs = nch * ppc;
    if (pairs <= 0) return hipSuccess;
    // the plan's tables in dynamic LDS (the kernel's layout); occupancy per call
    auto dyn_of = [&](const MelArgs& a) {
        const long long dp = (a.nnz + (long long)a.cw * a.nc + a.M + 1 + 3) & ~3LL;
        return sizeof(float) * (size_t)(dp + (MODE == 4 ? (long long)a.C * a.M + a.C : 0));
    };
    // log-mel (MODE 3): the chunk windows (cw = 0); MFCC: the windows too when
    // they keep the packed table's workgroups per CU, else the packed chunks
    MelArgs mel = mel_in;
    auto windows = [&](MelArgs& a) {
        a.W = mel_in.Ww;
        a.chunks = nullptr;
        a.cw = 0;
        a.lc = mel_in.lcw;
        a.lcs = MelArgs::window_stride(mel_in.lcw);
        a.nnz = mel_in.nc * a.lcs;
    };
    const bool have_w = mel_in.Ww && mel_in.lcw > 0 && mel_in.lcw % 4 == 0;
    if constexpr (MODE == 3) {
        if (!have_w) return hipErrorNotSupported;
        windows(mel);
    } else if (have_w && knob(KNOB_MFCC_WIN, 1) != 0) {   // knob MFCC_WIN = 0: the packed chunks (A/B)
        MelArgs mw = mel_in;
        windows(mw);
        int pw = 0, pp = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pw, (const void*)k_stft_pair<N, MODE, 0>, WG, dyn_of(mw)) ==
                hipSuccess &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&pp, (const void*)k_stft_pair<N, MODE, 0>, WG,
                                                         dyn_of(mel_in)) == hipSuccess &&
            pw >= pp)
            mel = mw;
    }
    const size_t dyn = dyn_of(mel);
    // knob MEL_R32 = 1 (with POW_R32 = 1, so the fused rows stay bit-identical to
    // the power rows + launch_mel_grp): the 32 x 32 split (A/B; round 5, same
    // buffers: log-mel 3.38 / MFCC 4.02 ms against 3.21 / 3.52 for 32 ch x 10 min
    // -- two serial mel tails per wave at two waves per SIMD)
    if (stft_r32_ok(hop, sig, nch, ch_stride) && knob(KNOB_MEL_R32, 0) == 1 && knob(KNOB_POW_R32, 0) == 1) {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_stft_r32<MODE>, 512, dyn) ==
                hipSuccess &&
            per_cu >= 1) {
            const int cap = persistent_grid((const void*)k_stft_r32<MODE>, 512, dyn, 1LL << 40);
            const long long couples = (pairs + 1) / 2, need = (couples + 7) / 8;
            const int grid = (int)(need < cap ? need : cap);
            stat_inc(STAT_MEL_R32);
            hipLaunchKernelGGL((k_stft_r32<MODE>), dim3(grid), dim3(512), dyn, s, sig, n, nch, ch_stride, frames, win,
                               out, out_ch_stride, 0LL, tN, mel);
            return hipGetLastError();
        }
    }
    const int cap = persistent_grid((const void*)k_stft_pair<N, MODE, 0>, WG, dyn, 1LL << 40);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_stft_pair<N, MODE, 0>, WG, dyn) !=
            hipSuccess ||
        per_cu < 1)
        return hipErrorNotSupported;
    unsigned* ctrs = nullptr;
    bool dyn_walk = knob(KNOB_STFT_DYN, -1) != 0 && cap >= 8 && pairs >= 16LL * F * cap;
    if (dyn_walk) {   // no counter block: the chunked walk (bit-identical)
        ctrs = stream_counters(s);
        dyn_walk = ctrs != nullptr;
    }
    long long grid, chunk = 0;
    if (dyn_walk) {
        grid = cap / 8 * 8;
    } else {
        long long cps = (pairs + (long long)F * cap - 1) / ((long long)F * cap);
        cps = cps < 1 ? 1 : (cps > 16 ? 16 : cps);
        chunk = cps * F;
        grid = (pairs + chunk - 1) / chunk;
    }
    if (dyn_walk)
        hipLaunchKernelGGL((k_stft_pair<N, MODE, 4>), dim3((unsigned)grid), dim3(WG), dyn, s, sig, n, nch, ch_stride,
                           frames, hop, 0LL, ppc, win, (void*)out, out_ch_stride, 0LL, pN, tN, chunk, sink, ctrs, mel);
    else
        hipLaunchKernelGGL((k_stft_pair<N, MODE, 0>), dim3((unsigned)grid), dim3(WG), dyn, s, sig, n, nch, ch_stride,
                           frames, hop, 0LL, ppc, win, (void*)out, out_ch_stride, 0LL, pN, tN, chunk, sink, ctrs, mel);
    return hipGetLastError();
}

hipError_t launch_stft_mel(int kind, long long nfft, long long hop, const float* sig, long long n, long long nch,
                           long long ch_stride, long long frames, const float* win, const MelArgs& mel, float* out,
                           long long out_ch_stride, hipStream_t s) {
    // the LDS-DMA span path's conditions (run_stft's `aligned`), one store
    // instruction per 64 output values, and power rows of this nfft
    const bool shape_ok = nfft == 1024 && hop % 4 == 0 && hop <= 256 && ((uintptr_t)sig & 15) == 0 &&
                          (ch_stride & 3) == 0 && mel.M >= 1 && mel.M <= 128 && mel.nc <= 64 * MEL_MAX_ROUNDS &&
                          mel.cw == 3 &&
                          (kind == 0 || (mel.C >= 1 && mel.C <= 64 && 2 * mel.M <= ri_floats<1024>() - MEL_LM_OFF));
    if (!shape_ok || (kind != 0 && kind != 1)) return hipErrorNotSupported;
    return kind == 0 ? run_stft_mel<3>(sig, n, nch, ch_stride, frames, hop, win, mel, out, out_ch_stride, s)
                     : run_stft_mel<4>(sig, n, nch, ch_stride, frames, hop, win, mel, out, out_ch_stride, s);
}

hipError_t launch_stft(long long nfft, long long hop, int mode, const float* sig, long long n,
                       long long nch, long long ch_stride, long long frames, const float* win,
                       void* out, long long out_ch_stride, hipStream_t s, long long row_pitch) {
#define CALL(NN)                                                                                                \
    (mode == 0   ? run_stft<NN, 0>(sig, n, nch, ch_stride, frames, hop, win, out, out_ch_stride, s, 0)         \
     : mode == 1 ? run_stft<NN, 1>(sig, n, nch, ch_stride, frames, hop, win, out, out_ch_stride, s, 0)         \
                 : run_stft<NN, 2>(sig, n, nch, ch_stride, frames, hop, win, out, out_ch_stride, s, row_pitch))
    switch (nfft) {
        case 2: return CALL(2); case 4: return CALL(4); case 8: return CALL(8); case 16: return CALL(16);
        case 32: return CALL(32); case 64: return CALL(64); case 128: return CALL(128);
        case 256: return CALL(256); case 512: return CALL(512); case 1024: return CALL(1024);
        case 2048: return CALL(2048); case 4096: return CALL(4096); case 8192: return CALL(8192);
        default: return hipErrorInvalidValue;
    }
#undef CALL
}

// stft_process over explicit frames [count][nfft] (no overlap): same kernels, hop = nfft.
hipError_t launch_stft_frames(long long nfft, const float* frames_in, const float* win, float2* out,
                              long long count, hipStream_t s) {
    return launch_stft(nfft, nfft, 1, frames_in, nfft * count, 1, 0, count, win, out, 0, s);
}

// ---- generic path (any nfft): gather windowed complex frames, then a batched
// C2C plan, then magnitudes.
__global__ void k_frame_gather(long long nfft, long long hop, const float* sig, long long n,
                               long long nch, long long ch_stride, long long frames,
                               const float* win, float2* out) {
    const long long total = nch * frames * nfft;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long e = i % nfft, fr = (i / nfft) % frames, c = i / (nfft * frames);
        const long long idx = fr * hop + e;
        const float v = (idx < n) ? sig[c * ch_stride + idx] : 0.0f;
        out[i] = make_float2(v * win[e], 0.0f);
    }
}

hipError_t launch_frame_gather(long long nfft, long long hop, const float* sig, long long n,
                               long long nch, long long ch_stride, long long frames, const float* win,
                               float2* out, hipStream_t s) {
    const long long total = nch * frames * nfft;
    if (total <= 0) return hipSuccess;
    long long blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_frame_gather, dim3((unsigned)blocks), dim3(256), 0, s, nfft, hop, sig, n, nch,
                       ch_stride, frames, win, out);
    return hipGetLastError();
}

__global__ void k_magnitude(const float2* in, float* out, long long count) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < count;
         i += (long long)gridDim.x * blockDim.x) {
        const float2 v = in[i];
        out[i] = cmag(v.x, v.y);
    }
}

hipError_t launch_magnitude(const float2* in, float* out, long long count, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    long long blocks = (count + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_magnitude, dim3((unsigned)blocks), dim3(256), 0, s, in, out, count);
    return hipGetLastError();
}

// Half-spectrum packing for the config-5 gather (SURVEY 8e row note 1): the
// magnitude rows of real frames are mirror-symmetric, |X[n-k]| = |X[k]|, so
// bins 0..n/2 carry the whole row.  Pack: [rows][n] -> [rows][n/2+1]; unpack:
// out[k] = in[k <= n/2 ? k : n-k].  One workgroup per row (grid-stride over rows).
__global__ void __launch_bounds__(256) k_rows_half_pack(const float* in, float* out, long long rows, long long n) {
    const long long h = n / 2 + 1;
    for (long long r = blockIdx.x; r < rows; r += gridDim.x) {
        const float* src = in + r * n;
        float* dst = out + r * h;
        for (long long k = threadIdx.x; k < h; k += 256) dst[k] = src[k];
    }
}

__global__ void __launch_bounds__(256) k_rows_half_unpack(const float* in, float* out, long long rows, long long n) {
    const long long h = n / 2 + 1;
    for (long long r = blockIdx.x; r < rows; r += gridDim.x) {
        const float* src = in + r * h;
        float* dst = out + r * n;
        for (long long k = threadIdx.x; k < n; k += 256) dst[k] = src[k < h ? k : n - k];
    }
}

hipError_t launch_rows_half(const float* in, float* out, long long rows, long long n, int unpack, hipStream_t s) {
    if (rows <= 0 || n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)(rows < 262144 ? rows : 262144);
    if (unpack) hipLaunchKernelGGL(k_rows_half_unpack, dim3(grid), dim3(256), 0, s, in, out, rows, n);
    else hipLaunchKernelGGL(k_rows_half_pack, dim3(grid), dim3(256), 0, s, in, out, rows, n);
    return hipGetLastError();
}

// |X[k]|^2 for k <= nfft/2 of rows [rows][nfft] -> [rows][nfft/2+1]
__global__ void k_power_half(const float2* in, float* out, long long nfft, long long count) {
    const long long nh = nfft / 2 + 1;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < count;
         i += (long long)gridDim.x * blockDim.x) {
        const long long r = i / nh, k = i - r * nh;
        const float2 v = in[r * nfft + k];
        out[i] = __builtin_fmaf(v.x, v.x, v.y * v.y);
    }
}

hipError_t launch_power_half(const float2* in, float* out, long long nfft, long long rows, hipStream_t s) {
    const long long count = rows * (nfft / 2 + 1);
    if (count <= 0) return hipSuccess;
    long long blocks = (count + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_power_half, dim3((unsigned)blocks), dim3(256), 0, s, in, out, nfft, count);
    return hipGetLastError();
}

// ISTFT accumulate for `count` frames placed at multiples of hop (stft.c:95-110
// applied frame after frame).  One thread per output sample sums its frames in
// frame order, so the f32 rounding matches sequential accumulation.
__global__ void k_ola(long long nfft, long long hop, const float2* tf, long long count,
                      const float* win, float* out_add, float* norm_add, long long len) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < len;
         i += (long long)gridDim.x * blockDim.x) {
        long long f_hi = i / hop;
        if (f_hi > count - 1) f_hi = count - 1;
        long long f_lo = (i - nfft + 1 + hop - 1) / hop;
        if (i - nfft + 1 <= 0) f_lo = 0;
        float acc = out_add[i];
        float nacc = norm_add ? norm_add[i] : 0.0f;
        for (long long f = f_lo; f <= f_hi; ++f) {
            const long long e = i - f * hop;
            if (e < 0 || e >= nfft) continue;
            const float w = win[e];
            float c = tf[f * nfft + e].x * w, w2 = w * w;
            asm volatile("" : "+v"(c), "+v"(w2));   // products rounded before the adds (no FMA), as stft.c
            acc += c;
            nacc += w2;
        }
        out_add[i] = acc;
        if (norm_add) norm_add[i] = nacc;
    }
}

// ------------------------------------------------------------------------
// k_istft<N>: inverse FFT + window + overlap-add of `count` frames in one pass
// (stft.c:95-110 applied frame after frame), N = 1024, hop | N, K = N/hop <= 4.
// Only Re(IFFT(X)) is used, and Re(IFFT(X)) = IFFT of the Hermitian part
// (X[k] + conj X[N-k])/2, so two frames share one complex inverse FFT:
// Z = Ha + i Hb gives frame a's samples in Re z and frame b's in Im z.
// A workgroup (4 waves = 8 frames per step) owns the frames [fa, fb) and the
// output hop-blocks [fa, fb) (the last one also the K-1 tail blocks), computes
// K-1 frames before fa as halo, and finalises each block once all of its
// frames are in: out_add[i] + c_{b-K+1} + ... + c_b in frame order, products
// re*w and w*w rounded before they are added -- the f32 rounding of the
// sequential loop.  Blocks still open after a step (the K-1 newest) are
// carried in LDS.  The windowed real parts of a step's 8 frames sit in LDS; a
// wave's FFT exchange reuses its own 2 frames' area.
// Traffic: the spectrum read once (8 B per bin), out_add (and norm_add) read
// and written once -- against ~3x that for IFFT-to-scratch + a separate OLA.
// (Measured variants: one frame per wave with the next frame's spectrum
// prefetched in registers, and a compile-time hop with batched accumulator
// loads, both ran slower -- 0.59-0.65 vs 0.44 ms for 600 s at hop 256.)
// ------------------------------------------------------------------------
template <int N>
__global__ void __launch_bounds__(256, 3)
k_istft(const float2* __restrict__ spec, long long count, int hop, int K, const float* __restrict__ win,
        float* __restrict__ out_add, float* __restrict__ norm_add, long long run, const float2* gpass) {
    using G = Geo<N>;
    static_assert(G::T == 64 && ri_floats<N>() <= 2 * N, "one wave per transform; exchange fits two frames");
    constexpr int TWL = G::tw_off(G::NPASS - 1) > 0 ? G::tw_off(G::NPASS - 1) : 1;
    __shared__ __attribute__((aligned(16))) float stage[8 * N];
    __shared__ float carry[N], ncarry[N];
    __shared__ float lwin[N];
    __shared__ float2 ltab[TWL];
    const int tid = threadIdx.x, wv = tid >> 6, t = tid & 63;
    for (int i = tid; i < G::tw_off(G::NPASS - 1); i += 256) ltab[i] = gpass[i];
    for (int i = tid; i < N; i += 256) lwin[i] = win[i];
    TwLastReg<N> tw;
    tw.tab = ltab;
    tw.load(gpass, t);
    __syncthreads();
    const long long fa = (long long)blockIdx.x * run;
    const long long fb = fa + run < count ? fa + run : count;
    const long long bend = fb == count ? count + K - 1 : fb;   // blocks this workgroup writes: [fa, bend)
    const long long g0 = fa - (K - 1);
    const float sc = 0.5f / (float)N;   // Hermitian half and the backward 1/N, exact (powers of two)
    const int lh = 31 - __builtin_clz((unsigned)hop);   // hop is a power of two (istft_fused_supported)
    float* my = stage + 2 * wv * N;
    for (long long g = g0; g < fb; g += 8) {
        // ---- two frames per wave: Z = Ha + i Hb, inverse FFT, window -> stage
        const long long f0 = uni<64>(g + 2 * wv);   // wave-uniform: SGPR row bases, 32-bit lane offsets
        const bool va = f0 >= 0 && f0 < fb, vb = f0 + 1 >= 0 && f0 + 1 < fb;
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = make_float2(0.0f, 0.0f);
        if (va) {
            const float2* xa = spec + f0 * N;
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                const int k = t + 64 * r;
                const float2 A = xa[k], Am = xa[(N - k) & (N - 1)];
                v[r] = make_float2((A.x + Am.x) * sc, (A.y - Am.y) * sc);   // Ha
            }
        }
        if (vb) {
            const float2* xb = spec + (f0 + 1) * N;
#pragma unroll
            for (int r = 0; r < G::P; ++r) {
                const int k = t + 64 * r;
                const float2 B = xb[k], Bm = xb[(N - k) & (N - 1)];
                const float2 hb = make_float2((B.x + Bm.x) * sc, (B.y - Bm.y) * sc);
                v[r] = make_float2(v[r].x - hb.y, v[r].y + hb.x);   // + i Hb
            }
        }
        tw.opaque();
        fft_regs<N, false, false, true>(v, t, reinterpret_cast<float2*>(my), tw);
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const int e = out_pos<N>(t, q);
            const float w = lwin[e];
            float ca = v[q].x * w, cb = v[q].y * w;
            asm volatile("" : "+v"(ca), "+v"(cb));   // re*w rounded before it is added
            my[e] = ca;
            my[N + e] = cb;
        }
        __syncthreads();
        // ---- combine: sum of block b's contributions of this step's frames, in frame order
        // ---- combine: sum of block b's contributions of this step's frames, in
        // frame order.  All per-sample index math is 32-bit and relative to the
        // step (block bb = b - g, frame r = f - g; hop is a power of two), with
        // the 64-bit bounds folded into uniform per-step limits.
        auto clampi = [](long long v) { return (int)(v < -(1LL << 30) ? -(1LL << 30) : (v > (1LL << 30) ? (1LL << 30) : v)); };
        const long long gh = g * hop;                           // sample index of block g
        const int rflo = g < 0 ? (int)(-g) : 0;                  // frames f >= 0
        const int rfhi = (int)(fb - 1 - g < 7 ? fb - 1 - g : 7);   // frames f < fb of this step
        const int bb_fa = clampi(fa - g), bb_bend = clampi(bend - g), bb_tot = clampi(count + K - 1 - g);
        auto combine = [&](int bb, int j, float acc, float nacc, float* acc_o, float* nacc_o) {
            int rlo = bb - K + 1;
            if (rlo < rflo) rlo = rflo;
            const int rhi = bb < rfhi ? bb : rfhi;
            for (int r = rlo; r <= rhi; ++r) {
                const int e = ((bb - r) << lh) + j;
                acc += stage[r * N + e];
                const float w = lwin[e];
                float w2 = w * w;
                asm volatile("" : "+v"(w2));   // no FMA: w*w rounded, then added (stft.c)
                nacc += w2;
            }
            *acc_o = acc;
            *nacc_o = nacc;
        };
        // Both phases read their out_add / norm_add words for eight samples per
        // thread before combining any (one memory latency per chunk instead of
        // one per sample: the loop body's load -> add -> store chain otherwise
        // serialises them).
        constexpr int CH = 8;
        for (int base = 0; base < 8 * hop; base += 256 * CH) {   // phase A: blocks [g, g+8) become final
            float a0[CH], n0[CH];
#pragma unroll
            for (int s = 0; s < CH; ++s) {
                const int idx = base + tid + 256 * s, bb = idx >> lh;
                const bool ok = idx < 8 * hop && bb >= bb_fa && bb < bb_bend && bb < bb_tot;
                const bool fresh = g == g0 || bb >= K - 1;
                a0[s] = ok ? (fresh ? out_add[gh + idx] : carry[idx]) : 0.0f;
                n0[s] = ok && norm_add ? (fresh ? norm_add[gh + idx] : ncarry[idx]) : 0.0f;
            }
#pragma unroll
            for (int s = 0; s < CH; ++s) {
                const int idx = base + tid + 256 * s, bb = idx >> lh, j = idx & (hop - 1);   // idx = bb * hop + j
                if (idx >= 8 * hop || bb < bb_fa || bb >= bb_bend || bb >= bb_tot) continue;
                float acc, nacc;
                combine(bb, j, a0[s], n0[s], &acc, &nacc);
                out_add[gh + idx] = acc;
                if (norm_add) norm_add[gh + idx] = nacc;
            }
        }
        __syncthreads();   // phase A's carry reads before phase B's carry writes
        const bool last = g + 8 >= fb;
        const long long gh8 = gh + 8LL * hop;
        for (int base = 0; base < (K - 1) * hop; base += 256 * CH) {   // phase B: blocks [g+8, g+8+K-1), fresh
            float a0[CH], n0[CH];
#pragma unroll
            for (int s = 0; s < CH; ++s) {
                const int idx = base + tid + 256 * s, bb = 8 + (idx >> lh);
                const bool ok = idx < (K - 1) * hop && bb < bb_tot;
                a0[s] = ok ? out_add[gh8 + idx] : 0.0f;
                n0[s] = ok && norm_add ? norm_add[gh8 + idx] : 0.0f;
            }
#pragma unroll
            for (int s = 0; s < CH; ++s) {
                const int idx = base + tid + 256 * s, bb = 8 + (idx >> lh), j = idx & (hop - 1);
                if (idx >= (K - 1) * hop || bb >= bb_tot) continue;
                float acc, nacc;
                combine(bb, j, a0[s], n0[s], &acc, &nacc);
                if (last) {
                    if (bb >= bb_fa && bb < bb_bend) {
                        out_add[gh8 + idx] = acc;
                        if (norm_add) norm_add[gh8 + idx] = nacc;
                    }
                } else {
                    carry[idx] = acc;   // = (b - (g+8)) * hop + j: next step's base
                    ncarry[idx] = nacc;
                }
            }
        }
        __syncthreads();   // stage and carry are reused by the next step
    }
}

bool istft_fused_supported(long long nfft, long long hop) {
    return nfft == 1024 && hop >= 256 && nfft % hop == 0 && (hop & (hop - 1)) == 0;   // K = nfft/hop <= 4
}

hipError_t launch_istft_fused(long long nfft, long long hop, const float2* spec, long long count,
                              const float* win, float* out_add, float* norm_add, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    if (!istft_fused_supported(nfft, hop)) return hipErrorInvalidValue;
    constexpr int N = 1024;
    const float2* pN = pass_twiddles(N);
    if (!pN) return hipErrorOutOfMemory;
    const int K = (int)(N / hop);
    // owned frames per workgroup: run + K - 1 computed frames = whole steps of 8
    long long run = 64 - (K - 1);
    if (count < 8 * run) run = 8 - (K - 1);   // small jobs: more workgroups
    const long long grid = (count + run - 1) / run;
hipLaunchKernelGGL((k_istft<N>), dim3((unsigned)grid), dim3(256), 0, s, spec, count, (int)hop, K, win, out_add,
                       norm_add, run, pN);
    return hipGetLastError();
}

hipError_t launch_ola(long long nfft, long long hop, const float2* time_frames, long long count,
                      const float* win, float* out_add, float* norm_add, hipStream_t s) {
    const long long len = (count - 1) * hop + nfft;
    if (count <= 0) return hipSuccess;
    long long blocks = (len + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_ola, dim3((unsigned)blocks), dim3(256), 0, s, nfft, hop, time_frames, count, win,
                       out_add, norm_add, len);
    return hipGetLastError();
}

}  // namespace vvh
