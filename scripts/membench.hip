// membench.hip -- store-pattern microbenchmark (tooling, not product).
// Writes `rows` rows of 1024 floats with one of several per-lane patterns so
// the cost of the STFT's mirrored dword stores can be compared with plain
// dword / dwordx2 / dwordx4 streaming stores.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC scripts/membench.hip -o scripts/libmembench.so
#include <hip/hip_runtime.h>

typedef float vf4 __attribute__((ext_vector_type(4)));
typedef float vf2 __attribute__((ext_vector_type(2)));

template <int MODE, bool NT>
__global__ void __launch_bounds__(256) k_wr(float* out, long long rows) {
    const int t = threadIdx.x & 63;
    const long long wave = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const long long nw = (long long)gridDim.x * 4;
    const float val = (float)t;
    for (long long row = wave; row < rows; row += nw) {
        float* o = out + row * 1024;
        if constexpr (MODE == 0) {   // dword, lane-contiguous
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if (NT) __builtin_nontemporal_store(val, o + t + 64 * j);
                else o[t + 64 * j] = val;
            }
        } else if constexpr (MODE == 1) {   // STFT paired-last-pass pattern (k and N-k)
            const int kb0 = t, kb1 = t == 0 ? 128 : 256 - t, kb2 = t + 64, kb3 = 192 - t;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ks[4] = {kb0 + 256 * r, kb1 + 256 * (3 - r), kb2 + 256 * r, kb3 + 256 * (3 - r)};
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    if (NT) __builtin_nontemporal_store(val, o + ks[s]);
                    else o[ks[s]] = val;
                }
            }
        } else if constexpr (MODE == 2) {   // dwordx2
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                vf2 v = {val, val};
                vf2* p = reinterpret_cast<vf2*>(o) + t + 64 * j;
                if (NT) __builtin_nontemporal_store(v, p);
                else *p = v;
            }
        } else {   // dwordx4
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                vf4 v = {val, val, val, val};
                vf4* p = reinterpret_cast<vf4*>(o) + t + 64 * j;
                if (NT) __builtin_nontemporal_store(v, p);
                else *p = v;
            }
        }
    }
}

extern "C" int membench_write(float* out, long long rows, int mode, int nt, int blocks, void* stream) {
    hipStream_t s = (hipStream_t)stream;
#define L(M, N) hipLaunchKernelGGL((k_wr<M, N>), dim3(blocks), dim3(256), 0, s, out, rows)
    switch (mode * 2 + (nt ? 1 : 0)) {
        case 0: L(0, false); break; case 1: L(0, true); break;
        case 2: L(1, false); break; case 3: L(1, true); break;
        case 4: L(2, false); break; case 5: L(2, true); break;
        case 6: L(3, false); break; case 7: L(3, true); break;
        default: return -1;
    }
#undef L
    return (int)hipGetLastError();
}

// ---- STFT bottleneck experiments: the product kernel's structure (nfft 1024,
// magnitudes) with parts switched off.  E bit0: no FFT, bit1: no stores
// (guarded by an impossible value), bit2: no loads (synthetic samples).
#include "../vv-dsp_amd/csrc/hip/fft_core.hpp"
using vvh::vf2_t;
using vvh::vf4_t;
#include <cmath>
#include <vector>

namespace vvh {
template <int E>
__global__ void __launch_bounds__(256) k_stft_exp(const float* sig, long long n, long long nch, long long ch_stride,
                                                  long long hop, long long ppc, const float* win, float* out,
                                                  long long out_ch_stride, const float2* gpass) {
    constexpr int N = 1024;
    using G = Geo<N>;
    using Mi = Mirror<N>;
    constexpr int F = Wg<N>::F, R = G::RL;
    __shared__ float2 lds[F * G::LDS];
    __shared__ float2 ltab[TwLayout<N>::ENTRIES];
    stage_twiddles<N, 256>(ltab, gpass, gpass);
    __syncthreads();
    const TwTab<N> tw{ltab};
    const int lt = threadIdx.x, slot = lt / G::T, t = lt % G::T;
    float2* my = lds + slot * G::LDS;
    float w[G::P];
#pragma unroll
    for (int r = 0; r < G::P; ++r) w[r] = 0.5f * win[t + r * G::T];
    const long long pairs = nch * ppc, S = (long long)gridDim.x * F, g = (long long)blockIdx.x * F + slot;
    const long long per = pairs / S, rem = pairs % S;
    long long p = g * per + (g < rem ? g : rem);
    long long p_end = p + per + (g < rem ? 1 : 0);
    p = uni<64>(p);
    p_end = uni<64>(p_end);
    if (p >= p_end) return;
    long long c = p / ppc, fa = 2 * (p - c * ppc);
    float xa[G::P], xb[G::P];
    auto load_pair = [&](long long cc, long long ff) {
        const float* sa = sig + cc * ch_stride + ff * hop;
        const float* sb = sa + hop;
#pragma unroll
        for (int r = 0; r < G::P; ++r) {
            if (E & 4) {
                xa[r] = (float)(ff + r) * 1e-3f + t;
                xb[r] = (float)(cc - r) * 1e-3f - t;
            } else {
                xa[r] = sa[t + r * G::T];
                xb[r] = sb[t + r * G::T];
            }
        }
    };
    load_pair(c, fa);
    int kb[G::NPT];
#pragma unroll
    for (int i = 0; i < G::NPT; ++i) kb[i] = bfly<N, G::NPASS - 1, true>(t, i);
    for (; p < p_end; ++p) {
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = make_float2(xa[r] * w[r], xb[r] * w[r]);
        long long cn = c, fn = fa + 2;
        if (fn >= 2 * ppc) {
            fn = 0;
            ++cn;
        }
        const bool more = p + 1 < p_end;
        load_pair(more ? cn : c, more ? fn : fa);
        if (!(E & 1)) fft_regs<N, true, true>(v, t, my, tw);
        float* rowa = out + c * out_ch_stride + fa * (long long)N;
        float* rowb = rowa + N;
#pragma unroll
        for (int i = 0; i < G::NPT; i += 2) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int q = i * R + r, qm = Mi::normal(q);
                const float2 Z = v[q], Zm = mirror_of<N, true>(v, t, q);
                const float ma = __builtin_amdgcn_sqrtf((Z.x + Zm.x) * (Z.x + Zm.x) + (Z.y - Zm.y) * (Z.y - Zm.y));
                const float mb = __builtin_amdgcn_sqrtf((Z.y + Zm.y) * (Z.y + Zm.y) + (Z.x - Zm.x) * (Z.x - Zm.x));
                const int k = kb[i] + r * G::NB, km = kb[i + 1] + (R - 1 - r) * G::NB;
                if (!(E & 2) || ma == 12345.678f) {
                    rowa[k] = ma;
                    rowa[km] = ma;
                    rowb[k] = mb;
                    rowb[km] = mb;
                }
                (void)qm;
            }
        }
        c = cn;
        fa = fn;
    }
}
}  // namespace vvh

extern "C" int membench_stft_exp(const float* sig, long long n, long long nch, long long hop, const float* win,
                                 float* out, int e, void* stream) {
    static float2* gpass = nullptr;
    using G = vvh::Geo<1024>;
    if (!gpass) {
        std::vector<float2> h(G::TW_PASS_ENTRIES);
        for (int p = 1; p < G::NPASS; ++p)
            for (int r = 1; r < G::radix(p); ++r)
                for (int j = 0; j < G::ns(p); ++j) {
                    const double a = -2.0 * M_PI * j * r / (G::ns(p) * G::radix(p));
                    h[G::tw_off(p) + (r - 1) * G::ns(p) + j] = make_float2((float)cos(a), (float)sin(a));
                }
        if (hipMalloc(&gpass, h.size() * sizeof(float2)) != hipSuccess) return -2;
        if (hipMemcpy(gpass, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess) return -3;
    }
    const long long frames = (n - 1024) / hop + 1;
    const long long ppc = frames / 2;
    hipStream_t s = (hipStream_t)stream;
    const int grid = 512;
#define L(EE)                                                                                                \
    hipLaunchKernelGGL((vvh::k_stft_exp<EE>), dim3(grid), dim3(256), 0, s, sig, n, nch, n, hop, ppc, win, out, \
                       frames * 1024, gpass)
    switch (e) {
        case 0: L(0); break; case 1: L(1); break; case 2: L(2); break; case 3: L(3); break;
        case 4: L(4); break; case 5: L(5); break; case 6: L(6); break; case 7: L(7); break;
        default: return -1;
    }
#undef L
    return (int)hipGetLastError();
}

// ---- mixed read/write streaming: each lane reads 1 float4 and writes W float4
// (W = 4: the STFT's 1:4 read:write byte mix; W = 1: copy).
template <int W>
__global__ void __launch_bounds__(256) k_rw(const vf4* __restrict__ in, vf4* __restrict__ out, long long n4) {
    const long long stride = (long long)gridDim.x * 256;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
        const vf4 v = __builtin_nontemporal_load(in + i);
#pragma unroll
        for (int w = 0; w < W; ++w) __builtin_nontemporal_store(v, out + (long long)w * n4 + i);   // W planes
    }
}

extern "C" int membench_rw(const float* in, float* out, long long n4, int w, int blocks, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (w == 1) hipLaunchKernelGGL((k_rw<1>), dim3(blocks), dim3(256), 0, s, (const vf4*)in, (vf4*)out, n4);
    else if (w == 4) hipLaunchKernelGGL((k_rw<4>), dim3(blocks), dim3(256), 0, s, (const vf4*)in, (vf4*)out, n4);
    else return -1;
    return (int)hipGetLastError();
}

// Contiguous mixed stream: wave item i reads 1 KB at in + i KB and writes W KB
// contiguous at out + i*W KB (the STFT's per-frame shape: hop 256 samples in,
// one 4 KB row out).  U items are loaded before any is stored (loads in flight).
template <int W, int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_rwc(const vf4* __restrict__ in, vf4* __restrict__ out, long long items) {
    const int lane = threadIdx.x & 63;
    const long long wave = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const long long nw = (long long)gridDim.x * 4;
    for (long long i0 = wave * U; i0 < items; i0 += nw * U) {
        vf4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long i = i0 + u < items ? i0 + u : items - 1;
            v[u] = NTL ? __builtin_nontemporal_load(in + i * 64 + lane) : in[i * 64 + lane];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i0 + u >= items) break;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                vf4* p = out + (i0 + u) * 64 * W + w * 64 + lane;
                if (NTS) __builtin_nontemporal_store(v[u], p);
                else *p = v[u];
            }
        }
    }
}

extern "C" int membench_rwc(const float* in, float* out, long long items, int w, int u, int ntl, int nts, int blocks,
                            void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const vf4* a = (const vf4*)in;
    vf4* b = (vf4*)out;
#define RWC(WW, UU, L, S)                                                                                  \
    if (w == WW && u == UU && ntl == L && nts == S) {                                                      \
        hipLaunchKernelGGL((k_rwc<WW, UU, L, S>), dim3(blocks), dim3(256), 0, s, a, b, items);             \
        return (int)hipGetLastError();                                                                     \
    }
    RWC(4, 1, 1, 1) RWC(4, 2, 1, 1) RWC(4, 4, 1, 1) RWC(4, 1, 0, 0) RWC(4, 2, 0, 0) RWC(4, 4, 0, 0)
    RWC(4, 2, 0, 1) RWC(4, 2, 1, 0) RWC(1, 2, 1, 1) RWC(1, 2, 0, 0) RWC(4, 8, 1, 1)
    RWC(1, 1, 1, 1) RWC(1, 4, 1, 1)
#undef RWC
    return -1;
}

// ---- model of the STFT bulk kernel's memory pipeline ------------------------
// Persistent 256-thread blocks (4 independent waves), xcd_walk over frame
// pairs, per pair: wait for the pair's 1280-float input span (LDS-DMA issued
// DEPTH pairs ahead), read 32 floats of it from LDS, WORK x 16 dependent-free
// v_pk_fma_f32 (stand-in for the FFT), 8 x 16 B/lane nt stores (two 4 KB rows).
// Dynamic LDS pads the block to `lds_bytes` to set the occupancy.
#include "../vv-dsp_amd/csrc/hip/fft_core.hpp"
using vvh::vf2_t;
using vvh::vf4_t;

template <int DEPTH, int WORK, int WALK, int LD = 0>
__global__ void __launch_bounds__(256) k_model(const float* __restrict__ sig, float* __restrict__ out, long long pairs,
                                               long long hop) {
    extern __shared__ __attribute__((aligned(16))) float dyn[];
    // LD 0: the whole 1280-float span by LDS-DMA (5 ops); 1: only the 512 new floats by LDS-DMA (2 ops);
    // 2: the 512 new floats into registers (2 x global_load_dwordx4, DEPTH must be 1)
    constexpr int SPAN = 1280, NLD = LD == 0 ? 5 : 2, NST = 8;
    vf4_t rg[2];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float* ring = dyn + wv * DEPTH * SPAN;
    long long p, p_end, p_step;
    if constexpr (WALK == 0) {   // 8 contiguous shares, one per XCD
        vvh::xcd_walk(pairs, 4, wv, &p, &p_end, &p_step);
    } else if constexpr (WALK == 1) {   // one front, consecutive waves -> consecutive pairs
        p = (long long)blockIdx.x * 4 + wv;
        p_step = (long long)gridDim.x * 4;
        p_end = pairs;
    } else if constexpr (WALK == 2) {   // one front; each XCD (blockIdx % 8) takes a contiguous block of it
        const long long ng = 8, nbg = ((long long)gridDim.x + 7) / 8;   // gridDim.x % 8 == 0 assumed
        const long long wx = nbg * 4;                                     // wave slots per XCD
        p = ((long long)blockIdx.x % ng) * wx + ((long long)blockIdx.x / ng) * 4 + wv;
        p_step = ng * wx;
        p_end = pairs;
    } else {   // not persistent: block b owns pairs [b*4*PPW, (b+1)*4*PPW), its waves interleaved
        constexpr long long PPW = WALK == 3 ? 16 : 4;
        p = (long long)blockIdx.x * 4 * PPW + wv;
        p_step = 4;
        p_end = (long long)(blockIdx.x + 1) * 4 * PPW;
        if (p_end > pairs) p_end = pairs;
    }
    p = vvh::uni<64>(p);
    p_end = vvh::uni<64>(p_end);
    p_step = vvh::uni<64>(p_step);
    if (p >= p_end) return;
    auto issue = [&](long long q, int slot) {
        const float* s0 = sig + q * 2 * hop;
        if constexpr (LD == 2) {
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(rg[0]) : "v"(s0 + lane * 4) : "memory");
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(rg[1]) : "v"(s0 + 256 + lane * 4) : "memory");
        } else {
            for (int u = 0; u < NLD; ++u) vvh::glds16(s0 + u * 256 + lane * 4, ring + slot * SPAN + u * 256);
        }
    };
    // prologue: DEPTH spans in flight (past the end: re-issue the last pair, counted the same)
    for (int d = 0; d < DEPTH; ++d) {
        const long long q = p + d * p_step;
        issue(q < p_end ? q : p, d);
    }
    vf2_t acc[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = vf2_t{(float)lane, 1.0f};
    const vf2_t a = {0.999f, 0.999f}, b = {0.001f, 0.001f};
    int slot = 0;
    long long it = 0;
    for (; p < p_end; p += p_step, ++it) {
        // outstanding younger than this pair's span: (DEPTH-1) later spans + the stores between
        if (it == 0) vvh::vm_wait<(DEPTH - 1) * NLD>();
        else vvh::vm_wait<(DEPTH - 1) * (NLD + NST) + NST>();
        const float* sp = ring + slot * SPAN;
        if constexpr (LD == 2) {
            acc[0] += vf2_t{rg[0].x, rg[0].y};
            acc[1] += vf2_t{rg[0].z, rg[0].w};
            acc[2] += vf2_t{rg[1].x, rg[1].y};
            acc[3] += vf2_t{rg[1].z, rg[1].w};
        } else {
#pragma unroll
            for (int r = 0; r < 8; ++r) acc[r] += vf2_t{sp[lane + 64 * r], sp[256 + lane + 64 * r]};
        }
        vvh::lgkm_wait0();
        {
            const long long q = p + DEPTH * p_step;
            issue(q < p_end ? q : p, slot);   // always NLD ops, so the counts stay exact
        }
        slot = slot + 1 == DEPTH ? 0 : slot + 1;
#pragma unroll 1
        for (int k = 0; k < WORK; ++k) {
#pragma unroll
            for (int r = 0; r < 8; ++r) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(acc[r]) : "v"(a), "v"(b));
#pragma unroll
            for (int r = 0; r < 8; ++r) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(acc[r]) : "v"(b), "v"(a));
        }
        float* o = out + p * 2048;
#pragma unroll
        for (int j = 0; j < NST; ++j) {
            const vf4_t v = {acc[j].x, acc[j].y, acc[(j + 1) & 7].x, acc[(j + 1) & 7].y};
            vvh::st16_nt_counted(reinterpret_cast<vf4_t*>(o) + j * 64 + lane, v);
        }
    }
    vvh::vm_wait<0>();
}

extern "C" int membench_model(const float* sig, float* out, long long pairs, long long hop, int depth, int work,
                              int lds_bytes, int walk, int ld, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
#define MODEL(D, W)                                                                                               \
    if (depth == D && work == W) {                                                                                \
        const void* k = walk == 0 ? (const void*)k_model<D, W, 0>                                                 \
                        : walk == 1 ? (const void*)k_model<D, W, 1>                                               \
                        : walk == 2 ? (const void*)k_model<D, W, 2>                                               \
                        : walk == 3 ? (const void*)k_model<D, W, 3> : (const void*)k_model<D, W, 4>;              \
        size_t need = (size_t)4 * D * 1280 * 4;                                                                   \
        size_t lds = (size_t)lds_bytes > need ? (size_t)lds_bytes : need;                                         \
        int per_cu = 0;                                                                                           \
        (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                       \
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, lds);                                 \
        if (per_cu < 1) per_cu = 1;                                                                               \
        if (walk == 0) hipLaunchKernelGGL((k_model<D, W, 0>), dim3(cus * per_cu), dim3(256), lds, s, sig, out, pairs, hop); \
        else if (walk == 1) hipLaunchKernelGGL((k_model<D, W, 1>), dim3(cus * per_cu), dim3(256), lds, s, sig, out, pairs, hop); \
        else if (walk == 2) hipLaunchKernelGGL((k_model<D, W, 2>), dim3(cus * per_cu), dim3(256), lds, s, sig, out, pairs, hop); \
        else if (walk == 3) hipLaunchKernelGGL((k_model<D, W, 3>), dim3((pairs + 63) / 64), dim3(256), lds, s, sig, out, pairs, hop); \
        else hipLaunchKernelGGL((k_model<D, W, 4>), dim3((pairs + 15) / 16), dim3(256), lds, s, sig, out, pairs, hop); \
        return (int)hipGetLastError();                                                                            \
    }
    if (ld == 0) { MODEL(1, 0) MODEL(1, 12) MODEL(1, 25) MODEL(2, 0) MODEL(2, 12) MODEL(2, 25) MODEL(3, 25) }
#undef MODEL
#define MODEL_LD(L, W)                                                                                              \
    if (ld == L && depth == 1 && work == W) {                                                                       \
        const void* k = (const void*)k_model<1, W, 1, L>;                                                           \
        int per_cu = 0;                                                                                             \
        size_t lds = (size_t)lds_bytes > 20480 ? (size_t)lds_bytes : 20480;                                         \
        (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                         \
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, lds);                                   \
        if (per_cu < 1) per_cu = 1;                                                                                 \
        hipLaunchKernelGGL((k_model<1, W, 1, L>), dim3(cus * per_cu), dim3(256), lds, s, sig, out, pairs, hop);     \
        return (int)hipGetLastError();                                                                              \
    }
    MODEL_LD(1, 0) MODEL_LD(1, 12) MODEL_LD(2, 0) MODEL_LD(2, 12)
#undef MODEL_LD
#define MODEL_LD4(L, W)                                                                                             \
    if (ld == L + 10 && depth == 1 && work == W) {                                                                  \
        size_t lds = (size_t)lds_bytes > 20480 ? (size_t)lds_bytes : 20480;                                         \
        (void)hipFuncSetAttribute((const void*)k_model<1, W, 4, L>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
        hipLaunchKernelGGL((k_model<1, W, 4, L>), dim3((pairs + 15) / 16), dim3(256), lds, s, sig, out, pairs, hop); \
        return (int)hipGetLastError();                                                                              \
    }
    MODEL_LD4(0, 12) MODEL_LD4(1, 12) MODEL_LD4(2, 12) MODEL_LD4(0, 0) MODEL_LD4(2, 0)
#undef MODEL_LD4
    return -1;
}

// ---- write-ceiling probe (round 4): pure streams of 4 KB items (the headline's
// 14.7 GB of magnitude rows), or the 1:4 read:write mix, in the shapes the STFT
// kernel could use.  W: 1 dword / 4 dwordx4 per lane; POL: 0 plain, 1 nt,
// 2 sc1, 3 sc0 sc1 nt; BAND: 0 one grid-wide interleaved front, 1 one
// contiguous eighth of the buffer per XCD group (block % 8), 2 per-XCD-group
// 2 MB chunks dealt round robin; RD: also read 1 KB per item (16 B/lane nt).
template <int POL>
__device__ __forceinline__ void wst4(float* p, vf4 v) {
    if constexpr (POL == 0) *reinterpret_cast<vf4*>(p) = v;
    else if constexpr (POL == 1) __builtin_nontemporal_store(v, reinterpret_cast<vf4*>(p));
    else if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}
template <int POL>
__device__ __forceinline__ void wst1(float* p, float v) {
    if constexpr (POL == 0) *p = v;
    else if constexpr (POL == 1) __builtin_nontemporal_store(v, p);
    else if constexpr (POL == 2) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dword %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}
template <int W, int POL, int BAND, int RD>
__global__ void __launch_bounds__(256) k_wprobe(const float* in, float* out, long long items) {
    const int t = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr long long CH = 512;   // 2 MB of output = 512 items
    long long first, step;
    const long long nb = gridDim.x, b = blockIdx.x, g = b % 8, nbg = (nb - g + 7) / 8;
    long long lo = 0, hi = items;
    if constexpr (BAND == 0) {
        first = b * 4 + wv;
        step = nb * 4;
    } else {
        first = (b / 8) * 4 + wv;
        step = nbg * 4;
        if constexpr (BAND == 1) {
            lo = g * items / 8;
            hi = (g + 1) * items / 8;
        } else {
            hi = (items / CH + 7 - g) / 8 * CH;   // this group's chunks g, g+8, ... (whole chunks)
        }
    }
    float acc = (float)t;
    for (long long s = first; lo + s < hi; s += step) {
        long long it = lo + s;
        if constexpr (BAND == 2) it = ((s / CH) * 8 + g) * CH + s % CH;
        if (it >= items) break;
        if constexpr (RD) {
            const vf4 x = __builtin_nontemporal_load(reinterpret_cast<const vf4*>(in + it * 256) + t);
            acc += x.x + x.y + x.z + x.w;
        }
        float* o = out + it * 1024;
        if constexpr (W == 4) {
#pragma unroll
            for (int j = 0; j < 4; ++j) wst4<POL>(o + 4 * (t + 64 * j), vf4{acc, acc, acc, acc});
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) wst1<POL>(o + t + 64 * j, acc);
        }
    }
}

extern "C" int membench_wprobe(const float* in, float* out, long long items, int w, int pol, int band, int rd,
                               int blocks, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const int key = ((w == 4 ? 1 : 0) * 4 + pol) * 6 + band * 2 + (rd ? 1 : 0);
#define L(W, P, B, R)                                                                                  \
    case ((W == 4 ? 1 : 0) * 4 + P) * 6 + B * 2 + R:                                                    \
        hipLaunchKernelGGL((k_wprobe<W, P, B, R>), dim3(blocks), dim3(256), 0, s, in, out, items); break;
#define LB(W, P) L(W, P, 0, 0) L(W, P, 0, 1) L(W, P, 1, 0) L(W, P, 1, 1) L(W, P, 2, 0) L(W, P, 2, 1)
    switch (key) {
        LB(1, 0) LB(1, 1) LB(1, 2) LB(1, 3) LB(4, 0) LB(4, 1) LB(4, 2) LB(4, 3)
        default: return -1;
    }
#undef LB
#undef L
    return (int)hipGetLastError();
}
