// stftlab.hip -- lab-only kernels (not part of the product; built into
// scripts/libstftlab.so by `make -C vv-dsp_amd lab`): superseded designs kept
// for timing comparisons (k_fir_bulk, k_c2c_r32) with their own ablation bits,
// an empty-kernel launch floor and the fused mel kernel's occupancy query.
// Since round 5 the product kernels carry no ablation code: A/B and ablations
// of them are separate library builds timed on the same buffers in one process
// (scripts/ab2.py).
#include "../vv-dsp_amd/csrc/hip/debug.hip"
#include "../vv-dsp_amd/csrc/hip/tables.hip"
#include "../vv-dsp_amd/csrc/hip/stft_kernels.hip"
#include "../vv-dsp_amd/csrc/hip/fir_kernels.hip"
#include "../vv-dsp_amd/csrc/hip/fft_kernels.hip"

namespace vvh {
// ------------------------------------------------------------------------
// k_fir_bulk<N, LQ>: the bulk pairs at three workgroups per CU (12 waves)
// instead of two.  LDS per workgroup of four transforms: the FFT exchange
// through the half-size real/imaginary buffer (pass_exchange_ri, conflict-free
// for N = 1024), H for bins 0..N/2 only (h is real, so H[N-k] = conj H[k]),
// the last pass' twiddles in registers (a thread's last-pass butterflies are
// the same for every pair: j = t + T*i) and only the earlier passes' table in
// LDS -- 52 KB instead of 80 KB.
// LQ (le == N/4, e.g. taps <= N/4 + 1): the outputs below le are exactly the
// registers q with q % RL == 0, so those stores are dropped at compile time
// (no sink stores: 3/4 of the store instructions of the general variant).
// ------------------------------------------------------------------------
// Lab only since round 4 (the register-load k_fir_bulk_reg and then k_fir_r32
// replaced it).  EXP: bit 0 FFTs without their LDS exchanges, bit 1 no FFTs, bit 2 no
// output stores, bit 3 no span loads.  Results are wrong under any of them.
template <int N, bool LQ, int EXP = 0>
__global__ void __launch_bounds__(256, 3)   // 3 waves per SIMD: the LDS allows 3 workgroups per CU
k_fir_bulk(long long le, const float2* Hg, const float* x, float* y, long long nch, long long x_stride,
           long long y_stride, long long cnt, long long q0, const float2* gpass, float* sink) {
    using G = Geo<N>;
    static_assert(G::T == 64 && N == 1024 && !TwLayout<N>::SPLIT, "one wave per transform (T = N/16), pass-major twiddles");
    constexpr int F = 4, RL = G::RL;
    constexpr int SPAN = N + (3 * N) / 4;
    constexpr int NST = (EXP & 4) ? 0 : LQ ? 2 * (G::P - G::P / RL) : 2 * G::P;   // stores per pair
    constexpr int TWL = G::tw_off(G::NPASS - 1) > 0 ? G::tw_off(G::NPASS - 1) : 1;
    constexpr int XW = ri_floats<N>();   // exchange floats per transform (a multiple of 4)
    __shared__ __attribute__((aligned(16))) float xch[F * XW];   // 16 B: pass_exchange_ri's b128 writes
    __shared__ float2 ltab[TWL];
    __shared__ float2 lH[N / 2 + 1];
    __shared__ float span_all[F * SPAN];
    for (int i = threadIdx.x; i < G::tw_off(G::NPASS - 1); i += 256) ltab[i] = gpass[i];
    for (int i = threadIdx.x; i <= N / 2; i += 256) lH[i] = Hg[i];
    const int lt = threadIdx.x, slot = lt >> 6, t = lt & 63;
    TwLastReg<N> tw;
    tw.tab = ltab;
    tw.load(gpass, t);
    __syncthreads();
    float2* my = reinterpret_cast<float2*>(xch + slot * XW);
    float* span = span_all + slot * SPAN;
    const long long lout = N - le;
    long long p, p_end, p_step;
    xcd_walk(nch * cnt, F, slot, &p, &p_end, &p_step);
    p = uni<64>(p);
    p_end = uni<64>(p_end);
    p_step = uni<64>(p_step);
    if (p >= p_end) return;
    auto locate = [&](long long it, long long* cc, long long* jj) {
        *cc = it / cnt;
        *jj = 2 * (q0 + (it - *cc * cnt));
    };
    long long c, j;
    locate(p, &c, &j);
    float* snk = sink + ((((long long)blockIdx.x * F + slot) * 64) % SINK_FLOATS) + t;
    auto issue_span = [&](long long cc, long long jj) {
        if constexpr (EXP & 8) return;
        const float* s0 = x + cc * x_stride + jj * lout - le;
        const int len = (int)(N + lout);
#pragma unroll
        for (int u = 0; u < SPAN / 256; ++u) {
            const int e = u * 256 + t * 4;
            glds16(s0 + (e < len ? e : 0), span + u * 256);
        }
    };
    issue_span(c, j);
    vm_wait<0>();
    for (; p < p_end; p += p_step) {
        const bool more = p + p_step < p_end;
        long long cn = c, jn = j;
        if (more) locate(p + p_step, &cn, &jn);
        vm_wait<NST>();   // this pair's span; the previous pair's stores may still fly
        float2 v[G::P];
#pragma unroll
        for (int r = 0; r < G::P; ++r) v[r] = make_float2(span[t + r * 64], span[lout + t + r * 64]);
        lgkm_wait0();
        if (more) issue_span(cn, jn);
        tw.opaque();
        if constexpr (!(EXP & 2)) fft_regs<N, true, false, true, TwLastReg<N>, (EXP & 1) != 0>(v, t, my, tw);
        float2 u[G::P];
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const int m = q / RL + G::NPT * (q % RL);   // out_pos<N>(t, q) = t + 64*m
            if (m < G::P / 2) u[m] = cmul(v[q], lH[t + 64 * m]);
            else u[m] = cmul(v[q], cconj(lH[N - t - 64 * m]));
        }
        tw.opaque();
        if constexpr (!(EXP & 2)) fft_regs<N, false, false, true, TwLastReg<N>, (EXP & 1) != 0>(u, t, my, tw);
        float* ya = y + c * y_stride + j * lout - le;   // + e: block j output (e >= le)
        if constexpr (LQ) {
            // le = N/4, lout = 3N/4: register q (q % RL != 0) holds outputs
            // e = t + 64 m of both blocks, m = out_pos' slot; streaming dword
            // stores at the wave-uniform row base + 4t + immediate (block b's
            // from a second base 4 KB on, the immediate is 13-bit)
            const unsigned lo = 4u * (unsigned)t;
            const float* yb = ya + 1024;
            if constexpr (EXP & 4) {
#pragma unroll
                for (int q = 0; q < G::P; ++q) asm volatile("" ::"v"(u[q].x), "v"(u[q].y));
            }
            static_for<0, G::P>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                constexpr int m = q / RL + G::NPT * (q % RL);
                if constexpr ((EXP & 4) == 0 && q % RL != 0) {
                    st4_nt_sbase<256 * m>(lo, u[q].x, ya);
                    st4_nt_sbase<256 * m + 4 * (3 * N / 4) - 4096>(lo, u[q].y, yb);
                }
            });
        } else {
#pragma unroll
        for (int q = 0; q < G::P; ++q) {
            const long long e = out_pos<N>(t, q);
            {
                const bool ok = e >= le;
                st4_counted(ok ? ya + e : snk, u[q].x);
                st4_counted(ok ? ya + e + lout : snk, u[q].y);
            }
        }
        }
        c = cn;
        j = jn;
    }
}

// ------------------------------------------------------------------------
// k_c2c_r32: 1024-point C2C with the transform split 32 x 32 on half a wave
// (fft_core.hpp dft32 / r32_transpose): lane m2 loads x[32 m1 + m2] (m1 = 0..31,
// lane-contiguous 8 B loads), DFT_32 over m1 in registers, twiddle W_1024^(m2 k1),
// ONE LDS transpose, DFT_32 over m2 -> X[k1 + 32 k2] in register k2 of lane k1
// (lane-contiguous stores).  One exchange per transform instead of k_c2c's two
// (each 8 KB through the LDS write path).  Lab only: it measured slower
// than the product's k_c2c (same buffers, k_c2c 0.1878 / 0.1847 ms fwd / bwd
// against 0.1943 / 0.1953; k_c2c's FFT hides under its memory pattern,
// 0.1796 ms without it, and this kernel's own pattern at two waves per SIMD is
// slower, 0.1945 ms; profiles/r04_kbench_r32.jsonl).  Two transforms per wave, the next
// couple's 64 points prefetched into registers: two waves per SIMD, 2 x 72 KB
// of LDS per CU.  EXP: bit 1 no FFT.
// ------------------------------------------------------------------------
template <bool FWD, int EXP = 0>
__global__ void __launch_bounds__(256, 2)
k_c2c_r32(const float2* in, float2* out, long long batch, long long in_dist, long long out_dist,
          const float2* tw1024, float scale) {
    constexpr int F = 4;
    __shared__ __attribute__((aligned(16))) float2 xch[F * 2 * R32_BUF];
    __shared__ float2 ltw[32 * 32];   // [r][m] = W_1024^(m r)
    for (int i = threadIdx.x; i < 32 * 32; i += 256) ltw[i] = tw1024[((i & 31) * (i >> 5)) & 1023];
    const int lt = threadIdx.x, slot = lt >> 6, lane = lt & 63, half = lane >> 5, m = lane & 31;
    float2* buf = xch + (2 * slot + half) * R32_BUF;
    const float2* atw = ltw + m;
    __syncthreads();
    const long long couples = (batch + 1) / 2, stride = (long long)gridDim.x * F;
    long long cp = uni<64>((long long)blockIdx.x * F + slot);
    // transform of this half in couple k (a missing second transform recomputes the first, stores nothing)
    auto tf = [&](long long k) { return 2 * k + half < batch ? 2 * k + half : 2 * k; };
    float2 nx[32];
    if (cp < couples) {
        const float2* src = in + tf(cp) * in_dist + m;
#pragma unroll
        for (int r = 0; r < 32; ++r) nx[r] = ld_nt(src + 32 * r);
    }
    for (; cp < couples; cp += stride) {
        float2 v[32];
#pragma unroll
        for (int r = 0; r < 32; ++r) v[r] = nx[r];
        const long long f = tf(cp);
        const bool valid = 2 * cp + half < batch;
        const long long cn = cp + stride;
        if (cn < couples) {
            const float2* src = in + tf(cn) * in_dist + m;
#pragma unroll
            for (int r = 0; r < 32; ++r) nx[r] = ld_nt(src + 32 * r);
        }
        if constexpr (!(EXP & 2)) {
            dft32<FWD>(v);
            r32_twiddle<FWD>(v, atw);
            r32_transpose(v, buf, m);
            dft32<FWD>(v);
        }
        if (valid) {
            float2* dst = out + f * out_dist + m;
#pragma unroll
            for (int k2 = 0; k2 < 32; ++k2) st_nt(FWD ? v[k2] : cscale(v[k2], scale), dst + 32 * k2);
        }
    }
}

__global__ void __launch_bounds__(256) k_lab_empty(float* sink, int flag) {
    if (flag == 12345 && threadIdx.x == 0) sink[blockIdx.x] = 1.0f;
}
// config 4's bulk launch (8 ch x 2^24, 257 taps: N 1024, le 256) of k_fir_bulk<1024, true, EXP>
template <int EXP>
static hipError_t lab_fir(const float2* H, const float* x, float* y, long long n, long long nch, hipStream_t s) {
    constexpr int N = 1024;
    const long long le = 256, lout = N - le, nblk = (n + lout - 1) / lout, ppc = (nblk + 1) / 2;
    const long long qf = (le + 2 * lout - 1) / (2 * lout);
    long long ql = n / (2 * lout);
    if (ql > ppc) ql = ppc;
    static std::atomic<int> cap;
    const int capv = cached_grid(cap, (const void*)k_fir_bulk<N, true, EXP>, 256, 0, 1LL << 40);
    const long long cnt = ql - qf, need = (nch * cnt + 3) / 4;
    const int grid = (int)(need < capv ? need : capv);
    hipLaunchKernelGGL((k_fir_bulk<N, true, EXP>), dim3(grid), dim3(256), 0, s, le, H, x, y, nch, n, n, cnt, qf,
                       pass_twiddles(N), store_sink());
    return hipGetLastError();
}
template <int EXP>
static hipError_t lab_c2c_r32(const float2* in, float2* out, long long batch, hipStream_t s) {
    static std::atomic<int> cap;
    const int grid_cap = cached_grid(cap, (const void*)k_c2c_r32<true, EXP>, 256, 0, 1LL << 40);
    const long long need = ((batch + 1) / 2 + 3) / 4;
    const int grid = (int)(need < grid_cap ? need : grid_cap);
    hipLaunchKernelGGL((k_c2c_r32<true, EXP>), dim3(grid), dim3(256), 0, s, in, out, batch, 1024LL, 1024LL,
                       twiddle_table(1024), 1.0f);
    return hipGetLastError();
}
}  // namespace vvh

extern "C" int c2cr32lab_run(int exp, const void* in, void* out, long long batch, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (exp) {
        case 0: return (int)vvh::lab_c2c_r32<0>((const float2*)in, (float2*)out, batch, s);
        case 2: return (int)vvh::lab_c2c_r32<2>((const float2*)in, (float2*)out, batch, s);
        default: return -1;
    }
}

extern "C" int firlab_run(int exp, const void* H, const float* x, float* y, long long n, long long nch, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const float2* h = (const float2*)H;
    switch (exp) {
#define C(E) case E: return (int)vvh::lab_fir<E>(h, x, y, n, nch, s);
        C(0) C(1) C(2) C(3) C(4) C(5) C(6) C(8) C(10) C(12) C(14)
#undef C
        default: return -1;
    }
}

// workgroups per CU of the fused log-mel (mode 3) / MFCC (mode 4) kernel with `dyn` bytes of dynamic LDS
extern "C" int lab_mel_occupancy(int mode, long long dyn) {
    int per_cu = -1;
    const void* k = mode == 3 ? (const void*)vvh::k_stft_pair<1024, 3, 4> : (const void*)vvh::k_stft_pair<1024, 4, 4>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, (size_t)dyn) != hipSuccess) return -2;
    return per_cu;
}

// an empty kernel of `grid` x 256 threads: the launch + boundary floor of config 3
extern "C" int emptylab_run(int grid, void* stream) {
    hipLaunchKernelGGL(vvh::k_lab_empty, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, vvh::store_sink(), 0);
    return (int)hipGetLastError();
}
