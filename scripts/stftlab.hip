// stftlab.hip -- timing ablations of the product STFT kernel (not part of the
// product; built into scripts/libstftlab.so by `make -C vv-dsp_amd lab`).
// Includes the product sources so the kernel under test is byte-for-byte the
// library's k_stft_pair<1024, 0, 0, EXP>; EXP bits (stft_kernels.hip): 1 FFT
// without LDS exchanges, 2 no FFT, 4 no row stores, 8 no span loads,
// 16 rows as 16 B/lane stores (garbage values), 32 plain instead of streaming stores.
#include "../vv-dsp_amd/csrc/hip/debug.hip"
#include "../vv-dsp_amd/csrc/hip/tables.hip"
#include "../vv-dsp_amd/csrc/hip/stft_kernels.hip"
#include "../vv-dsp_amd/csrc/hip/fir_kernels.hip"
#include "../vv-dsp_amd/csrc/hip/fft_kernels.hip"

namespace vvh {
__global__ void __launch_bounds__(256) k_lab_empty(float* sink, int flag) {
    if (flag == 12345 && threadIdx.x == 0) sink[blockIdx.x] = 1.0f;
}
template <int EXP>
static hipError_t lab_launch(const float* sig, long long n, long long nch, const float* win, float* out,
                             hipStream_t s) {
    constexpr int N = 1024, F = Wg<N>::F;
    const long long hop = 256, frames = n < N ? 1 : 1 + (n - N + hop) / hop, ppc = (frames + 1) / 2;
    static std::atomic<int> cap;
    const int cap0 = cached_grid(cap, (const void*)k_stft_pair<N, 0, 0, EXP>, 256, 0, 1LL << 40);
    const long long pairs = nch * ppc;
    long long cps = (pairs + (long long)F * cap0 - 1) / ((long long)F * cap0);
    cps = cps < 1 ? 1 : (cps > 16 ? 16 : cps);
    const long long chunk = cps * F;
    const long long grid = (EXP & (4096 | 8192)) ? (cap0 / 8) * 8 : (pairs + chunk - 1) / chunk;
    float* sink = store_sink();
    unsigned* ctr = (EXP & 8192) ? stream_counters(s) : nullptr;   // XCD counters (the kernel's last waves reset them)
    hipLaunchKernelGGL((k_stft_pair<N, 0, 0, EXP>), dim3((unsigned)grid), dim3(256), 0, s, sig, n, nch, n, frames, hop,
                       0LL, ppc, win, (void*)out, frames * N, pass_twiddles(N), twiddle_table(N), chunk, sink, ctr, MelArgs{});
    return hipGetLastError();
}
// the product's magnitude launch for large jobs: k_stft_pair<1024, 0, 5, EXP> (persistent,
// dynamic walk in runs of 2 pairs on a span ring, band 2^6 runs per stream)
template <int EXP>
static hipError_t lab_launch5(const float* sig, long long n, long long nch, const float* win, float* out,
                              hipStream_t s) {
    constexpr int N = 1024;
    const long long hop = 256, frames = n < N ? 1 : 1 + (n - N + hop) / hop, ppc = (frames + 1) / 2;
    static std::atomic<int> cap;
    const int capv = cached_grid(cap, (const void*)k_stft_pair<N, 0, 5, EXP>, 256, 0, 1LL << 40);
    const long long chunk = (2LL << 40) | 6;
    unsigned* ctr = stream_counters(s);
    if (!ctr) return hipErrorOutOfMemory;
    hipLaunchKernelGGL((k_stft_pair<N, 0, 5, EXP>), dim3((unsigned)(capv / 8 * 8)), dim3(256), 0, s, sig, n, nch, n,
                       frames, hop, 0LL, ppc, win, (void*)out, frames * N, pass_twiddles(N), twiddle_table(N), chunk,
                       store_sink(), ctr, MelArgs{});
    return hipGetLastError();
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
// the same bulk pairs through the product's register-load kernel k_fir_bulk_reg<1024, EXP>
template <int EXP>
static hipError_t lab_firreg(const float2* H, const float* x, float* y, long long n, long long nch, hipStream_t s) {
    constexpr int N = 1024;
    const long long le = 256, lout = N - le, nblk = (n + lout - 1) / lout, ppc = (nblk + 1) / 2;
    const long long qf = (le + 2 * lout - 1) / (2 * lout);
    long long ql = n / (2 * lout);
    if (ql > ppc) ql = ppc;
    static std::atomic<int> cap;
    const int capv = cached_grid(cap, (const void*)k_fir_bulk_reg<N, EXP>, 256, 0, 1LL << 40);
    const long long cnt = ql - qf, need = (nch * cnt + 3) / 4;
    const int grid = (EXP & 64) ? (int)((nch * cnt + 31) / 32) : (EXP & (128 | 256)) ? capv / 8 * 8 : (int)(need < capv ? need : capv);
    unsigned* ctr = (EXP & 256) ? stream_counters(s) : nullptr;
    hipLaunchKernelGGL((k_fir_bulk_reg<N, EXP>), dim3(grid), dim3(256), 0, s, H, x, y, nch, n, n, cnt, qf,
                       pass_twiddles(N), n, (const float*)nullptr, le, qf, ql, ctr);
    return hipGetLastError();
}
// config 4 through k_fir_r32<EXP> (every pair, edges included; EXP bits 2 no
// FFT, 4 no stores, 8 no loads)
template <int EXP>
static hipError_t lab_firr32(const float2* H, const float* x, float* y, long long n, long long nch, hipStream_t s) {
    constexpr int N = 1024;
    const long long le = 256, lout = N - le, nblk = (n + lout - 1) / lout, ppc = (nblk + 1) / 2;
    long long qf = (le + 2 * lout - 1) / (2 * lout), ql = n / (2 * lout);
    if (ql > ppc) ql = ppc;
    static std::atomic<int> cap;
    const int capv = cached_grid(cap, (const void*)k_fir_r32<EXP>, 256, 0, 1LL << 40);
    const long long couples = (nch * ppc + 1) / 2, need = (couples + 3) / 4;
    int grid = (int)(need < capv ? need : capv);
    if (EXP & 16) grid = (int)((couples + 31) / 32);   // chunks of 8 couples per wave
    if (EXP & 32) grid = capv / 8 * 8;
    unsigned* ctr = (EXP & 32) ? stream_counters(s) : nullptr;
    hipLaunchKernelGGL((k_fir_r32<EXP>), dim3(grid), dim3(256), 0, s, H, x, y, nch, n, n, ppc, twiddle_table(N), n,
                       (const float*)nullptr, le, qf, ql, ctr);
    return hipGetLastError();
}
template <int EXP>
static hipError_t lab_c2c(const float2* in, float2* out, long long batch, hipStream_t s) {
    constexpr int N = 1024, F = Wg<N>::F;
    static std::atomic<int> cap;
    const int grid_cap = cached_grid(cap, (const void*)k_c2c<N, true, EXP>, 256, 0, 1LL << 40);
    const long long need = (batch + F - 1) / F;
    const int grid = (int)(need < grid_cap ? need : grid_cap);
    hipLaunchKernelGGL((k_c2c<N, true, EXP>), dim3(grid), dim3(256), 0, s, in, out, batch, (long long)N, (long long)N,
                       pass_twiddles(N), twiddle_table(N), 1.0f);
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

extern "C" int c2clab_run(int exp, const void* in, void* out, long long batch, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (exp) {
        case 0: return (int)vvh::lab_c2c<0>((const float2*)in, (float2*)out, batch, s);
        case 1: return (int)vvh::lab_c2c<1>((const float2*)in, (float2*)out, batch, s);
        case 2: return (int)vvh::lab_c2c<2>((const float2*)in, (float2*)out, batch, s);
        case 4: return (int)vvh::lab_c2c<4>((const float2*)in, (float2*)out, batch, s);
        case 6: return (int)vvh::lab_c2c<6>((const float2*)in, (float2*)out, batch, s);
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

extern "C" int firreglab_run(int exp, const void* H, const float* x, float* y, long long n, long long nch,
                             void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const float2* h = (const float2*)H;
    switch (exp) {
#define C(E) case E: return (int)vvh::lab_firreg<E>(h, x, y, n, nch, s);
        C(0) C(2) C(4) C(6) C(8) C(10) C(12) C(14) C(16) C(32) C(64) C(80) C(18) C(34) C(66) C(82) C(128) C(144) C(130)
        C(256) C(258) C(266) C(512) C(768) C(770) C(778) C(1536) C(1792) C(1794)
#undef C
        default: return -1;
    }
}

extern "C" int firr32lab_run(int exp, const void* H, const float* x, float* y, long long n, long long nch,
                             void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const float2* h = (const float2*)H;
    switch (exp) {
#define C(E) case E: return (int)vvh::lab_firr32<E>(h, x, y, n, nch, s);
        C(0) C(2) C(4) C(6) C(8) C(10) C(12) C(16) C(32) C(64) C(128) C(96) C(192) C(18) C(34)
#undef C
        default: return -1;
    }
}

extern "C" int stftlab_run(int exp, const float* sig, long long n, long long nch, const float* win, float* out,
                           void* stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (exp) {
#define C(E) case E: return (int)vvh::lab_launch<E>(sig, n, nch, win, out, s);
        C(0) C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13) C(14) C(15)
        C(16) C(18) C(24) C(26) C(32) C(34) C(40) C(42) C(64) C(66) C(68) C(80) C(82)
        C(128) C(256) C(512) C(1024) C(640) C(1152) C(2048) C(2050) C(2052) C(2056) C(4096) C(4098) C(8192) C(8194)
        C(16384) C(16448) C(32782) C(65550) C(98318)
#undef C
        default: return -1;
    }
}

extern "C" int stftlab5_run(int exp, const float* sig, long long n, long long nch, const float* win, float* out,
                            void* stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (exp) {
#define C(E) case E: return (int)vvh::lab_launch5<E>(sig, n, nch, win, out, s);
        C(0) C(2) C(4) C(6) C(8) C(10) C(16) C(18) C(32) C(34) C(512) C(514) C(1024) C(1026) C(128) C(256)
#undef C
        default: return -1;
    }
}

// an empty kernel of `grid` x 256 threads: the launch + boundary floor of config 3
extern "C" int emptylab_run(int grid, void* stream) {
    hipLaunchKernelGGL(vvh::k_lab_empty, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, vvh::store_sink(), 0);
    return (int)hipGetLastError();
}
