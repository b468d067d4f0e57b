// shim.hip -- the extern "C" HIP shim (include/vv_dsp_hip.h).
//
// Owns the device-side objects behind the C99 front-end: FFT plans (own stream,
// lazily grown host-path staging buffers), STFT handles (device window), FIR
// handles (device taps + per-block-size spectra H), and dispatches to the
// kernel launchers of fft_kernels.hip / stft_kernels.hip / fir_kernels.hip /
// spectral_kernels.hip.  There is no CPU compute path: every transform runs on
// the GPU, and every entry point reports UNSUPPORTED/INTERNAL when no device is
// present or a launch fails.
#include "../../../include/vv_dsp_hip.h"
#include "vvhip_internal.hpp"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <algorithm>
#include <vector>

using namespace vvh;

namespace {

enum { ST_OK = 0, ST_NULL = 1, ST_SIZE = 2, ST_RANGE = 3, ST_INTERNAL = 4, ST_NAN = 5, ST_UNSUP = 6 };

thread_local std::string g_err;

int fail(int code, const char* what, hipError_t e = hipSuccess) {
    g_err = what;
    if (e != hipSuccess) {
        g_err += ": ";
        g_err += hipGetErrorString(e);
    }
    return code;
}

#define HIPCHK(expr, code)                                           \
    do {                                                             \
        hipError_t e__ = (expr);                                     \
        if (e__ != hipSuccess) return fail((code), #expr, e__);      \
    } while (0)

int device_count() {
    static int cnt = -1;
    static std::once_flag once;
    std::call_once(once, [] {
        int c = 0;
        if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
        cnt = c;
    });
    return cnt;
}

bool is_pow2(size_t n) { return n && !(n & (n - 1)); }

// Growable device buffer.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
        if (e == hipSuccess) cap = bytes;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Stream-ordered scratch for multi-kernel paths on device pointers.
// Makes device `d` current for a scope and restores the caller's device after
// (host-buffer calls of a handle run on the handle's creation device: its
// stream, staging buffers and window live there).
struct DevGuard {
    int prev = -1;
    explicit DevGuard(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev >= 0 && prev != d && hipSetDevice(d) != hipSuccess) prev = -1;
        if (prev == d) prev = -1;
    }
    ~DevGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DevGuard(const DevGuard&) = delete;
    DevGuard& operator=(const DevGuard&) = delete;
};

struct Scratch {
    void* p = nullptr;
    hipStream_t s;
    explicit Scratch(hipStream_t st) : s(st) {}
    hipError_t alloc(size_t bytes) { return hipMallocAsync(&p, bytes ? bytes : 16, s); }
    ~Scratch() {
        if (p) (void)hipFreeAsync(p, s);
    }
};

// Host-buffer pipeline (the reference API's host pointers).  A large call is
// cut into chunks that alternate between two lanes; each lane is a host thread
// with its own stream and device buffers and runs host->device copy, kernels
// and device->host copy for its chunks.  PCIe is full duplex, so one lane's
// device->host copy overlaps the other lane's host->device copy; a pageable
// hipMemcpy blocks its calling thread, hence two threads rather than two
// streams issued from one.
struct HostLane {
    hipStream_t s = nullptr;
    DevBuf a, b;
    hipError_t init() { return s ? hipSuccess : hipStreamCreateWithFlags(&s, hipStreamNonBlocking); }
    void release() {
        if (s) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
        s = nullptr;
        a.release();
        b.release();
    }
};

size_t host_chunk_bytes() {
    const long long mb = knob(KNOB_HOST_CHUNK_MB, 16);
    return (size_t)(mb > 0 ? mb : 16) << 20;
}

// fn(chunk, lane) enqueues one chunk on lane.s and returns a status; the lane
// synchronises its stream after every chunk, so the caller's host buffers are
// complete when this returns.
template <class F>
int run_lanes(HostLane* lanes, long long nchunks, F&& fn) {
    for (int l = 0; l < 2; ++l) HIPCHK(lanes[l].init(), ST_INTERNAL);
    int dev = 0;
    HIPCHK(hipGetDevice(&dev), ST_INTERNAL);
    int st1 = ST_OK;
    std::string err1;
    std::thread worker([&] {
        if (hipSetDevice(dev) != hipSuccess) {
            st1 = ST_INTERNAL;
            err1 = "host pipeline: hipSetDevice";
            return;
        }
        for (long long c = 1; c < nchunks && st1 == ST_OK; c += 2) {
            st1 = fn(c, lanes[1]);
            if (st1 == ST_OK && hipStreamSynchronize(lanes[1].s) != hipSuccess) st1 = ST_INTERNAL;
        }
        if (st1 != ST_OK) err1 = g_err.empty() ? "host pipeline lane 1" : g_err;
    });
    int st0 = ST_OK;
    for (long long c = 0; c < nchunks && st0 == ST_OK; c += 2) {
        st0 = fn(c, lanes[0]);
        if (st0 == ST_OK) HIPCHK(hipStreamSynchronize(lanes[0].s), ST_INTERNAL);
    }
    worker.join();
    if (st0 != ST_OK) return st0;
    if (st1 != ST_OK) return fail(st1, err1.c_str());
    return ST_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// FFT plans
// ---------------------------------------------------------------------------
struct vvhip_fft {
    size_t n = 0;
    int type = 0;   // 0 C2C 1 R2C 2 C2R
    int dir = 1;
    size_t batch = 1;
    hipStream_t stream = nullptr;
    DevBuf din, dout;
    HostLane lanes[2];
    // The host-buffer path's stream, staging buffers and lanes are per plan:
    // calls on one plan from several threads take turns (the reference's
    // execute takes a const plan and Kiss is reentrant, fft.h:227).
    std::mutex host_mu;
};

static size_t fft_in_elems_bytes(const vvhip_fft* p) {
    switch (p->type) {
        case 0: return p->n * 8;
        case 1: return p->n * 4;
        default: return (p->n / 2 + 1) * 8;
    }
}
static size_t fft_out_elems_bytes(const vvhip_fft* p) {
    switch (p->type) {
        case 0: return p->n * 8;
        case 1: return (p->n / 2 + 1) * 8;
        default: return p->n * 4;
    }
}

// Non-power-of-two DFT: the mixed-radix kernel for 7-smooth n <= 4096, else the
// exact-angle f64 O(n^2) kernel for short lengths and Bluestein over the
// power-of-two kernels from BLUESTEIN_MIN on.  Knob NO_MIXED = 1 skips the
// mixed-radix kernel (A/B and the tests that compare the two).
static bool use_mixed(long long n) { return knob(KNOB_NO_MIXED, 0) != 1 && mixed_supported(n); }
static hipError_t dft_any(long long n, int fwd, const void* in, int real_in, float2* out, long long nout,
                          long long batch, long long in_dist, long long out_dist, float scale, hipStream_t s) {
    if (use_mixed(n))
        return launch_fft_mixed(n, fwd, in, real_in, out, nout, batch, in_dist, out_dist, scale, s);
    if (n >= BLUESTEIN_MIN && bluestein_supported(n))
        return launch_bluestein(n, fwd, in, real_in, out, nout, batch, in_dist, out_dist, scale, s);
    return launch_dft_naive(n, fwd, in, real_in, out, nout, batch, in_dist, out_dist, scale, s);
}

// Core device dispatch: `batch` transforms, contiguous, device pointers.
static int fft_run(size_t n, int type, int dir, const void* in, void* out, size_t batch, hipStream_t s) {
    const long long N = (long long)n, B = (long long)batch;
    if (B == 0) return ST_OK;
    const int fwd = dir > 0;
    if (type == 0) {
        if (c2c_supported(N)) {
            HIPCHK(launch_c2c(N, fwd, (const float2*)in, (float2*)out, B, N, N, 1.0f / (float)N, s), ST_INTERNAL);
            return ST_OK;
        }
        if (n == 1) {
            if (in != out) HIPCHK(hipMemcpyAsync(out, in, 8 * batch, hipMemcpyDeviceToDevice, s), ST_INTERNAL);
            return ST_OK;
        }
        if (is_pow2(n)) {
            if (!c2c_large_supported(N)) return fail(ST_UNSUP, "C2C power-of-two length > 2^24 not supported");
            HIPCHK(launch_c2c_large(N, fwd, (const float2*)in, (float2*)out, B, s), ST_INTERNAL);
            return ST_OK;
        }
        const void* src = in;
        Scratch tmp(s);
        if (in == out && !use_mixed(N)) {   // the mixed-radix kernel reads a transform whole before writing it
            HIPCHK(tmp.alloc(8 * n * batch), ST_INTERNAL);
            HIPCHK(hipMemcpyAsync(tmp.p, in, 8 * n * batch, hipMemcpyDeviceToDevice, s), ST_INTERNAL);
            src = tmp.p;
        }
        HIPCHK(dft_any(N, fwd, src, 0, (float2*)out, N, B, N, N, fwd ? 1.0f : 1.0f / (float)N, s),
               ST_INTERNAL);
        return ST_OK;
    }
    const long long NH = N / 2 + 1;
    if (type == 1) {   // R2C: real[n] -> cpx[n/2+1]
        if (r2c_supported(N)) {
            HIPCHK(launch_r2c(N, (const float*)in, (float2*)out, B, N, NH, s), ST_INTERNAL);
            return ST_OK;
        }
        if (is_pow2(n) && n > 8192 && c2c_large_supported(N / 2) && knob(KNOB_REAL_PROMOTE, 0) != 1) {
            // the n/2-point C2C of the rows as complex pairs, then the split step
            Scratch Z(s);
            HIPCHK(Z.alloc(8 * (n / 2) * batch), ST_INTERNAL);
            HIPCHK(launch_c2c_large(N / 2, 1, (const float2*)in, (float2*)Z.p, B, s), ST_INTERNAL);
            HIPCHK(launch_real_split_fwd((const float2*)Z.p, (float2*)out, N / 2, B, s), ST_INTERNAL);
            return ST_OK;
        }
        if (is_pow2(n) && n > 8192) {   // promote, four-step C2C, keep bins 0..n/2 (fft_kiss.c:120-147)
            if (!c2c_large_supported(N)) return fail(ST_UNSUP, "R2C power-of-two length > 2^24 not supported");
            Scratch z(s), Z(s);
            HIPCHK(z.alloc(8 * n * batch), ST_INTERNAL);
            HIPCHK(Z.alloc(8 * n * batch), ST_INTERNAL);
            HIPCHK(launch_promote_real((const float*)in, (float2*)z.p, N * B, s), ST_INTERNAL);
            HIPCHK(launch_c2c_large(N, 1, (const float2*)z.p, (float2*)Z.p, B, s), ST_INTERNAL);
            HIPCHK(hipMemcpy2DAsync(out, 8 * NH, Z.p, 8 * n, 8 * NH, batch, hipMemcpyDeviceToDevice, s), ST_INTERNAL);
            HIPCHK(launch_zero_nyquist_imag((float2*)out, N, B, NH, s), ST_INTERNAL);
            return ST_OK;
        }
        HIPCHK(dft_any(N, 1, in, 1, (float2*)out, NH, B, N, NH, 1.0f, s), ST_INTERNAL);
        // the single-pass mixed-radix kernels store Im X[n/2] = 0 themselves;
        // the f64 DFT, Bluestein and four-step paths get it here
        if (!(use_mixed(N) && stft_mixed_supported(N)))
            HIPCHK(launch_zero_nyquist_imag((float2*)out, N, B, NH, s), ST_INTERNAL);
        return ST_OK;
    }
    // C2R: cpx[n/2+1] -> real[n]
    if (r2c_supported(N)) {
        HIPCHK(launch_c2r(N, (const float2*)in, (float*)out, B, NH, N, s), ST_INTERNAL);
        return ST_OK;
    }
    if (is_pow2(n) && n > 8192 && c2c_large_supported(N / 2) && knob(KNOB_REAL_PROMOTE, 0) != 1) {
        // inverse split step, then the n/2-point inverse C2C straight into the real rows
        Scratch V(s);
        HIPCHK(V.alloc(8 * (n / 2) * batch), ST_INTERNAL);
        HIPCHK(launch_real_split_inv((const float2*)in, (float2*)V.p, N / 2, B, s), ST_INTERNAL);
        HIPCHK(launch_c2c_large(N / 2, 0, (const float2*)V.p, (float2*)out, B, s), ST_INTERNAL);
        return ST_OK;
    }
    if (is_pow2(n) && n > 8192 && !c2c_large_supported(N))
        return fail(ST_UNSUP, "C2R power-of-two length > 2^24 not supported");
    Scratch full(s), tim(s);
    HIPCHK(full.alloc(8 * n * batch), ST_INTERNAL);
    HIPCHK(tim.alloc(8 * n * batch), ST_INTERNAL);
    HIPCHK(launch_hermitian_expand(N, (const float2*)in, (float2*)full.p, B, NH, 0, s), ST_INTERNAL);
    if (is_pow2(n) && n > 8192)   // Hermitian expand (fft_kiss.c:149-174), four-step inverse
        HIPCHK(launch_c2c_large(N, 0, (const float2*)full.p, (float2*)tim.p, B, s), ST_INTERNAL);
    else
        HIPCHK(dft_any(N, 0, full.p, 0, (float2*)tim.p, N, B, N, N, 1.0f / (float)N, s), ST_INTERNAL);
    HIPCHK(launch_take_real((const float2*)tim.p, (float*)out, N * B, s), ST_INTERNAL);
    return ST_OK;
}

extern "C" {

int vvhip_available(void) { return device_count(); }

const char* vvhip_last_error(void) { return g_err.c_str(); }

const char* vvhip_version(void) { return "vvhip gfx950 (CDNA4) ROCm 7.2"; }

void* vvhip_malloc(size_t bytes) {
    void* p = nullptr;
    if (device_count() <= 0 || hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
    return p;
}
void vvhip_free(void* p) {
    if (p) (void)hipFree(p);
}
int vvhip_memcpy_h2d(void* dst, const void* src, size_t bytes) {
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice), ST_INTERNAL);
    return ST_OK;
}
int vvhip_memcpy_d2h(void* dst, const void* src, size_t bytes) {
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost), ST_INTERNAL);
    return ST_OK;
}
// stream-ordered scratch (hipMallocAsync pool of the stream's device) and copies,
// for the C host code (dist.c); errors land in vvhip_last_error
int vvhip_malloc_async(void** p, size_t bytes, void* stream) {
    if (!p) return ST_NULL;
    *p = nullptr;
    HIPCHK(hipMallocAsync(p, bytes ? bytes : 16, (hipStream_t)stream), ST_INTERNAL);
    return ST_OK;
}
int vvhip_free_async(void* p, void* stream) {
    if (p) HIPCHK(hipFreeAsync(p, (hipStream_t)stream), ST_INTERNAL);
    return ST_OK;
}
int vvhip_memcpy_d2d_async(void* dst, const void* src, size_t bytes, void* stream) {
    if (bytes == 0 || dst == src) return ST_OK;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream), ST_INTERNAL);
    return ST_OK;
}
// the device a stream belongs to (the null stream: the current device's)
int vvhip_stream_device(void* stream, int* device) {
    if (!device) return ST_NULL;
    if (device_count() <= 0) return fail(ST_UNSUP, "no HIP device");
    HIPCHK(hipStreamGetDevice((hipStream_t)stream, device), ST_INTERNAL);
    return ST_OK;
}
// `waiter` waits (on the device) for the work enqueued on `producer` so far:
// an event recorded on the producer's device, waited on by the waiter; the
// event is released once it has completed (hipEventDestroy defers)
int vvhip_stream_wait(void* waiter, void* producer) {
    if (waiter == producer) return ST_OK;
    int prev = 0, pdev = 0;
    HIPCHK(hipGetDevice(&prev), ST_INTERNAL);
    HIPCHK(hipStreamGetDevice((hipStream_t)producer, &pdev), ST_INTERNAL);
    hipEvent_t ev = nullptr;
    hipError_t e = hipSetDevice(pdev);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ev, (hipStream_t)producer);
    (void)hipSetDevice(prev);
    if (e == hipSuccess) e = hipStreamWaitEvent((hipStream_t)waiter, ev, 0);
    if (ev) (void)hipEventDestroy(ev);
    HIPCHK(e, ST_INTERNAL);
    return ST_OK;
}
void vvhip_set_error(const char* what) { g_err = what ? what : ""; }

int vvhip_memset(void* dst, int value, size_t bytes) {
    HIPCHK(hipMemset(dst, value, bytes), ST_INTERNAL);
    return ST_OK;
}
int vvhip_stream_sync(void* stream) {
    HIPCHK(hipStreamSynchronize((hipStream_t)stream), ST_INTERNAL);
    return ST_OK;
}
int vvhip_device_sync(void) {
    HIPCHK(hipDeviceSynchronize(), ST_INTERNAL);
    return ST_OK;
}

int vvhip_set_device(int device) {
    const int nd = device_count();
    if (nd <= 0) return fail(ST_UNSUP, "no HIP device");
    if (device < 0 || device >= nd) return fail(ST_RANGE, "device index");
    HIPCHK(hipSetDevice(device), ST_INTERNAL);
    return ST_OK;
}

int vvhip_get_device(int* device) {
    if (!device) return ST_NULL;
    if (device_count() <= 0) return fail(ST_UNSUP, "no HIP device");
    HIPCHK(hipGetDevice(device), ST_INTERNAL);
    return ST_OK;
}

int vvhip_rows_half_device(const float* d_in, float* d_out, size_t rows, size_t n, int unpack, void* stream) {
    if (!d_in || !d_out) return ST_NULL;
    if (n == 0) return ST_SIZE;
    {   // the kernel reads rows while writing others: any overlap of the byte ranges races
        const size_t h = n / 2 + 1, in_w = unpack ? h : n, out_w = unpack ? n : h;
        const uintptr_t a0 = (uintptr_t)d_in, a1 = a0 + sizeof(float) * rows * in_w;
        const uintptr_t b0 = (uintptr_t)d_out, b1 = b0 + sizeof(float) * rows * out_w;
        if (rows > 0 && a0 < b1 && b0 < a1) return fail(ST_RANGE, "half-row pack/unpack: in and out overlap");
    }
    HIPCHK(launch_rows_half(d_in, d_out, (long long)rows, (long long)n, unpack ? 1 : 0, (hipStream_t)stream),
           ST_INTERNAL);
    return ST_OK;
}

int vvhip_fft_plan_create(size_t n, int type, int dir, size_t batch, vvhip_fft** out) {
    if (!out) return ST_NULL;
    *out = nullptr;
    if (n == 0 || batch == 0) return ST_SIZE;
    if (type < 0 || type > 2 || (dir != 1 && dir != -1)) return ST_RANGE;
    if (device_count() <= 0) return fail(ST_UNSUP, "no HIP device");
    if (is_pow2(n) && n > (1u << 24)) return fail(ST_UNSUP, "power-of-two length > 2^24 not supported");
    vvhip_fft* p = new (std::nothrow) vvhip_fft;
    if (!p) return ST_INTERNAL;
    p->n = n;
    p->type = type;
    p->dir = dir;
    p->batch = batch;
    *out = p;
    return ST_OK;
}

int vvhip_fft_exec_device(vvhip_fft* p, const void* d_in, void* d_out, size_t batch, void* stream) {
    if (!p || !d_in || !d_out) return ST_NULL;
    return fft_run(p->n, p->type, p->dir, d_in, d_out, batch ? batch : p->batch, (hipStream_t)stream);
}

int vvhip_fft_exec_host(vvhip_fft* p, const void* in, void* out) {
    if (!p || !in || !out) return ST_NULL;
    std::lock_guard<std::mutex> host_lock(p->host_mu);
    const size_t ie = fft_in_elems_bytes(p), oe = fft_out_elems_bytes(p);
    const size_t chunk_b = host_chunk_bytes();
    if ((ie + oe) * p->batch >= 2 * chunk_b && p->batch >= 2) {
        // pipelined: chunks of whole transforms on two lanes
        size_t per = chunk_b / (ie > oe ? ie : oe);
        if (per < 1) per = 1;
        const long long nchunks = (long long)((p->batch + per - 1) / per);
        return run_lanes(p->lanes, nchunks, [&](long long c, HostLane& L) -> int {
            const size_t b0 = (size_t)c * per, nb = (p->batch - b0) < per ? (p->batch - b0) : per;
            HIPCHK(L.a.ensure(ie * per), ST_INTERNAL);
            HIPCHK(L.b.ensure(oe * per), ST_INTERNAL);
            HIPCHK(hipMemcpyAsync(L.a.p, (const char*)in + ie * b0, ie * nb, hipMemcpyHostToDevice, L.s),
                   ST_INTERNAL);
            int st = fft_run(p->n, p->type, p->dir, L.a.p, L.b.p, nb, L.s);
            if (st != ST_OK) return st;
            HIPCHK(hipMemcpyAsync((char*)out + oe * b0, L.b.p, oe * nb, hipMemcpyDeviceToHost, L.s), ST_INTERNAL);
            return ST_OK;
        });
    }
    if (!p->stream) HIPCHK(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking), ST_INTERNAL);
    const size_t ib = fft_in_elems_bytes(p) * p->batch, ob = fft_out_elems_bytes(p) * p->batch;
    HIPCHK(p->din.ensure(ib), ST_INTERNAL);
    HIPCHK(p->dout.ensure(ob), ST_INTERNAL);
    HIPCHK(hipMemcpyAsync(p->din.p, in, ib, hipMemcpyHostToDevice, p->stream), ST_INTERNAL);
    int st = fft_run(p->n, p->type, p->dir, p->din.p, p->dout.p, p->batch, p->stream);
    if (st != ST_OK) return st;
    HIPCHK(hipMemcpyAsync(out, p->dout.p, ob, hipMemcpyDeviceToHost, p->stream), ST_INTERNAL);
    HIPCHK(hipStreamSynchronize(p->stream), ST_INTERNAL);
    return ST_OK;
}

void vvhip_fft_plan_destroy(vvhip_fft* p) {
    if (!p) return;
    if (p->stream) {
        (void)hipStreamSynchronize(p->stream);
        (void)hipStreamDestroy(p->stream);
    }
    p->din.release();
    p->dout.release();
    p->lanes[0].release();
    p->lanes[1].release();
    delete p;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// STFT
// ---------------------------------------------------------------------------
struct vvhip_stft {
    size_t nfft = 0, hop = 0;
    float* d_win = nullptr;   // on device `dev` (current at create)
    int dev = 0;
    std::vector<float> h_win;
    std::mutex win_mu;        // per-device window copies for device-pointer calls on other GPUs
    std::vector<std::pair<int, float*>> other_wins;
    hipStream_t stream = nullptr;
    DevBuf b0, b1, b2;
    HostLane lanes[2];
    std::mutex host_mu;   // host-buffer calls on one handle take turns (staging buffers, stream)
};

// out_kind: 0 magnitude rows [frame][nfft], 1 complex rows [frame][nfft],
// 2 power rows [frame][nfft/2+1]
// frame0/nframes: rows of frames [frame0, frame0 + nframes) only (nframes =
// SIZE_MAX: all).  The signal is viewed from frame0's first sample on: frame
// f >= frame0 of the whole signal is frame f - frame0 of that view, and the
// zero padding past n is the same.
// The handle's window on the calling thread's current device: a device-pointer
// call may run on any GPU of the node (one handle, several shards), so the
// window is copied once to each device that uses it.
static const float* stft_window_here(vvhip_stft* h) {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) return nullptr;
    if (d == h->dev) return h->d_win;
    std::lock_guard<std::mutex> lk(h->win_mu);
    for (auto& w : h->other_wins)
        if (w.first == d) return w.second;
    float* p = nullptr;
    if (hipMalloc(&p, sizeof(float) * (h->nfft + 2)) != hipSuccess) return nullptr;
    if (hipMemcpy(p, h->h_win.data(), sizeof(float) * h->nfft, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(p);
        return nullptr;
    }
    h->other_wins.push_back({d, p});
    return p;
}

static int stft_frames_run(vvhip_stft* h, const float* sig, size_t n, size_t nch, size_t ch_stride,
                           void* out, size_t out_ch_stride, int out_kind, hipStream_t s, size_t frame0 = 0,
                           size_t nframes = SIZE_MAX) {
    size_t frames = vvhip_stft_num_frames(n, h->nfft, h->hop);
    const float* win = stft_window_here(h);
    if (!win) return fail(ST_INTERNAL, "stft window on the current device");
    if (out_kind < 0 || out_kind > 2) return fail(ST_RANGE, "stft output kind");
    if (frame0 != 0 || nframes != SIZE_MAX) {
        if (frame0 > frames || (nframes != SIZE_MAX && nframes > frames - frame0))
            return fail(ST_RANGE, "stft frame range past the last frame");
        if (nframes == SIZE_MAX) nframes = frames - frame0;
        if (nframes == 0) return ST_OK;
        const size_t off = frame0 * h->hop;   // < n for every existing frame but a wholly padded last one
        sig += off < n ? off : n;
        n -= off < n ? off : n;
        frames = nframes;
    }
    const long long NF = (long long)h->nfft;
    if (stft_fused_supported(NF)) {
        HIPCHK(launch_stft(NF, (long long)h->hop, out_kind, sig, (long long)n, (long long)nch, (long long)ch_stride,
                           (long long)frames, win, out, (long long)out_ch_stride, s),
               ST_INTERNAL);
        return ST_OK;
    }
    if (knob(KNOB_NO_MIXED, 0) != 1 && stft_mixed_supported(NF)) {   // 7-smooth nfft <= 4096: one kernel
        HIPCHK(launch_stft_mixed(NF, (long long)h->hop, out_kind, sig, (long long)n, (long long)nch,
                                 (long long)ch_stride, (long long)frames, win, out, (long long)out_ch_stride, s),
               ST_INTERNAL);
        return ST_OK;
    }
    const int complex_out = out_kind == 1;
    // generic nfft: gather windowed complex frames, batched C2C, magnitude
    for (size_t c = 0; c < nch; ++c) {
        Scratch fr(s);
        const size_t cnt = frames * h->nfft;
        HIPCHK(fr.alloc(8 * cnt), ST_INTERNAL);
        HIPCHK(launch_frame_gather(NF, (long long)h->hop, sig + c * ch_stride, (long long)n, 1, 0,
                                   (long long)frames, win, (float2*)fr.p, s),
               ST_INTERNAL);
        if (complex_out) {
            int st = fft_run(h->nfft, 0, 1, fr.p, (float2*)out + c * out_ch_stride, frames, s);
            if (st) return st;
        } else {
            int st = fft_run(h->nfft, 0, 1, fr.p, fr.p, frames, s);
            if (st) return st;
            if (out_kind == 2)
                HIPCHK(launch_power_half((const float2*)fr.p, (float*)out + c * out_ch_stride, NF, (long long)frames,
                                         s),
                       ST_INTERNAL);
            else
                HIPCHK(launch_magnitude((const float2*)fr.p, (float*)out + c * out_ch_stride, (long long)cnt, s),
                       ST_INTERNAL);
        }
    }
    return ST_OK;
}

extern "C" {

size_t vvhip_stft_num_frames(size_t n, size_t nfft, size_t hop) {
    if (hop == 0) return 0;
    return (n < nfft) ? 1 : 1 + (n - nfft + hop) / hop;
}

int vvhip_stft_create(size_t nfft, size_t hop, const float* window, vvhip_stft** out) {
    if (!out || !window) return ST_NULL;
    *out = nullptr;
    if (nfft == 0 || hop == 0 || hop > nfft) return ST_SIZE;
    if (device_count() <= 0) return fail(ST_UNSUP, "no HIP device");
    vvhip_stft* h = new (std::nothrow) vvhip_stft;
    if (!h) return ST_INTERNAL;
    h->nfft = nfft;
    h->hop = hop;
    h->h_win.assign(window, window + nfft);
    if (hipGetDevice(&h->dev) != hipSuccess) h->dev = 0;
    if (hipMalloc(&h->d_win, sizeof(float) * (nfft + 2)) != hipSuccess ||
        hipMemcpy(h->d_win, window, sizeof(float) * nfft, hipMemcpyHostToDevice) != hipSuccess) {
        vvhip_stft_destroy(h);
        return fail(ST_INTERNAL, "stft window upload");
    }
    *out = h;
    return ST_OK;
}

void vvhip_stft_destroy(vvhip_stft* h) {
    if (!h) return;
    if (h->stream) {
        (void)hipStreamSynchronize(h->stream);
        (void)hipStreamDestroy(h->stream);
    }
    if (h->d_win) (void)hipFree(h->d_win);
    for (auto& w : h->other_wins) (void)hipFree(w.second);
    h->b0.release();
    h->b1.release();
    h->b2.release();
    h->lanes[0].release();
    h->lanes[1].release();
    delete h;
}

static int stft_stream(vvhip_stft* h) {
    if (!h->stream) HIPCHK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking), ST_INTERNAL);
    return ST_OK;
}

int vvhip_stft_spectrogram_device(vvhip_stft* h, const float* d_signal, size_t n, size_t nch,
                                  size_t ch_stride, void* d_out, size_t out_ch_stride, int complex_out,
                                  void* stream) {
    if (!h || !d_signal || !d_out) return ST_NULL;
    if (nch == 0) return ST_OK;
    return stft_frames_run(h, d_signal, n, nch, ch_stride, d_out, out_ch_stride, complex_out,
                           (hipStream_t)stream);
}

// power rows [ch][frame][nfft/2+1] with rows row_pitch floats apart: in the
// kernel for power-of-two nfft; other lengths write packed rows to scratch and
// place them with one strided copy (the same values)
int vvhip_stft_power_pitched_device(vvhip_stft* h, const float* d_signal, size_t n, size_t nch, size_t ch_stride,
                                    float* d_out, size_t out_ch_stride, size_t row_pitch, void* stream) {
    if (!h || !d_signal || !d_out) return ST_NULL;
    const size_t nb = h->nfft / 2 + 1, frames = vvhip_stft_num_frames(n, h->nfft, h->hop);
    if (row_pitch < nb) return fail(ST_SIZE, "power row pitch below nfft/2+1");
    if (nch > 1 && out_ch_stride < frames * row_pitch) return fail(ST_SIZE, "channel stride below frames x row pitch");
    if (nch == 0) return ST_OK;
    const hipStream_t s = (hipStream_t)stream;
    if (row_pitch == nb)
        return stft_frames_run(h, d_signal, n, nch, ch_stride, d_out, out_ch_stride, 2, s);
    const float* win = stft_window_here(h);
    if (!win) return fail(ST_INTERNAL, "stft window on the current device");
    if (stft_fused_supported((long long)h->nfft)) {
        HIPCHK(launch_stft((long long)h->nfft, (long long)h->hop, 2, d_signal, (long long)n, (long long)nch,
                           (long long)ch_stride, (long long)frames, win, d_out, (long long)out_ch_stride, s,
                           (long long)row_pitch),
               ST_INTERNAL);
        return ST_OK;
    }
    Scratch pw(s);
    HIPCHK(pw.alloc(sizeof(float) * nch * frames * nb), ST_INTERNAL);
    if (int st = stft_frames_run(h, d_signal, n, nch, ch_stride, pw.p, frames * nb, 2, s)) return st;
    for (size_t c = 0; c < nch; ++c)
        HIPCHK(hipMemcpy2DAsync(d_out + c * out_ch_stride, sizeof(float) * row_pitch, (const float*)pw.p + c * frames * nb,
                                sizeof(float) * nb, sizeof(float) * nb, frames, hipMemcpyDeviceToDevice, s),
               ST_INTERNAL);
    return ST_OK;
}

int vvhip_stft_spectrogram_range_device(vvhip_stft* h, const float* d_signal, size_t n, size_t nch,
                                        size_t ch_stride, size_t frame0, size_t nframes, void* d_out,
                                        size_t out_ch_stride, int out_kind, void* stream) {
    if (!h || !d_signal || !d_out) return ST_NULL;
    if (nch == 0) return ST_OK;
    if (nframes == SIZE_MAX) return fail(ST_RANGE, "stft frame count");
    return stft_frames_run(h, d_signal, n, nch, ch_stride, d_out, out_ch_stride, out_kind, (hipStream_t)stream,
                           frame0, nframes);
}

int vvhip_stft_spectrogram_host(vvhip_stft* h, const float* signal, size_t n, float* out_mag) {
    if (!h || !signal || !out_mag) return ST_NULL;
    std::lock_guard<std::mutex> host_lock(h->host_mu);
    DevGuard on_dev(h->dev);   // the handle's stream, buffers and window live on its creation device
    if (int st = stft_stream(h)) return st;
    const size_t frames = vvhip_stft_num_frames(n, h->nfft, h->hop);
    const size_t ob = sizeof(float) * frames * h->nfft;
    const size_t row = sizeof(float) * h->nfft;
    size_t per = (host_chunk_bytes() / row) & ~(size_t)1;   // even: frames pair up as in one launch
    if (per < 2) per = 2;
    if (n >= h->nfft && frames >= 2 * per && stft_fused_supported((long long)h->nfft)) {
        // pipelined over frame chunks; chunk c reads its own span (with the nfft-hop overlap)
        const long long nchunks = (long long)((frames + per - 1) / per);
        return run_lanes(h->lanes, nchunks, [&](long long c, HostLane& L) -> int {
            const size_t f0 = (size_t)c * per, fc = (frames - f0) < per ? (frames - f0) : per;
            const size_t start = f0 * h->hop;
            const size_t want = (fc - 1) * h->hop + h->nfft;
            const size_t len = (n - start) < want ? (n - start) : want;
            HIPCHK(L.a.ensure(sizeof(float) * ((per - 1) * h->hop + h->nfft)), ST_INTERNAL);
            HIPCHK(L.b.ensure(row * per), ST_INTERNAL);
            HIPCHK(hipMemcpyAsync(L.a.p, signal + start, sizeof(float) * len, hipMemcpyHostToDevice, L.s),
                   ST_INTERNAL);
            HIPCHK(launch_stft((long long)h->nfft, (long long)h->hop, 0, (const float*)L.a.p, (long long)len, 1, 0,
                               (long long)fc, h->d_win, L.b.p, (long long)(fc * h->nfft), L.s),
                   ST_INTERNAL);
            HIPCHK(hipMemcpyAsync(out_mag + f0 * h->nfft, L.b.p, row * fc, hipMemcpyDeviceToHost, L.s),
                   ST_INTERNAL);
            return ST_OK;
        });
    }
    HIPCHK(h->b0.ensure(sizeof(float) * (n ? n : 1)), ST_INTERNAL);
    HIPCHK(h->b1.ensure(ob), ST_INTERNAL);
    if (n) HIPCHK(hipMemcpyAsync(h->b0.p, signal, sizeof(float) * n, hipMemcpyHostToDevice, h->stream), ST_INTERNAL);
    int st = stft_frames_run(h, (const float*)h->b0.p, n, 1, 0, h->b1.p, frames * h->nfft, 0, h->stream);
    if (st) return st;
    HIPCHK(hipMemcpyAsync(out_mag, h->b1.p, ob, hipMemcpyDeviceToHost, h->stream), ST_INTERNAL);
    HIPCHK(hipStreamSynchronize(h->stream), ST_INTERNAL);
    return ST_OK;
}

int vvhip_stft_process_device(vvhip_stft* h, const float* d_frames, size_t count, float* d_spec,
                              void* stream) {
    if (!h || !d_frames || !d_spec) return ST_NULL;
    // explicit frames laid back to back: hop = nfft over a count*nfft signal
    const size_t n = count * h->nfft;
    const long long NF = (long long)h->nfft;
    hipStream_t s = (hipStream_t)stream;
    const float* win = stft_window_here(h);
    if (!win) return fail(ST_INTERNAL, "stft window on the current device");
    if (stft_fused_supported(NF)) {
        HIPCHK(launch_stft(NF, NF, 1, d_frames, (long long)n, 1, 0, (long long)count, win, d_spec, 0, s),
               ST_INTERNAL);
        return ST_OK;
    }
    Scratch fr(s);
    HIPCHK(fr.alloc(8 * n), ST_INTERNAL);
    HIPCHK(launch_frame_gather(NF, NF, d_frames, (long long)n, 1, 0, (long long)count, win,
                               (float2*)fr.p, s),
           ST_INTERNAL);
    return fft_run(h->nfft, 0, 1, fr.p, d_spec, count, s);
}

int vvhip_stft_process_host(vvhip_stft* h, const float* frame, float* spec_out) {
    if (!h || !frame || !spec_out) return ST_NULL;
    std::lock_guard<std::mutex> host_lock(h->host_mu);
    DevGuard on_dev(h->dev);   // the handle's stream, buffers and window live on its creation device
    if (int st = stft_stream(h)) return st;
    HIPCHK(h->b0.ensure(sizeof(float) * h->nfft), ST_INTERNAL);
    HIPCHK(h->b1.ensure(8 * h->nfft), ST_INTERNAL);
    HIPCHK(hipMemcpyAsync(h->b0.p, frame, sizeof(float) * h->nfft, hipMemcpyHostToDevice, h->stream),
           ST_INTERNAL);
    int st = vvhip_stft_process_device(h, (const float*)h->b0.p, 1, (float*)h->b1.p, h->stream);
    if (st) return st;
    HIPCHK(hipMemcpyAsync(spec_out, h->b1.p, 8 * h->nfft, hipMemcpyDeviceToHost, h->stream), ST_INTERNAL);
    HIPCHK(hipStreamSynchronize(h->stream), ST_INTERNAL);
    return ST_OK;
}

int vvhip_stft_reconstruct_device(vvhip_stft* h, const float* d_spec, size_t count, size_t hop,
                                  float* d_out_add, float* d_norm_add, void* stream) {
    if (!h || !d_spec || !d_out_add) return ST_NULL;
    if (hop == 0) return ST_SIZE;
    hipStream_t s = (hipStream_t)stream;
    const float* win = stft_window_here(h);
    if (!win) return fail(ST_INTERNAL, "stft window on the current device");
    // knob ISTFT_OLD = 1 (A/B, scripts/kbench.py): IFFT to scratch + k_ola
    if (istft_fused_supported((long long)h->nfft, (long long)hop) && knob(KNOB_ISTFT_OLD, 0) != 1) {
        HIPCHK(launch_istft_fused((long long)h->nfft, (long long)hop, (const float2*)d_spec, (long long)count,
                                  win, d_out_add, d_norm_add, s),
               ST_INTERNAL);
        return ST_OK;
    }
    Scratch tf(s);
    HIPCHK(tf.alloc(8 * h->nfft * count), ST_INTERNAL);
    int st = fft_run(h->nfft, 0, -1, d_spec, tf.p, count, s);
    if (st) return st;
    HIPCHK(launch_ola((long long)h->nfft, (long long)hop, (const float2*)tf.p, (long long)count, win,
                      d_out_add, d_norm_add, s),
           ST_INTERNAL);
    return ST_OK;
}

int vvhip_stft_reconstruct_host(vvhip_stft* h, const float* spec, float* out_add, float* norm_add) {
    if (!h || !spec || !out_add) return ST_NULL;
    std::lock_guard<std::mutex> host_lock(h->host_mu);
    DevGuard on_dev(h->dev);   // the handle's stream, buffers and window live on its creation device
    if (int st = stft_stream(h)) return st;
    const size_t nb = sizeof(float) * h->nfft;
    HIPCHK(h->b0.ensure(2 * nb), ST_INTERNAL);
    HIPCHK(h->b1.ensure(nb), ST_INTERNAL);
    HIPCHK(h->b2.ensure(nb), ST_INTERNAL);
    HIPCHK(hipMemcpyAsync(h->b0.p, spec, 2 * nb, hipMemcpyHostToDevice, h->stream), ST_INTERNAL);
    HIPCHK(hipMemcpyAsync(h->b1.p, out_add, nb, hipMemcpyHostToDevice, h->stream), ST_INTERNAL);
    if (norm_add) HIPCHK(hipMemcpyAsync(h->b2.p, norm_add, nb, hipMemcpyHostToDevice, h->stream), ST_INTERNAL);
    int st = vvhip_stft_reconstruct_device(h, (const float*)h->b0.p, 1, h->nfft, (float*)h->b1.p,
                                           norm_add ? (float*)h->b2.p : nullptr, h->stream);
    if (st) return st;
    HIPCHK(hipMemcpyAsync(out_add, h->b1.p, nb, hipMemcpyDeviceToHost, h->stream), ST_INTERNAL);
    if (norm_add) HIPCHK(hipMemcpyAsync(norm_add, h->b2.p, nb, hipMemcpyDeviceToHost, h->stream), ST_INTERNAL);
    HIPCHK(hipStreamSynchronize(h->stream), ST_INTERNAL);
    return ST_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// FIR
// ---------------------------------------------------------------------------
struct vvhip_fir {
    size_t taps = 0;
    float* d_h = nullptr;
    struct Spec {
        size_t nfft;
        float2* H;
    };
    std::vector<Spec> specs;   // H per overlap-save block size
    std::mutex mu;
    hipStream_t stream = nullptr;
    DevBuf bx, by, bp;
    std::mutex host_mu;   // host-buffer calls on one handle take turns (staging buffers, stream)
};

// Overlap-save block N (= complex FFT size of k_fir_pair): the smallest power
// of two >= max(4*(L-1), 64), so that at least 3/4 of every block is output,
// grown toward the preferred size (1024: four transforms per 256-thread
// workgroup, H and twiddles in 51 KB of LDS) while the signal is longer.
// Knob FIR_BLOCK overrides the preferred size.  0 = no OLS block (long
// filters use the direct form).
static size_t fir_block(const vvhip_fir* f, size_t n) {
    size_t pref = (size_t)knob(KNOB_FIR_BLOCK, 1024);
    if (pref < 64 || pref > 8192 || (pref & (pref - 1))) pref = 1024;
    const size_t lm1 = f->taps - 1;
    size_t nr = 64;
    while (nr < 4 * lm1 && nr < 8192) nr <<= 1;
    while (nr < pref && nr < n + lm1) nr <<= 1;
    if (nr <= lm1 || nr - lm1 < nr / 4) return 0;
    return nr;
}

// Overlap-save block for filters the fused kernels cannot take (taps > 6145):
// N = pow2 >= max(4 (L-1), 16384), at most 2^22, so >= 3/4 of a block is output.
// 0 = none (longer filters than that use the direct form).
static size_t fir_long_block(size_t taps) {
    const size_t lm1 = taps - 1;
    size_t nr = 16384;
    while (nr < 4 * lm1 && nr < ((size_t)1 << 22)) nr <<= 1;
    if (nr <= lm1 || nr - lm1 < nr / 4) return 0;
    return nr;
}

// H for block nr: FFT(h zero-padded to nr) over all nr bins, cached per nr.
// nr <= 8192 (fused kernels): scaled by 1/nr.  nr > 8192 (fir_long_block, the
// four-step path whose inverse applies 1/nr itself): unscaled.
static int fir_spectrum(vvhip_fir* f, size_t nr, const float2** H, hipStream_t s) {
    std::lock_guard<std::mutex> lk(f->mu);
    for (auto& sp : f->specs)
        if (sp.nfft == nr) {
            *H = sp.H;
            return ST_OK;
        }
    float2* Hd = nullptr;
    void* t1 = nullptr;
    void* t2 = nullptr;
    hipError_t e = hipMalloc(&Hd, sizeof(float2) * nr);
    if (nr > 8192) {   // promote h, zero pad, four-step FFT
        if (e == hipSuccess) e = hipMalloc(&t1, sizeof(float2) * nr);
        if (e == hipSuccess) e = hipMemsetAsync(t1, 0, sizeof(float2) * nr, s);
        if (e == hipSuccess) e = launch_promote_real(f->d_h, (float2*)t1, (long long)f->taps, s);
        if (e == hipSuccess) e = launch_c2c_large((long long)nr, 1, (const float2*)t1, Hd, 1, s);
    } else {           // R2C of h zero-padded, Hermitian expand, 1/nr
        if (e == hipSuccess) e = hipMalloc(&t1, sizeof(float) * nr);
        if (e == hipSuccess) e = hipMalloc(&t2, sizeof(float2) * (nr / 2 + 1));
        if (e == hipSuccess) e = hipMemsetAsync(t1, 0, sizeof(float) * nr, s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(t1, f->d_h, sizeof(float) * f->taps, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess)
            e = launch_r2c((long long)nr, (const float*)t1, (float2*)t2, 1, (long long)nr, (long long)(nr / 2 + 1), s);
        if (e == hipSuccess)
            e = launch_hermitian_expand((long long)nr, (const float2*)t2, Hd, 1, (long long)(nr / 2 + 1), 0, s);
        if (e == hipSuccess) e = launch_scale_cpx(Hd, (long long)nr, 1.0f / (float)nr, s);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (t1) (void)hipFree(t1);
    if (t2) (void)hipFree(t2);
    if (e != hipSuccess) {
        if (Hd) (void)hipFree(Hd);
        return fail(ST_INTERNAL, "fir filter spectrum", e);
    }
    f->specs.push_back({nr, Hd});
    *H = Hd;
    return ST_OK;
}

// Zero-state linear convolution (first n outputs) for long filters: overlap-save
// with N = fir_long_block(taps), two blocks per complex row, in chunks of rows
// whose two scratch buffers stay within ~512 MiB.
static int fir_ols_long(vvhip_fir* f, size_t nr, const float* d_x, float* d_y, size_t n, size_t nch,
                        size_t x_stride, size_t y_stride, hipStream_t s) {
    const float2* H = nullptr;
    if (int st = fir_spectrum(f, nr, &H, s)) return st;
    const long long N = (long long)nr, le = (long long)f->taps - 1, lout = N - le;
    const long long nblk = ((long long)n + lout - 1) / lout, ppc = (nblk + 1) / 2;
    const long long items = ppc * (long long)nch;
    long long rows = (256LL << 20) / (8 * N);
    if (rows < 1) rows = 1;
    if (rows > items) rows = items;
    Scratch za(s), zb(s);
    HIPCHK(za.alloc(sizeof(float2) * (size_t)(rows * N)), ST_INTERNAL);
    HIPCHK(zb.alloc(sizeof(float2) * (size_t)(rows * N)), ST_INTERNAL);
    float2* A = (float2*)za.p;
    float2* B = (float2*)zb.p;
    for (long long p0 = 0; p0 < items; p0 += rows) {
        const long long r = items - p0 < rows ? items - p0 : rows;
        HIPCHK(launch_fir_long_gather(d_x, (long long)n, (long long)x_stride, N, le, lout, ppc, p0, r, A, s),
               ST_INTERNAL);
        HIPCHK(launch_c2c_large(N, 1, A, B, r, s), ST_INTERNAL);
        HIPCHK(launch_fir_long_mul(B, H, N, r, s), ST_INTERNAL);
        HIPCHK(launch_c2c_large(N, 0, B, A, r, s), ST_INTERNAL);
        HIPCHK(launch_fir_long_scatter(A, d_y, (long long)n, (long long)y_stride, N, le, lout, ppc, p0, r, s),
               ST_INTERNAL);
    }
    return ST_OK;
}

extern "C" {

int vvhip_fir_create(const float* h, size_t taps, vvhip_fir** out) {
    if (!out || !h) return ST_NULL;
    *out = nullptr;
    if (taps == 0) return ST_SIZE;
    if (device_count() <= 0) return fail(ST_UNSUP, "no HIP device");
    vvhip_fir* f = new (std::nothrow) vvhip_fir;
    if (!f) return ST_INTERNAL;
    f->taps = taps;
    if (hipMalloc(&f->d_h, sizeof(float) * taps) != hipSuccess ||
        hipMemcpy(f->d_h, h, sizeof(float) * taps, hipMemcpyHostToDevice) != hipSuccess) {
        vvhip_fir_destroy(f);
        return fail(ST_INTERNAL, "fir taps upload");
    }
    *out = f;
    return ST_OK;
}

void vvhip_fir_destroy(vvhip_fir* f) {
    if (!f) return;
    if (f->stream) {
        (void)hipStreamSynchronize(f->stream);
        (void)hipStreamDestroy(f->stream);
    }
    if (f->d_h) (void)hipFree(f->d_h);
    for (auto& sp : f->specs) (void)hipFree(sp.H);
    f->bx.release();
    f->by.release();
    f->bp.release();
    delete f;
}

size_t vvhip_fir_block_size(vvhip_fir* f, size_t n) { return f ? fir_block(f, n) : 0; }

int vvhip_fir_apply_device(vvhip_fir* f, const float* d_x, float* d_y, size_t n, size_t nch,
                           size_t x_stride, size_t y_stride, const float* d_prefix, int mode,
                           void* stream) {
    if (!f || !d_x || !d_y) return ST_NULL;
    if (n == 0 || nch == 0) return ST_OK;
    hipStream_t s = (hipStream_t)stream;
    const long long L = (long long)f->taps;
    const size_t nr = mode == 0 ? fir_block(f, n) : 0;
    if (nr) {
        const float2* H = nullptr;
        if (int st = fir_spectrum(f, nr, &H, s)) return st;
        HIPCHK(launch_fir_ols((long long)nr, L, H, d_x, d_y, (long long)n, (long long)nch, (long long)x_stride,
                              (long long)y_stride, d_prefix, s),
               ST_INTERNAL);
        return ST_OK;
    }
    if (mode == 0 && !d_prefix) {   // long zero-state filters: overlap-save over the four-step FFTs
        // (a caller-supplied history takes the direct form below, which reads it)
        const size_t nl = fir_long_block(f->taps);
        if (nl) return fir_ols_long(f, nl, d_x, d_y, n, nch, x_stride, y_stride, s);
    }
    HIPCHK(launch_fir_direct(f->d_h, L, d_x, d_y, (long long)n, (long long)nch, (long long)x_stride,
                             (long long)y_stride, d_prefix, s),
           ST_INTERNAL);
    return ST_OK;
}

int vvhip_fir_apply_host(vvhip_fir* f, const float* x, float* y, size_t n, const float* prefix, int mode) {
    if (!f || !x || !y) return ST_NULL;
    std::lock_guard<std::mutex> host_lock(f->host_mu);
    if (n == 0) return ST_OK;
    if (!f->stream) HIPCHK(hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking), ST_INTERNAL);
    HIPCHK(f->bx.ensure(sizeof(float) * n), ST_INTERNAL);
    HIPCHK(f->by.ensure(sizeof(float) * n), ST_INTERNAL);
    const float* dp = nullptr;
    if (prefix && f->taps > 1) {
        HIPCHK(f->bp.ensure(sizeof(float) * (f->taps - 1)), ST_INTERNAL);
        HIPCHK(hipMemcpyAsync(f->bp.p, prefix, sizeof(float) * (f->taps - 1), hipMemcpyHostToDevice, f->stream),
               ST_INTERNAL);
        dp = (const float*)f->bp.p;
    }
    HIPCHK(hipMemcpyAsync(f->bx.p, x, sizeof(float) * n, hipMemcpyHostToDevice, f->stream), ST_INTERNAL);
    int st = vvhip_fir_apply_device(f, (const float*)f->bx.p, (float*)f->by.p, n, 1, n, n, dp, mode, f->stream);
    if (st) return st;
    HIPCHK(hipMemcpyAsync(y, f->by.p, sizeof(float) * n, hipMemcpyDeviceToHost, f->stream), ST_INTERNAL);
    HIPCHK(hipStreamSynchronize(f->stream), ST_INTERNAL);
    return ST_OK;
}

int vvhip_fir_filtfilt_device(vvhip_fir* f, const float* d_x, float* d_y, size_t n, size_t nch, size_t x_stride,
                              size_t y_stride, void* stream) {
    if (!f || !d_x || !d_y) return ST_NULL;
    if (n == 0 || nch == 0) return ST_OK;
    hipStream_t s = (hipStream_t)stream;
    Scratch tmp(s);
    HIPCHK(tmp.alloc(sizeof(float) * (n + f->taps - 1) * nch), ST_INTERNAL);
    HIPCHK(launch_filtfilt(f->d_h, (long long)f->taps, d_x, d_y, (long long)n, (long long)nch, (long long)x_stride,
                           (long long)y_stride, (float*)tmp.p, s),
           ST_INTERNAL);
    return ST_OK;
}

int vvhip_fir_filtfilt_host(vvhip_fir* f, const float* x, float* y, size_t n) {
    if (!f || !x || !y) return ST_NULL;
    std::lock_guard<std::mutex> host_lock(f->host_mu);
    if (n == 0) return ST_OK;
    if (!f->stream) HIPCHK(hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking), ST_INTERNAL);
    HIPCHK(f->bx.ensure(sizeof(float) * n), ST_INTERNAL);
    HIPCHK(f->by.ensure(sizeof(float) * n), ST_INTERNAL);
    HIPCHK(hipMemcpyAsync(f->bx.p, x, sizeof(float) * n, hipMemcpyHostToDevice, f->stream), ST_INTERNAL);
    int st = vvhip_fir_filtfilt_device(f, (const float*)f->bx.p, (float*)f->by.p, n, 1, n, n, f->stream);
    if (st) return st;
    HIPCHK(hipMemcpyAsync(y, f->by.p, sizeof(float) * n, hipMemcpyDeviceToHost, f->stream), ST_INTERNAL);
    HIPCHK(hipStreamSynchronize(f->stream), ST_INTERNAL);
    return ST_OK;
}

// ---------------------------------------------------------------------------
// Hilbert
// ---------------------------------------------------------------------------
int vvhip_hilbert_device(const float* d_x, size_t n, size_t batch, float* d_z, void* stream) {
    if (!d_x || !d_z) return ST_NULL;
    if (n == 0) return ST_SIZE;
    hipStream_t s = (hipStream_t)stream;
    if (hilbert_fused_supported((long long)n)) {   // one pass: rows in, analytic rows out
        HIPCHK(launch_hilbert_fused((long long)n, d_x, (float2*)d_z, (long long)batch, s), ST_INTERNAL);
        return ST_OK;
    }
    const size_t nh = n / 2 + 1;
    Scratch half(s);
    HIPCHK(half.alloc(8 * nh * batch), ST_INTERNAL);
    int st = fft_run(n, 1, 1, d_x, half.p, batch, s);
    if (st) return st;
    // mask straight into the output buffer, then inverse C2C in place
    HIPCHK(launch_hilbert_mask((long long)n, (const float2*)half.p, (float2*)d_z, (long long)batch, (long long)nh, s),
           ST_INTERNAL);
    return fft_run(n, 0, -1, d_z, d_z, batch, s);
}

int vvhip_hilbert_host(const float* x, size_t n, float* z_out) {
    if (!x || !z_out) return ST_NULL;
    if (n == 0) return ST_SIZE;
    if (device_count() <= 0) return fail(ST_UNSUP, "no HIP device");
    hipStream_t s = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), ST_INTERNAL);
    float* dx = nullptr;
    float* dz = nullptr;
    int st = ST_OK;
    if (hipMalloc(&dx, sizeof(float) * n) != hipSuccess || hipMalloc(&dz, 8 * n) != hipSuccess) {
        st = fail(ST_INTERNAL, "hilbert alloc");
    } else if (hipMemcpyAsync(dx, x, sizeof(float) * n, hipMemcpyHostToDevice, s) != hipSuccess) {
        st = fail(ST_INTERNAL, "hilbert h2d");
    } else {
        st = vvhip_hilbert_device(dx, n, 1, dz, s);
        if (st == ST_OK && (hipMemcpyAsync(z_out, dz, 8 * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
                            hipStreamSynchronize(s) != hipSuccess))
            st = fail(ST_INTERNAL, "hilbert d2h");
    }
    (void)hipStreamSynchronize(s);
    if (dx) (void)hipFree(dx);
    if (dz) (void)hipFree(dz);
    (void)hipStreamDestroy(s);
    return st;
}

// Instantaneous phase / frequency (hilbert.c:77-113)
static constexpr double kTwoPiD = 2.0 * 3.141592653589793238462643383279502884;   // 2 * VV_DSP_PI_D

int vvhip_inst_phase_device(const float* d_z, size_t n, size_t batch, float* d_phase, void* stream) {
    if (!d_z || !d_phase) return ST_NULL;
    if (n == 0) return ST_SIZE;
    if (batch == 0) return ST_OK;
    if (batch > 65535) return fail(ST_RANGE, "instantaneous phase: more than 65535 rows per call");
    HIPCHK(launch_inst_phase((const float2*)d_z, (long long)n, (long long)batch, d_phase, (hipStream_t)stream),
           ST_INTERNAL);
    return ST_OK;
}

int vvhip_inst_freq_device(const float* d_phase, size_t n, size_t batch, double fs, float* d_freq, void* stream) {
    if (!d_phase || !d_freq) return ST_NULL;
    if (n == 0) return ST_SIZE;
    if (batch == 0) return ST_OK;
    hipStream_t s = (hipStream_t)stream;
    Scratch tmp(s);
    if (d_phase == d_freq) {   // f[i] needs p[i-1], which a neighbouring thread overwrites: read a copy
        HIPCHK(tmp.alloc(4 * n * batch), ST_INTERNAL);
        HIPCHK(hipMemcpyAsync(tmp.p, d_phase, 4 * n * batch, hipMemcpyDeviceToDevice, s), ST_INTERNAL);
        d_phase = (const float*)tmp.p;
    }
    HIPCHK(launch_inst_freq(d_phase, (long long)n, (long long)batch, fs / kTwoPiD, d_freq, s), ST_INTERNAL);
    return ST_OK;
}

}  // extern "C"

// one row through the device: in (in_bytes) up, kernel, n floats down
template <class F>
static int host_row(const void* in, size_t in_bytes, float* out, size_t n, const char* what, F&& run) {
    if (device_count() <= 0) return fail(ST_UNSUP, "no HIP device");
    hipStream_t s = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), ST_INTERNAL);
    int st = ST_OK;
    {
        Scratch din(s), dout(s);
        if (din.alloc(in_bytes) != hipSuccess || dout.alloc(sizeof(float) * n) != hipSuccess ||
            hipMemcpyAsync(din.p, in, in_bytes, hipMemcpyHostToDevice, s) != hipSuccess) {
            st = fail(ST_INTERNAL, what);
        } else if ((st = run(din.p, (float*)dout.p, s)) == ST_OK &&
                   (hipMemcpyAsync(out, dout.p, sizeof(float) * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
                    hipStreamSynchronize(s) != hipSuccess)) {
            st = fail(ST_INTERNAL, what);
        }
    }
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    return st;
}

extern "C" {

int vvhip_inst_phase_host(const float* z, size_t n, float* phase) {
    if (!z || !phase) return ST_NULL;
    if (n == 0) return ST_SIZE;
    return host_row(z, 8 * n, phase, n, "instantaneous phase", [&](void* dz, float* dp, hipStream_t s) {
        return vvhip_inst_phase_device((const float*)dz, n, 1, dp, s);
    });
}

int vvhip_inst_freq_host(const float* phase, size_t n, double fs, float* freq) {
    if (!phase || !freq) return ST_NULL;
    if (n == 0) return ST_SIZE;
    return host_row(phase, 4 * n, freq, n, "instantaneous frequency", [&](void* dp, float* df, hipStream_t s) {
        return vvhip_inst_freq_device((const float*)dp, n, 1, fs, df, s);
    });
}

// ---------------------------------------------------------------------------
// Framing (framing.c:58-146)
// ---------------------------------------------------------------------------
int vvhip_fetch_frames_device(const float* d_signal, size_t n, float* d_frames, size_t frame_len, size_t hop,
                              size_t frame0, size_t count, int center, const float* d_window, void* stream) {
    if (!d_signal || !d_frames) return ST_NULL;
    if (n == 0 || frame_len == 0 || hop == 0) return ST_SIZE;
    HIPCHK(launch_fetch_frames(d_signal, 0, (long long)n, d_frames, (long long)frame_len, (long long)hop,
                               (long long)frame0, (long long)count, center, d_window, (hipStream_t)stream),
           ST_INTERNAL);
    return ST_OK;
}

int vvhip_overlap_add_device(const float* d_frames, size_t count, float* d_out, size_t out_len, size_t frame_len,
                             size_t hop, size_t frame0, void* stream) {
    if (!d_frames || !d_out) return ST_NULL;
    if (out_len == 0 || frame_len == 0 || hop == 0) return ST_SIZE;
    HIPCHK(launch_overlap_add(d_frames, (long long)count, d_out, (long long)out_len, (long long)frame_len,
                              (long long)hop, (long long)frame0, (hipStream_t)stream),
           ST_INTERNAL);
    return ST_OK;
}

// One frame through the device: only the span of samples the frame reads
// goes up (for a centred frame near an end, the reflected indices' span).
int vvhip_fetch_frame_host(const float* signal, size_t n, float* frame, size_t frame_len, size_t hop,
                           size_t frame_index, int center, const float* window) {
    if (!signal || !frame) return ST_NULL;
    if (n == 0 || frame_len == 0 || hop == 0) return ST_SIZE;
    if (device_count() <= 0) return fail(ST_UNSUP, "no HIP device");
    const long long N = (long long)n, L = (long long)frame_len;
    const long long start = (long long)(frame_index * hop) - (center ? L / 2 : 0);
    long long lo = N, hi = 0;   // sample span [lo, hi) the frame reads
    if (center) {
        for (long long i = 0; i < L; ++i) {
            const long long k = reflect_sample(start + i, N);
            lo = k < lo ? k : lo;
            hi = k + 1 > hi ? k + 1 : hi;
        }
    } else {
        lo = start < 0 ? 0 : (start < N ? start : N);
        hi = start + L < N ? (start + L > lo ? start + L : lo) : N;
    }
    const long long span = hi > lo ? hi - lo : 0;
    hipStream_t s = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), ST_INTERNAL);
    int st = ST_OK;
    {
        Scratch dsig(s), dwin(s), dfr(s);
        if (dsig.alloc(sizeof(float) * (span > 0 ? span : 1)) != hipSuccess || dfr.alloc(sizeof(float) * L) != hipSuccess ||
            (window && dwin.alloc(sizeof(float) * L) != hipSuccess)) {
            st = fail(ST_INTERNAL, "fetch_frame alloc");
        } else if ((span > 0 && hipMemcpyAsync(dsig.p, signal + lo, sizeof(float) * span, hipMemcpyHostToDevice, s) !=
                                    hipSuccess) ||
                   (window && hipMemcpyAsync(dwin.p, window, sizeof(float) * L, hipMemcpyHostToDevice, s) != hipSuccess)) {
            st = fail(ST_INTERNAL, "fetch_frame h2d");
        } else if (launch_fetch_frames((const float*)dsig.p, lo, N, (float*)dfr.p, L, (long long)hop,
                                       (long long)frame_index, 1, center, window ? (const float*)dwin.p : nullptr,
                                       s) != hipSuccess ||
                   hipMemcpyAsync(frame, dfr.p, sizeof(float) * L, hipMemcpyDeviceToHost, s) != hipSuccess ||
                   hipStreamSynchronize(s) != hipSuccess) {
            st = fail(ST_INTERNAL, "fetch_frame run");
        }
    }
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    return st;
}

// One frame added into out[s0, s0 + frame_len) (clipped to out_len) on the device.
int vvhip_overlap_add_host(const float* frame, float* out, size_t out_len, size_t frame_len, size_t hop,
                           size_t frame_index) {
    if (!frame || !out) return ST_NULL;
    if (out_len == 0 || frame_len == 0 || hop == 0) return ST_SIZE;
    if (device_count() <= 0) return fail(ST_UNSUP, "no HIP device");
    const size_t s0 = frame_index * hop;
    if (s0 >= out_len) return ST_OK;   // nothing lands inside the output (framing.c:137-144)
    const size_t span = out_len - s0 < frame_len ? out_len - s0 : frame_len;
    hipStream_t s = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), ST_INTERNAL);
    int st = ST_OK;
    {
        Scratch dfr(s), dout(s);
        if (dfr.alloc(sizeof(float) * frame_len) != hipSuccess || dout.alloc(sizeof(float) * span) != hipSuccess) {
            st = fail(ST_INTERNAL, "overlap_add alloc");
        } else if (hipMemcpyAsync(dfr.p, frame, sizeof(float) * frame_len, hipMemcpyHostToDevice, s) != hipSuccess ||
                   hipMemcpyAsync(dout.p, out + s0, sizeof(float) * span, hipMemcpyHostToDevice, s) != hipSuccess) {
            st = fail(ST_INTERNAL, "overlap_add h2d");
        } else if (launch_overlap_add((const float*)dfr.p, 1, (float*)dout.p, (long long)span, (long long)frame_len,
                                      (long long)hop, 0, s) != hipSuccess ||
                   hipMemcpyAsync(out + s0, dout.p, sizeof(float) * span, hipMemcpyDeviceToHost, s) != hipSuccess ||
                   hipStreamSynchronize(s) != hipSuccess) {
            st = fail(ST_INTERNAL, "overlap_add run");
        }
    }
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    return st;
}

// ---------------------------------------------------------------------------
// DCT
// ---------------------------------------------------------------------------
// *out_written: whether d_out was written (the ERROR policy stops at a NaN/Inf
// input before anything is written, as dct.c:96-100 returns before the output)
static int dct_run(const float* d_in, float* d_out, size_t n, size_t batch, int type, int dir, int nan_policy,
                   hipStream_t s, bool* out_written);

int vvhip_dct_device(const float* d_in, float* d_out, size_t n, size_t batch, int type, int dir,
                     int nan_policy, void* stream) {
    bool wrote = false;
    return dct_run(d_in, d_out, n, batch, type, dir, nan_policy, (hipStream_t)stream, &wrote);
}

static int dct_run(const float* d_in, float* d_out, size_t n, size_t batch, int type, int dir, int nan_policy,
                   hipStream_t s, bool* out_written) {
    *out_written = false;
    if (!d_in || !d_out) return ST_NULL;
    if (n == 0) return ST_SIZE;
    if ((type != 2 && type != 3 && type != 4) || (dir != 1 && dir != -1)) return ST_RANGE;
    const long long N = (long long)n, B = (long long)batch;
    if (type == 2 && dir > 0 && nan_policy != 2 && dct2_fused_supported(N)) {   // one pass, policy on read
        HIPCHK(launch_dct2_fused(N, d_in, d_out, B, nan_policy, s), ST_INTERNAL);
        *out_written = true;
        return ST_OK;
    }
    Scratch xin(s), flag(s), v(s), V(s);
    HIPCHK(xin.alloc(sizeof(float) * n * batch), ST_INTERNAL);
    HIPCHK(hipMemcpyAsync(xin.p, d_in, sizeof(float) * n * batch, hipMemcpyDeviceToDevice, s), ST_INTERNAL);
    int* dflag = nullptr;
    if (nan_policy == 2) {
        HIPCHK(flag.alloc(sizeof(int)), ST_INTERNAL);
        dflag = (int*)flag.p;
        HIPCHK(hipMemsetAsync(dflag, 0, sizeof(int), s), ST_INTERNAL);
    }
    HIPCHK(launch_nan_policy((float*)xin.p, N * B, nan_policy, dflag, s), ST_INTERNAL);
    if (nan_policy == 2) {
        int h = 0;
        HIPCHK(hipMemcpyAsync(&h, dflag, sizeof(int), hipMemcpyDeviceToHost, s), ST_INTERNAL);
        HIPCHK(hipStreamSynchronize(s), ST_INTERNAL);
        if (h) return ST_NAN;
    }
    // Makhoul re-ordering + a real FFT: power-of-two n, and even 7-smooth n
    // through the mixed-radix kernels (odd n would need the other permutation)
    const bool fast = (is_pow2(n) && n >= 4 && n <= 16384) || (n % 2 == 0 && n >= 4 && use_mixed(N));
    if (fast && type == 2 && dir > 0) {
        const float2* tw4n = twiddle_table((int)(4 * n));
        if (!tw4n) return fail(ST_INTERNAL, "dct twiddles");
        HIPCHK(v.alloc(sizeof(float) * n * batch), ST_INTERNAL);
        HIPCHK(V.alloc(8 * (n / 2 + 1) * batch), ST_INTERNAL);
        HIPCHK(launch_dct2_pre(N, (const float*)xin.p, (float*)v.p, B, s), ST_INTERNAL);
        int st = fft_run(n, 1, 1, v.p, V.p, batch, s);
        if (st) return st;
        HIPCHK(launch_dct2_post(N, (const float2*)V.p, d_out, B, tw4n, s), ST_INTERNAL);
    } else if (fast && (type == 2 || type == 3) && dir < 0) {
        const float2* tw4n = twiddle_table((int)(4 * n));
        if (!tw4n) return fail(ST_INTERNAL, "dct twiddles");
        HIPCHK(v.alloc(sizeof(float) * n * batch), ST_INTERNAL);
        HIPCHK(V.alloc(8 * (n / 2 + 1) * batch), ST_INTERNAL);
        HIPCHK(launch_dct3_pre(N, (const float*)xin.p, (float2*)V.p, B, tw4n, s), ST_INTERNAL);
        int st = fft_run(n, 2, -1, V.p, v.p, batch, s);
        if (st) return st;
        HIPCHK(launch_dct3_post(N, (const float*)v.p, d_out, B, 1.0f, s), ST_INTERNAL);
    } else {
        HIPCHK(launch_dct_naive(N, type, dir, (const float*)xin.p, d_out, B, s), ST_INTERNAL);
    }
    *out_written = true;
    if (nan_policy != 0) {
        if (nan_policy == 2) HIPCHK(hipMemsetAsync(dflag, 0, sizeof(int), s), ST_INTERNAL);
        HIPCHK(launch_nan_policy(d_out, N * B, nan_policy, dflag, s), ST_INTERNAL);
        if (nan_policy == 2) {
            int h = 0;
            HIPCHK(hipMemcpyAsync(&h, dflag, sizeof(int), hipMemcpyDeviceToHost, s), ST_INTERNAL);
            HIPCHK(hipStreamSynchronize(s), ST_INTERNAL);
            if (h) return ST_NAN;
        }
    }
    return ST_OK;
}

int vvhip_dct_host(const float* in, float* out, size_t n, int type, int dir, int nan_policy) {
    if (!in || !out) return ST_NULL;
    if (n == 0) return ST_SIZE;
    if (device_count() <= 0) return fail(ST_UNSUP, "no HIP device");
    hipStream_t s = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), ST_INTERNAL);
    float* di = nullptr;
    float* dout = nullptr;
    int st = ST_OK;
    if (hipMalloc(&di, sizeof(float) * n) != hipSuccess || hipMalloc(&dout, sizeof(float) * n) != hipSuccess) {
        st = fail(ST_INTERNAL, "dct alloc");
    } else if (hipMemcpyAsync(di, in, sizeof(float) * n, hipMemcpyHostToDevice, s) != hipSuccess) {
        st = fail(ST_INTERNAL, "dct h2d");
    } else {
        bool wrote = false;
        st = dct_run(di, dout, n, 1, type, dir, nan_policy, s, &wrote);
        // the reference writes the output buffer even when the OUTPUT check fails
        // (dct.c:128-131), and leaves it untouched when the input check does (:96-100)
        if (wrote && (st == ST_OK || st == ST_NAN) &&
            (hipMemcpyAsync(out, dout, sizeof(float) * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
             hipStreamSynchronize(s) != hipSuccess))
            st = fail(ST_INTERNAL, "dct d2h");
    }
    (void)hipStreamSynchronize(s);
    if (di) (void)hipFree(di);
    if (dout) (void)hipFree(dout);
    (void)hipStreamDestroy(s);
    return st;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Mel / MFCC (src/features/mel.c): filterbank tables staged on the device
// ---------------------------------------------------------------------------
struct vvhip_mel {
    int n_mels = 0, nbins = 0, n_coeffs = 0, nnz = 0;
    float eps = 0.0f;
    float* W = nullptr;     // non-zero weight ranges of every filter, packed
    int* chunks = nullptr;  // balanced chunk schedule of the filters (mel_chunk_schedule)
    int* cbeg = nullptr;    // first chunk of each filter, [n_mels + 1]
    int nc = 0;
    float* Wf = nullptr;    // the fused kernels' chunk windows (MelArgs: rows of lc + 1 floats, lo last)
    int lc = 0;             // window length (0: no fused layout)
    float* D = nullptr;     // DCT-II table [n_coeffs][n_mels]
    float* lift = nullptr;  // lifter factors [n_coeffs]
    hipStream_t stream = nullptr;
    DevBuf bin, bout;
    std::mutex host_mu;   // host-buffer calls on one handle take turns (staging buffers, stream)
};

extern "C" {

void vvhip_mel_destroy(vvhip_mel* m) {
    if (!m) return;
    if (m->stream) {
        (void)hipStreamSynchronize(m->stream);
        (void)hipStreamDestroy(m->stream);
    }
    if (m->W) (void)hipFree(m->W);
    if (m->Wf) (void)hipFree(m->Wf);
    if (m->chunks) (void)hipFree(m->chunks);
    if (m->cbeg) (void)hipFree(m->cbeg);
    if (m->D) (void)hipFree(m->D);
    if (m->lift) (void)hipFree(m->lift);
    m->bin.release();
    m->bout.release();
    delete m;
}

int vvhip_mel_create(const float* fb, size_t n_mels, size_t nbins, size_t n_coeffs, float lifter, float eps,
                     vvhip_mel** out) {
    if (!out) return ST_NULL;
    *out = nullptr;
    if (n_mels == 0 || (fb && nbins == 0) || n_coeffs > n_mels) return ST_SIZE;
    if (device_count() <= 0) return fail(ST_UNSUP, "no HIP device");
    vvhip_mel* m = new (std::nothrow) vvhip_mel;
    if (!m) return ST_INTERNAL;
    m->n_mels = (int)n_mels;
    m->nbins = fb ? (int)nbins : 0;
    m->n_coeffs = (int)n_coeffs;
    m->eps = eps;
    std::vector<float> w;
    std::vector<int> meta(3 * n_mels, 0);   // per filter: lo, len, offset into W (host: the chunk schedule)
    if (fb) {
        for (size_t f = 0; f < n_mels; ++f) {
            const float* r = fb + f * nbins;
            size_t lo = 0, hi = 0;
            for (size_t k = 0; k < nbins; ++k)
                if (r[k] != 0.0f) {
                    if (hi == 0) lo = k;
                    hi = k + 1;
                }
            meta[3 * f] = (int)lo;
            meta[3 * f + 1] = (int)(hi > lo ? hi - lo : 0);
            meta[3 * f + 2] = (int)w.size();
            for (size_t k = lo; k < hi; ++k) w.push_back(r[k]);
        }
    }
    m->nnz = (int)w.size();
    std::vector<int> chunks, cbeg;
    const int lc = mel_chunk_schedule(meta.data(), (int)n_mels, &chunks, &cbeg);
    m->nc = (int)(chunks.size() / 3);
    // The fused kernels' layout (MelArgs, cw = 0): one window of lcw bins per lane
    // slot, a row of MelArgs::window_stride(lcw) floats (the chunk's weights at its
    // own bins, zeros elsewhere, then start | chunk << 16 as int bits).
    // Bank-aware order: the kernel's 64 lanes read their windows' power pairs in
    // lockstep, so chunks whose windows start on the same bank residue (start mod
    // 32, in bins) within one lane group of the read instruction conflict.  Each
    // window may start anywhere in [lo + len - lc, lo] -- extra leading / trailing
    // zero weights add exact zeros, so the sums are bit-identical -- and any chunk
    // may sit in any lane slot, since each slot writes its partial to its chunk's
    // own index (the row's last float: start | chunk << 16).  With MelArgs::W2 the
    // windows are the schedule's lc + 4 bins and start on even bins (two bins per
    // ds_read_b128, whose lane groups are {0-3,12-15,20-27}, {4-11,16-19,28-31},
    // and the same + 32: MI355X_MICROARCH.md LDS table); otherwise ds_read_b64's
    // two 32-lane groups.  Greedy: chunks with the least slack first, each to the
    // (group, start) with the fewest windows on that residue.  The 40-mel /
    // 1024-point plan: 5 -> 2 extra LDS cycles per b64 bin step.
    std::vector<float> wf;
    const int lcw = MelArgs::W2 ? lc + 4 : lc, SS = MelArgs::W2 ? 2 : 1;
    if (fb && m->nc > 0 && lc % 4 == 0 && lcw <= (int)nbins && m->nc < 32768 && nbins < 65536 &&
        (!MelArgs::W2 || nbins == 513)) {   // W2: the fused kernel's rows (nfft 1024) only
        const int lcs = MelArgs::window_stride(lcw), nc = m->nc, nb = (int)nbins;
        // the lane groups of every round (64 slots), as slot lists
        std::vector<std::vector<int>> groups;
        for (int r = 0; 64 * r < nc; ++r) {
            auto add = [&](std::initializer_list<std::pair<int, int>> ranges) {
                std::vector<int> g;
                for (auto rg : ranges)
                    for (int l = rg.first; l <= rg.second; ++l)
                        if (64 * r + l < nc) g.push_back(64 * r + l);
                if (!g.empty()) groups.push_back(g);
            };
            if (MelArgs::W2) {
                for (int h = 0; h < 64; h += 32) {
                    add({{h + 0, h + 3}, {h + 12, h + 15}, {h + 20, h + 27}});
                    add({{h + 4, h + 11}, {h + 16, h + 19}, {h + 28, h + 31}});
                }
            } else {
                add({{0, 31}});
                add({{32, 63}});
            }
        }
        const int ng = (int)groups.size();
        std::vector<int> order(nc), used((size_t)ng * 32, 0), start(nc);
        std::vector<std::vector<int>> members(ng);
        auto smin = [&](int c) { const int v = chunks[3 * c] + chunks[3 * c + 1] - lcw; return v > 0 ? v : 0; };
        // W2: a window may reach 3 bins past the row (the kernel zeroes P's bins
        // nb .. nb + 2), so even the last chunk has an even start
        const int top = MelArgs::W2 ? nb + 3 - lcw : nb - lcw;
        auto smax = [&](int c) { return chunks[3 * c] < top ? chunks[3 * c] : top; };
        for (int c = 0; c < nc; ++c) order[c] = c;
        std::stable_sort(order.begin(), order.end(),
                         [&](int a, int b) { return smax(a) - smin(a) < smax(b) - smin(b); });
        bool ok_sched = true;
        for (int c : order) {
            int bg = -1, bs = 0, bu = 0, bn = 0;
            for (int g = 0; g < ng; ++g) {
                const int n = (int)members[g].size();
                if (n >= (int)groups[g].size()) continue;
                for (int st = smax(c) / SS * SS; st >= smin(c); st -= SS) {
                    const int u = used[(size_t)g * 32 + st % 32];
                    if (bg < 0 || u < bu || (u == bu && n < bn)) {
                        bg = g;
                        bs = st;
                        bu = u;
                        bn = n;
                    }
                }
            }
            if (bg < 0) {   // no start in range (not for lc <= nbins): no windows
                ok_sched = false;
                break;
            }
            ++used[(size_t)bg * 32 + bs % 32];
            members[bg].push_back(c);
            start[c] = bs;
        }
        if (ok_sched) {
            wf.assign((size_t)nc * lcs, 0.0f);
            for (int g = 0; g < ng; ++g)
                for (size_t q = 0; q < members[g].size(); ++q) {
                    const int c = members[g][q], slot = groups[g][q];
                    const int lo = chunks[3 * c], len = chunks[3 * c + 1], off = chunks[3 * c + 2], st = start[c];
                    for (int j = 0; j < lcw; ++j) {
                        const int k = st + j;
                        if (k >= lo && k < lo + len) wf[(size_t)slot * lcs + j] = w[(size_t)off + (k - lo)];
                    }
                    const int bits = st | (c << 16);
                    std::memcpy(&wf[(size_t)slot * lcs + lcw], &bits, sizeof bits);
                }
            m->lc = lcw;
        }
    }
    // DCT-II rows cos(pi (j + 1/2) i / M) (dct.c:21-30), and the lifter of mel.c:300-302
    std::vector<float> D(n_coeffs * n_mels), L(n_coeffs, 1.0f);
    for (size_t i = 0; i < n_coeffs; ++i)
        for (size_t j = 0; j < n_mels; ++j)
            D[i * n_mels + j] = (float)std::cos(M_PI * ((double)j + 0.5) * (double)i / (double)n_mels);
    if (lifter > 0.0f)
        for (size_t i = 1; i < n_coeffs; ++i)
            L[i] = 1.0f + (lifter / 2.0f) * sinf((float)M_PI * (float)i / lifter);
    bool ok = hipMalloc(&m->chunks, sizeof(int) * (chunks.size() + 1)) == hipSuccess &&
              (chunks.empty() ||
               hipMemcpy(m->chunks, chunks.data(), sizeof(int) * chunks.size(), hipMemcpyHostToDevice) == hipSuccess) &&
              hipMalloc(&m->cbeg, sizeof(int) * cbeg.size()) == hipSuccess &&
              hipMemcpy(m->cbeg, cbeg.data(), sizeof(int) * cbeg.size(), hipMemcpyHostToDevice) == hipSuccess &&
              hipMalloc(&m->W, sizeof(float) * (w.size() + 1)) == hipSuccess &&
              hipMalloc(&m->Wf, sizeof(float) * (wf.size() + 1)) == hipSuccess &&
              (wf.empty() || hipMemcpy(m->Wf, wf.data(), sizeof(float) * wf.size(), hipMemcpyHostToDevice) == hipSuccess) &&
              (w.empty() || hipMemcpy(m->W, w.data(), sizeof(float) * w.size(), hipMemcpyHostToDevice) == hipSuccess) &&
              hipMalloc(&m->D, sizeof(float) * (D.size() + 1)) == hipSuccess &&
              (D.empty() || hipMemcpy(m->D, D.data(), sizeof(float) * D.size(), hipMemcpyHostToDevice) == hipSuccess) &&
              hipMalloc(&m->lift, sizeof(float) * (L.size() + 1)) == hipSuccess &&
              (L.empty() || hipMemcpy(m->lift, L.data(), sizeof(float) * L.size(), hipMemcpyHostToDevice) == hipSuccess);
    if (!ok) {
        vvhip_mel_destroy(m);
        return fail(ST_INTERNAL, "mel tables upload");
    }
    *out = m;
    return ST_OK;
}

static size_t mel_in_len(const vvhip_mel* m, int kind) { return kind == 2 ? (size_t)m->n_mels : (size_t)m->nbins; }
static size_t mel_out_len(const vvhip_mel* m, int kind) { return kind == 0 ? (size_t)m->n_mels : (size_t)m->n_coeffs; }

// row_pitch (kinds 0 / 1): floats from one power row's start to the next, >= nbins (0: nbins)
int vvhip_mel_pitched_device(vvhip_mel* m, const float* d_in, size_t frames, size_t row_pitch, float* d_out, int kind,
                             void* stream) {
    if (!m || !d_in || !d_out) return ST_NULL;
    if (kind < 0 || kind > 2) return fail(ST_RANGE, "mel output kind");
    if ((kind != 2 && m->nbins == 0) || (kind != 0 && m->n_coeffs == 0)) return fail(ST_RANGE, "mel plan lacks tables");
    if (kind == 2) row_pitch = 0;
    if (row_pitch != 0 && row_pitch < (size_t)m->nbins) return fail(ST_SIZE, "mel input row pitch below the row length");
    if (frames == 0) return ST_OK;
    const hipStream_t s = (hipStream_t)stream;
    // the kernel stages whole pitched rows (pad included) through LDS; a pad
    // past 64 floats would cost reads (and, far out, more LDS than a CU has):
    // such rows are packed first by one 2-D copy, then run as packed rows
    Scratch packed(s);
    if (row_pitch > (size_t)m->nbins + 64) {
        const size_t rb = sizeof(float) * (size_t)m->nbins;
        HIPCHK(packed.alloc(rb * frames), ST_INTERNAL);
        HIPCHK(hipMemcpy2DAsync(packed.p, rb, d_in, sizeof(float) * row_pitch, rb, frames, hipMemcpyDeviceToDevice, s),
               ST_INTERNAL);
        d_in = (const float*)packed.p;
        row_pitch = 0;
    }
    HIPCHK(launch_mel_grp(kind, d_in, (long long)frames, m->nbins, m->n_mels, m->n_coeffs, m->W, m->nnz, m->chunks,
                          m->nc, m->cbeg, m->D, m->lift, m->eps, d_out, s, (int)row_pitch),
           ST_INTERNAL);
    return ST_OK;
}
int vvhip_mel_device(vvhip_mel* m, const float* d_in, size_t frames, float* d_out, int kind, void* stream) {
    return vvhip_mel_pitched_device(m, d_in, frames, 0, d_out, kind, stream);
}

// Signal -> log-mel (kind 0) / MFCC (kind 1) rows [ch][frame][n_mels or
// n_coeffs]: one fused launch (launch_stft_mel) when the shape allows it, else
// the power rows into scratch and the plan's mel kernel -- the same values.
int vvhip_stft_mel_device(vvhip_stft* h, vvhip_mel* m, const float* d_signal, size_t n, size_t nch, size_t ch_stride,
                          float* d_out, size_t out_ch_stride, int kind, void* stream) {
    if (!h || !m || !d_signal || !d_out) return ST_NULL;
    if (kind != 0 && kind != 1) return fail(ST_RANGE, "stft mel output kind");
    if (m->nbins != (int)(h->nfft / 2 + 1)) return fail(ST_SIZE, "mfcc plan bins differ from the stft's nfft/2+1");
    if (kind == 1 && m->n_coeffs == 0) return fail(ST_RANGE, "mfcc plan lacks the DCT");
    if (nch == 0) return ST_OK;
    const hipStream_t s = (hipStream_t)stream;
    const size_t frames = vvhip_stft_num_frames(n, h->nfft, h->hop);
    const float* win = stft_window_here(h);
    if (!win) return fail(ST_INTERNAL, "stft window on the current device");
    if (knob(KNOB_MEL_FUSED, 1) != 0) {   // 0: the two launches (A/B)
        MelArgs a;
        a.W = m->W;
        a.chunks = m->chunks;
        a.Ww = m->lc > 0 ? m->Wf : nullptr;   // the chunk windows (launch_stft_mel's choice)
        a.lcw = m->lc;
        a.cbeg = m->cbeg;
        a.D = m->D;
        a.lift = m->lift;
        a.nnz = m->nnz;
        a.nc = m->nc;
        a.M = m->n_mels;
        a.C = m->n_coeffs;
        a.eps = m->eps;
        const hipError_t e = launch_stft_mel(kind, (long long)h->nfft, (long long)h->hop, d_signal, (long long)n,
                                             (long long)nch, (long long)ch_stride, (long long)frames, win, a, d_out,
                                             (long long)out_ch_stride, s);
        if (e == hipSuccess) {
            stat_inc(STAT_MEL_FUSED);
            return ST_OK;
        }
        if (e != hipErrorNotSupported) return fail(ST_INTERNAL, hipGetErrorString(e));
        (void)hipGetLastError();
    }
    stat_inc(STAT_MEL_SPLIT);
    const size_t nb = h->nfft / 2 + 1, width = kind == 0 ? (size_t)m->n_mels : (size_t)m->n_coeffs;
    Scratch pw(s);
    HIPCHK(pw.alloc(sizeof(float) * nch * frames * nb), ST_INTERNAL);
    int st = stft_frames_run(h, d_signal, n, nch, ch_stride, pw.p, frames * nb, 2, s);
    if (st) return st;
    if (out_ch_stride == frames * width) return vvhip_mel_device(m, (const float*)pw.p, nch * frames, d_out, kind, stream);
    for (size_t c = 0; c < nch && !st; ++c)
        st = vvhip_mel_device(m, (const float*)pw.p + c * frames * nb, frames, d_out + c * out_ch_stride, kind, stream);
    return st;
}

int vvhip_mel_host(vvhip_mel* m, const float* in, size_t frames, float* out, int kind) {
    if (!m || !in || !out) return ST_NULL;
    std::lock_guard<std::mutex> host_lock(m->host_mu);
    if (kind < 0 || kind > 2) return fail(ST_RANGE, "mel output kind");
    if (frames == 0) return ST_OK;
    if (!m->stream) HIPCHK(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking), ST_INTERNAL);
    const size_t ib = sizeof(float) * frames * mel_in_len(m, kind), ob = sizeof(float) * frames * mel_out_len(m, kind);
    HIPCHK(m->bin.ensure(ib), ST_INTERNAL);
    HIPCHK(m->bout.ensure(ob), ST_INTERNAL);
    HIPCHK(hipMemcpyAsync(m->bin.p, in, ib, hipMemcpyHostToDevice, m->stream), ST_INTERNAL);
    int st = vvhip_mel_device(m, (const float*)m->bin.p, frames, (float*)m->bout.p, kind, m->stream);
    if (st) return st;
    HIPCHK(hipMemcpyAsync(out, m->bout.p, ob, hipMemcpyDeviceToHost, m->stream), ST_INTERNAL);
    HIPCHK(hipStreamSynchronize(m->stream), ST_INTERNAL);
    return ST_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Chirp-z transform (src/spectral/czt.c:58-178) and the cepstrum family
// (src/envelope/cepstrum.c:7-78, minphase.c:7-31): element-wise kernels of
// czt_kernels.hip around the library's own FFTs (fft_run).
// ---------------------------------------------------------------------------
struct vvhip_czt {
    size_t n = 0, m = 0, p = 0;
    float2* g = nullptr;      // [n] A^-n W^(n^2/2)
    float2* post = nullptr;   // [m] W^(k^2/2)
    float2* B = nullptr;      // [p] FFT_p of b[i] = W^(-(i-n+1)^2/2), zero past n+m-1
    float2* Bs = nullptr;     // [p] B / p (the fused kernel's inverse-transform scale folded in)
};

namespace {

// z^e for z = exp(lm + i th) (lm = log|z|, th = arg z) in extended precision:
// e = k^2/2 is exact, the angle is reduced mod 2 pi before cos/sin.  |z| enters
// rounded to float, as the reference's magW = (float)hypot(W) (czt.c:81-82): the
// float components of exp(-2 pi i / N) then give an exact unit-circle arc (their
// |W| = 1 +- 1e-8 would otherwise grow a spiral factor of e^(k^2 * 1e-8 / 2)).
struct Chirp {
    long double lm, th;
    Chirp(float re, float im)
        : lm(logl((long double)(float)hypot((double)re, (double)im))), th(atan2l((long double)im, (long double)re)) {}
};
float2 chirp_value(long double log_mag, long double angle) {
    const long double two_pi = 6.283185307179586476925286766559005768L;
    const long double a = fmodl(angle, two_pi);
    const long double mag = expl(log_mag);
    return make_float2((float)(mag * cosl(a)), (float)(mag * sinl(a)));
}

int czt_run(const vvhip_czt* h, const void* x, int real_in, size_t batch, float2* X, hipStream_t s) {
    if (batch == 0) return ST_OK;
    if (h->Bs && knob(KNOB_CZT_UNFUSED, 0) != 1) {   // knob CZT_UNFUSED = 1: the multi-kernel chain (A/B, tests)
        HIPCHK(launch_czt_fused((long long)h->p, x, real_in, (long long)h->n, (long long)h->m, (long long)batch, h->g,
                                h->Bs, h->post, X, s),
               ST_INTERNAL);
        return ST_OK;
    }
    const size_t p = h->p, esz = real_in ? sizeof(float) : sizeof(float2);
    size_t rows = ((size_t)256 << 20) / (8 * p);   // scratch <= 256 MiB per chunk
    if (rows < 1) rows = 1;
    if (rows > batch) rows = batch;
    Scratch a(s);
    HIPCHK(a.alloc(8 * p * rows), ST_INTERNAL);
    float2* ap = (float2*)a.p;
    for (size_t r0 = 0; r0 < batch; r0 += rows) {
        const size_t rc = batch - r0 < rows ? batch - r0 : rows;
        HIPCHK(launch_czt_pre((const char*)x + esz * h->n * r0, real_in, (long long)h->n, (long long)p,
                              (long long)rc, (long long)h->n, h->g, ap, s),
               ST_INTERNAL);
        int st = fft_run(p, 0, 1, ap, ap, rc, s);
        if (st) return st;
        HIPCHK(launch_cmul_rows(ap, h->B, (long long)p, (long long)rc, s), ST_INTERNAL);
        if ((st = fft_run(p, 0, -1, ap, ap, rc, s))) return st;
        HIPCHK(launch_czt_post(ap, (long long)h->n, (long long)p, (long long)h->m, (long long)rc, h->post,
                               X + h->m * r0, (long long)h->m, s),
               ST_INTERNAL);
    }
    return ST_OK;
}

// One call through the device: in_bytes up, run(din, dout, stream), out_bytes down.
template <class F>
int host_io(const void* in, size_t in_bytes, void* out, size_t out_bytes, const char* what, F&& run) {
    if (device_count() <= 0) return fail(ST_UNSUP, "no HIP device");
    hipStream_t s = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), ST_INTERNAL);
    int st = ST_OK;
    {
        Scratch din(s), dout(s);
        if (din.alloc(in_bytes) != hipSuccess || dout.alloc(out_bytes) != hipSuccess ||
            hipMemcpyAsync(din.p, in, in_bytes, hipMemcpyHostToDevice, s) != hipSuccess) {
            st = fail(ST_INTERNAL, what);
        } else if ((st = run(din.p, dout.p, s)) == ST_OK &&
                   (hipMemcpyAsync(out, dout.p, out_bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
                    hipStreamSynchronize(s) != hipSuccess)) {
            st = fail(ST_INTERNAL, what);
        }
    }
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    return st;
}

}  // namespace

extern "C" {

int vvhip_czt_create(size_t n, size_t m, float w_re, float w_im, float a_re, float a_im, vvhip_czt** out) {
    if (!out) return ST_NULL;
    *out = nullptr;
    if (n == 0 || m == 0) return ST_SIZE;
    if (device_count() <= 0) return fail(ST_UNSUP, "no HIP device");
    const size_t L = n + m - 1;
    size_t p = 1;
    while (p < L) p <<= 1;
    if (p > ((size_t)1 << 24)) return fail(ST_UNSUP, "CZT: N + M - 1 above 2^24");
    const Chirp W(w_re, w_im), A(a_re, a_im);
    std::vector<float2> g(n), post(m), b(p, make_float2(0.0f, 0.0f));
    for (size_t k = 0; k < n; ++k) {   // A^-k W^(k^2/2)
        const long double e = 0.5L * (long double)k * (long double)k, kk = (long double)k;
        g[k] = chirp_value(e * W.lm - kk * A.lm, e * W.th - kk * A.th);
    }
    for (size_t k = 0; k < m; ++k) {
        const long double e = 0.5L * (long double)k * (long double)k;
        post[k] = chirp_value(e * W.lm, e * W.th);
    }
    for (size_t i = 0; i < L; ++i) {   // W^(-j^2/2), j = i - (n - 1)
        const long double j = (long double)i - (long double)(n - 1), e = 0.5L * j * j;
        b[i] = chirp_value(-e * W.lm, -e * W.th);
    }
    vvhip_czt* h = new (std::nothrow) vvhip_czt;
    if (!h) return fail(ST_INTERNAL, "czt alloc");
    h->n = n;
    h->m = m;
    h->p = p;
    int st = ST_OK;
    if (hipMalloc(&h->g, 8 * n) != hipSuccess || hipMalloc(&h->post, 8 * m) != hipSuccess ||
        hipMalloc(&h->B, 8 * p) != hipSuccess || hipMemcpy(h->g, g.data(), 8 * n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(h->post, post.data(), 8 * m, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(h->B, b.data(), 8 * p, hipMemcpyHostToDevice) != hipSuccess) {
        st = fail(ST_INTERNAL, "czt tables");
    } else if ((st = fft_run(p, 0, 1, h->B, h->B, 1, nullptr)) == ST_OK && hipDeviceSynchronize() != hipSuccess) {
        st = fail(ST_INTERNAL, "czt chirp spectrum");
    } else if (st == ST_OK && czt_fused_supported((long long)p)) {   // B / p for the one-pass kernel
        if (hipMalloc(&h->Bs, 8 * p) != hipSuccess ||
            hipMemcpy(h->Bs, h->B, 8 * p, hipMemcpyDeviceToDevice) != hipSuccess ||
            launch_scale_cpx(h->Bs, (long long)p, 1.0f / (float)p, nullptr) != hipSuccess ||
            hipDeviceSynchronize() != hipSuccess)
            st = fail(ST_INTERNAL, "czt scaled chirp spectrum");
    }
    if (st != ST_OK) {
        vvhip_czt_destroy(h);
        return st;
    }
    *out = h;
    return ST_OK;
}

void vvhip_czt_destroy(vvhip_czt* h) {
    if (!h) return;
    if (h->g) (void)hipFree(h->g);
    if (h->post) (void)hipFree(h->post);
    if (h->B) (void)hipFree(h->B);
    if (h->Bs) (void)hipFree(h->Bs);
    delete h;
}

int vvhip_czt_exec_device(const vvhip_czt* h, const void* d_x, int real_in, size_t batch, void* d_X,
                          void* stream) {
    if (!h || !d_x || !d_X) return ST_NULL;
    return czt_run(h, d_x, real_in, batch, (float2*)d_X, (hipStream_t)stream);
}

int vvhip_czt_exec_host(const void* x, int real_in, size_t n, size_t m, float w_re, float w_im, float a_re,
                        float a_im, void* X) {
    if (!x || !X) return ST_NULL;
    vvhip_czt* h = nullptr;
    int st = vvhip_czt_create(n, m, w_re, w_im, a_re, a_im, &h);
    if (st) return st;
    st = host_io(x, (real_in ? 4 : 8) * n, X, 8 * m, "czt", [&](void* dx, void* dX, hipStream_t s) {
        return czt_run(h, dx, real_in, 1, (float2*)dX, s);
    });
    vvhip_czt_destroy(h);
    return st;
}

// one-pass kernels for pow2 n <= 4096; knob CEPS_UNFUSED = 1 selects the chains (A/B, tests)
static bool ceps_fused(size_t n) { return ceps_fused_supported((long long)n) && knob(KNOB_CEPS_UNFUSED, 0) != 1; }

int vvhip_cepstrum_device(const float* d_x, size_t n, size_t batch, float* d_c, void* stream) {
    if (!d_x || !d_c) return ST_NULL;
    if (n == 0) return ST_SIZE;
    if (batch == 0) return ST_OK;
    hipStream_t s = (hipStream_t)stream;
    if (ceps_fused(n)) {
        HIPCHK(launch_ceps_fused(0, (long long)n, d_x, (long long)batch, d_c, s), ST_INTERNAL);
        return ST_OK;
    }
    const size_t nh = n / 2 + 1;
    Scratch half(s);
    HIPCHK(half.alloc(8 * nh * batch), ST_INTERNAL);
    int st = fft_run(n, 1, 1, d_x, half.p, batch, s);
    if (st) return st;
    HIPCHK(launch_log_magnitude((float2*)half.p, (long long)(nh * batch), s), ST_INTERNAL);
    return fft_run(n, 2, -1, half.p, d_c, batch, s);
}

int vvhip_icepstrum_minphase_device(const float* d_c, size_t n, size_t batch, float* d_x, void* stream) {
    if (!d_c || !d_x) return ST_NULL;
    if (n == 0) return ST_SIZE;
    if (batch == 0) return ST_OK;
    hipStream_t s = (hipStream_t)stream;
    if (ceps_fused(n)) {
        HIPCHK(launch_ceps_fused(1, (long long)n, d_c, (long long)batch, d_x, s), ST_INTERNAL);
        return ST_OK;
    }
    Scratch C(s);
    HIPCHK(C.alloc(8 * n * batch), ST_INTERNAL);
    float2* cp = (float2*)C.p;
    HIPCHK(launch_cepstrum_fold(d_c, (long long)n, (long long)batch, cp, s), ST_INTERNAL);
    int st = fft_run(n, 0, 1, cp, cp, batch, s);
    if (st) return st;
    HIPCHK(launch_exp_real(cp, (long long)(n * batch), 0, s), ST_INTERNAL);
    if ((st = fft_run(n, 0, -1, cp, cp, batch, s))) return st;
    HIPCHK(launch_take_real(cp, d_x, (long long)(n * batch), s), ST_INTERNAL);
    return ST_OK;
}

int vvhip_minphase_from_cepstrum_device(const float* d_c, size_t n, size_t batch, float* d_spec, void* stream) {
    if (!d_c || !d_spec) return ST_NULL;
    if (n == 0) return ST_SIZE;
    if (batch == 0) return ST_OK;
    hipStream_t s = (hipStream_t)stream;
    if (ceps_fused(n)) {
        HIPCHK(launch_ceps_fused(2, (long long)n, d_c, (long long)batch, d_spec, s), ST_INTERNAL);
        return ST_OK;
    }
    float2* sp = (float2*)d_spec;
    HIPCHK(launch_cepstrum_fold(d_c, (long long)n, (long long)batch, sp, s), ST_INTERNAL);
    int st = fft_run(n, 0, 1, sp, sp, batch, s);
    if (st) return st;
    HIPCHK(launch_exp_real(sp, (long long)(n * batch), 1, s), ST_INTERNAL);
    return ST_OK;
}

int vvhip_cepstrum_host(const float* x, size_t n, float* c) {
    if (!x || !c) return ST_NULL;
    if (n == 0) return ST_SIZE;
    return host_io(x, 4 * n, c, 4 * n, "cepstrum", [&](void* dx, void* dc, hipStream_t s) {
        return vvhip_cepstrum_device((const float*)dx, n, 1, (float*)dc, s);
    });
}

int vvhip_icepstrum_minphase_host(const float* c, size_t n, float* x) {
    if (!c || !x) return ST_NULL;
    if (n == 0) return ST_SIZE;
    return host_io(c, 4 * n, x, 4 * n, "icepstrum", [&](void* dc, void* dx, hipStream_t s) {
        return vvhip_icepstrum_minphase_device((const float*)dc, n, 1, (float*)dx, s);
    });
}

int vvhip_minphase_from_cepstrum_host(const float* c, size_t n, float* spec) {
    if (!c || !spec) return ST_NULL;
    if (n == 0) return ST_SIZE;
    return host_io(c, 4 * n, spec, 8 * n, "minphase", [&](void* dc, void* ds, hipStream_t s) {
        return vvhip_minphase_from_cepstrum_device((const float*)dc, n, 1, (float*)ds, s);
    });
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Spectral utilities (src/spectral/utils.c:5-73): fftshift / ifftshift,
// phase wrap and unwrap on `batch` contiguous rows of n.
// ---------------------------------------------------------------------------
extern "C" {

int vvhip_fftshift_device(const void* d_in, void* d_out, size_t n, size_t batch, int cpx, int inverse,
                          void* stream) {
    if (!d_in || !d_out) return ST_NULL;
    if (n == 0) return ST_SIZE;
    hipStream_t s = (hipStream_t)stream;
    const size_t bytes = (cpx ? 8 : 4) * n * batch;
    const void* src = d_in;
    Scratch tmp(s);
    if (d_in == d_out && batch) {   // a permutation in place: read from a copy
        HIPCHK(tmp.alloc(bytes), ST_INTERNAL);
        HIPCHK(hipMemcpyAsync(tmp.p, d_in, bytes, hipMemcpyDeviceToDevice, s), ST_INTERNAL);
        src = tmp.p;
    }
    HIPCHK(launch_fftshift(src, d_out, (long long)n, (long long)batch, cpx, inverse, s), ST_INTERNAL);
    return ST_OK;
}

int vvhip_phase_wrap_device(const float* d_in, float* d_out, size_t count, void* stream) {
    if (!d_in || !d_out) return ST_NULL;
    HIPCHK(launch_phase_wrap(d_in, d_out, (long long)count, (hipStream_t)stream), ST_INTERNAL);
    return ST_OK;
}

int vvhip_phase_unwrap_device(const float* d_in, float* d_out, size_t n, size_t batch, void* stream) {
    if (!d_in || !d_out) return ST_NULL;
    if (n == 0) return ST_SIZE;
    if (batch == 0) return ST_OK;
    if (batch > 65535) return fail(ST_RANGE, "phase unwrap: more than 65535 rows per call");
    hipStream_t s = (hipStream_t)stream;
    const float* src = d_in;
    Scratch tmp(s);
    if (d_in == d_out) {   // the scan reads neighbours: read from a copy
        HIPCHK(tmp.alloc(4 * n * batch), ST_INTERNAL);
        HIPCHK(hipMemcpyAsync(tmp.p, d_in, 4 * n * batch, hipMemcpyDeviceToDevice, s), ST_INTERNAL);
        src = (const float*)tmp.p;
    }
    HIPCHK(launch_phase_unwrap(src, (long long)n, (long long)batch, d_out, s), ST_INTERNAL);
    return ST_OK;
}

int vvhip_fftshift_host(const void* in, void* out, size_t n, int cpx, int inverse) {
    if (!in || !out) return ST_NULL;
    if (n == 0) return ST_SIZE;
    const size_t bytes = (cpx ? 8 : 4) * n;
    return host_io(in, bytes, out, bytes, "fftshift", [&](void* di, void* dout, hipStream_t s) {
        return vvhip_fftshift_device(di, dout, n, 1, cpx, inverse, s);
    });
}

int vvhip_phase_wrap_host(const float* in, float* out, size_t n) {
    if (!in || !out) return ST_NULL;
    if (n == 0) return ST_OK;   // utils.c:51-61 loops zero times
    return host_io(in, 4 * n, out, 4 * n, "phase wrap", [&](void* di, void* dout, hipStream_t s) {
        return vvhip_phase_wrap_device((const float*)di, (float*)dout, n, s);
    });
}

int vvhip_phase_unwrap_host(const float* in, float* out, size_t n) {
    if (!in || !out) return ST_NULL;
    if (n == 0) return ST_SIZE;
    return host_io(in, 4 * n, out, 4 * n, "phase unwrap", [&](void* di, void* dout, hipStream_t s) {
        return vvhip_phase_unwrap_device((const float*)di, (float*)dout, n, 1, s);
    });
}

}  // extern "C"
