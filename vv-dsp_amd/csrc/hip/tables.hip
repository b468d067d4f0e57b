// tables.hip -- device-resident twiddle tables (computed in double on the
// host, rounded once to f32) and persistent-grid sizing.  Tables are cached per
// (device, kind, n) for the process lifetime; kernels stage them into LDS.
#include "fft_core.hpp"
#include "vvhip_internal.hpp"
#include <cstdlib>

#include <cmath>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

namespace vvh {

namespace {
std::mutex g_mu;
std::map<std::tuple<int, int, long long>, void*> g_cache;   // (device, kind, n) -> device buffer

enum Kind { KIND_WN = 0, KIND_WN_D = 1, KIND_PASS = 2, KIND_SINK = 3, KIND_SPLIT = 4 };

int current_device() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    return dev;
}

// exp(-2*pi*i*num/den) in double, reduced exactly (num mod den) first
void wn(long long num, long long den, double* c, double* s) {
    const long long m = ((num % den) + den) % den;
    const double a = -2.0 * M_PI * (double)m / (double)den;
    *c = std::cos(a);
    *s = std::sin(a);
}

template <class Fill>
void* cached(Kind kind, long long n, size_t bytes, Fill fill) {
    const auto key = std::make_tuple(current_device(), (int)kind, n);
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_cache.find(key);
    if (it != g_cache.end()) return it->second;
    std::vector<unsigned char> h(bytes);
    fill(h.data());
    void* d = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess) return nullptr;
    if (hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return nullptr;
    }
    g_cache[key] = d;
    return d;
}

// Host mirror of Geo<N>::radix / ns (fft_core.hpp) for runtime N.
int radix_of(int n, int p) {
    const int lg = ilog2(n);
    if (n < 16) return n;
    return (lg - 4 * p) >= 4 ? 16 : (1 << (lg - 4 * p));
}
int npass_of(int n) { return n >= 16 ? (ilog2(n) + 3) / 4 : 1; }
}  // namespace

const float2* twiddle_table(int n) {
    return (const float2*)cached(KIND_WN, n, sizeof(float2) * n, [n](unsigned char* b) {
        float2* h = reinterpret_cast<float2*>(b);
        for (int k = 0; k < n; ++k) {
            double c, s;
            wn(k, n, &c, &s);
            h[k] = make_float2((float)c, (float)s);
        }
    });
}

const double2* twiddle_table_d(long long n) {
    return (const double2*)cached(KIND_WN_D, n, sizeof(double2) * n, [n](unsigned char* b) {
        double2* h = reinterpret_cast<double2*>(b);
        for (long long k = 0; k < n; ++k) {
            double c, s;
            wn(k, n, &c, &s);
            h[k] = make_double2(c, s);
        }
    });
}

// Two-level W_n^k for large n: lo[j] = W_n^j (j < 2^lo_bits), then
// hi[j] = W_n^(j << lo_bits) (j < ceil(n / 2^lo_bits)); W_n^k = lo[k & mask] * hi[k >> lo_bits].
const float2* twiddle_split(long long n, int* lo_bits) {
    int lg = 0;
    while ((1LL << lg) < n) ++lg;
    const int lb = (lg + 1) / 2;
    *lo_bits = lb;
    const long long nlo = 1LL << lb, nhi = (n + nlo - 1) >> lb;   // k < n for any n (not only powers of two)
    return (const float2*)cached(KIND_SPLIT, n, sizeof(float2) * (nlo + nhi), [=](unsigned char* b) {
        float2* h = reinterpret_cast<float2*>(b);
        double c, s;
        for (long long j = 0; j < nlo; ++j) {
            wn(j, n, &c, &s);
            h[j] = make_float2((float)c, (float)s);
        }
        for (long long j = 0; j < nhi; ++j) {
            wn(j << lb, n, &c, &s);
            h[nlo + j] = make_float2((float)c, (float)s);
        }
    });
}

// Work counters of the dynamically scheduled launches (k_stft_pair VAR 4/5,
// k_fir_bulk_reg's band walk): blocks of STFT_CTR_WORDS words from per-device
// chunks of CTR_POOL_BLOCKS blocks, each allocated and zeroed ONCE (hipMalloc +
// synchronous memset, outside any graph capture).
//  * eager launches: one block per (device, stream), handed out on the stream's
//    first dynamic launch and kept; the kernel's last wave of each counter
//    stream resets it, so launches ordered on one stream find it zero, and
//    launches on different streams never share one.  A destroyed stream's
//    handle that comes back for a new stream finds its block reset.  When a
//    chunk is used up the next eager request allocates another, so any number
//    of streams gets its own block.
//  * launches recorded into a HIP graph (hipStreamIsCapturing): a block of the
//    capture's own that no other launch uses, zeroed by a captured one-block
//    kernel ahead of the launch, so every replay starts from zero and a replay
//    never shares counters with eager work on the capture stream.  The block is
//    tied to the captured graph by a user object (hipGraphRetainUserObject):
//    when the last graph (and executable graph) holding it is destroyed the
//    block returns to a free list for later captures.  Executable graphs
//    instantiated from ONE captured graph share its blocks: replays of them must
//    not run concurrently (one replay at a time per captured graph, as with any
//    graph whose nodes read and write the same memory).
// Nothing here blocks inside a capture.  When no block is available (a capture
// with every block taken and none freed, or no chunk yet on the device) it
// returns nullptr and the launcher takes its static walk (bit-identical results).
namespace {
// the captured zeroing of a capture's counter block (a kernel node)
__global__ void k_zero_words(unsigned* p, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0u;
}
constexpr int CTR_POOL_BLOCKS = 256;   // 256 x 4 KB per chunk
struct CtrPool {
    std::vector<unsigned*> chunks;
    int used = 0;                           // blocks handed out of the newest chunk
    bool failed = false;
    std::map<hipStream_t, unsigned*> by_stream;
    std::vector<unsigned*> free_capture;    // capture blocks whose graphs are gone
};
std::map<int, CtrPool> g_ctr;
struct CaptureBlock {   // a user object's payload: the block and its pool's device
    int dev;
    unsigned* block;
};
// hipUserObject destructor (runs on a runtime thread once no graph holds it)
void release_capture_block(void* p) {
    CaptureBlock* cb = static_cast<CaptureBlock*>(p);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_ctr[cb->dev].free_capture.push_back(cb->block);
    }
    delete cb;
}
// a fresh block from the chunks; a new chunk only when `grow` (outside captures)
unsigned* bump_block(CtrPool& p, bool grow) {
    constexpr size_t bytes = sizeof(unsigned) * STFT_CTR_WORDS;
    if (p.chunks.empty() || p.used >= CTR_POOL_BLOCKS) {
        if (!grow || p.failed) return nullptr;
        void* d = nullptr;
        if (hipMalloc(&d, bytes * CTR_POOL_BLOCKS) != hipSuccess) {
            p.failed = true;
            return nullptr;
        }
        if (hipMemset(d, 0, bytes * CTR_POOL_BLOCKS) != hipSuccess) {
            (void)hipFree(d);
            p.failed = true;
            return nullptr;
        }
        p.chunks.push_back((unsigned*)d);
        p.used = 0;
    }
    return p.chunks.back() + (size_t)p.used++ * STFT_CTR_WORDS;
}
}  // namespace

unsigned* stream_counters(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipGraph_t graph = nullptr;
    if (hipStreamGetCaptureInfo_v2(s, &cs, nullptr, &graph, nullptr, nullptr) != hipSuccess)
        cs = hipStreamCaptureStatusNone;
    const bool capturing = cs == hipStreamCaptureStatusActive;
    if (cs != hipStreamCaptureStatusNone && !capturing) return nullptr;   // an invalidated capture
    const int dev = current_device();
    if (capturing) {
        if (!graph) return nullptr;
        unsigned* b = nullptr;
        {
            std::lock_guard<std::mutex> lk(g_mu);
            CtrPool& p = g_ctr[dev];
            if (!p.free_capture.empty()) {
                b = p.free_capture.back();
                p.free_capture.pop_back();
            } else {
                b = bump_block(p, false);
            }
        }
        if (!b) return nullptr;
        // tie the block to the captured graph (outside the lock: the destructor
        // takes it): the block comes back when the last graph holding it goes
        CaptureBlock* cb = new (std::nothrow) CaptureBlock{dev, b};
        hipUserObject_t obj = nullptr;
        if (!cb || hipUserObjectCreate(&obj, cb, release_capture_block, 1, hipUserObjectNoDestructorSync) != hipSuccess) {
            if (cb) release_capture_block(cb);   // back to the free list
            return nullptr;
        }
        if (hipGraphRetainUserObject(graph, obj, 1, hipGraphUserObjectMove) != hipSuccess) {
            (void)hipUserObjectRelease(obj, 1);   // the destructor files the block as free
            return nullptr;
        }
        (void)hipGetLastError();   // a stale error must not read as this launch's
        hipLaunchKernelGGL(k_zero_words, dim3(1), dim3(256), 0, s, b, (int)STFT_CTR_WORDS);
        if (hipGetLastError() != hipSuccess) return nullptr;   // the graph still returns it later
        return b;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    CtrPool& p = g_ctr[dev];
    auto it = p.by_stream.find(s);
    if (it != p.by_stream.end()) return it->second;
    unsigned* b = bump_block(p, true);
    if (!b) return nullptr;
    p.by_stream[s] = b;
    return b;
}

// Write sink for lanes whose store has no destination in a kernel that keeps
// its count of memory instructions fixed (SINK_FLOATS floats, never read).
float* store_sink() {
    return (float*)cached(KIND_SINK, 0, sizeof(float) * SINK_FLOATS, [](unsigned char* b) {
        for (size_t i = 0; i < sizeof(float) * SINK_FLOATS; ++i) b[i] = 0;
    });
}

// Pass-major inter-pass twiddles of a length-n Stockham FFT (fft_core.hpp):
// for pass p >= 1 (radix R, stride Ns), entry (r-1)*Ns + j = W_{Ns*R}^{j*r}.
const float2* pass_twiddles(int n) {
    long long entries = 0;
    for (int p = 1, ns = radix_of(n, 0); p < npass_of(n); ns *= radix_of(n, p), ++p)
        entries += (long long)(radix_of(n, p) - 1) * ns;
    if (entries == 0) entries = 1;
    return (const float2*)cached(KIND_PASS, n, sizeof(float2) * entries, [n](unsigned char* b) {
        float2* h = reinterpret_cast<float2*>(b);
        h[0] = make_float2(1.0f, 0.0f);
        long long o = 0;
        for (int p = 1, ns = radix_of(n, 0); p < npass_of(n); ns *= radix_of(n, p), ++p) {
            const int R = radix_of(n, p);
            for (int r = 1; r < R; ++r)
                for (int j = 0; j < ns; ++j) {
                    double c, s;
                    wn((long long)j * r, (long long)ns * R, &c, &s);
                    h[o + (long long)(r - 1) * ns + j] = make_float2((float)c, (float)s);
                }
            o += (long long)(R - 1) * ns;
        }
    });
}

int persistent_grid(const void* kernel, int block, size_t dyn_lds, long long work_blocks, int max_per_cu) {
    static std::atomic<int> cus_cache{0};
    int cus = cus_cache.load(std::memory_order_relaxed);
    if (cus == 0) {
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, current_device());
        if (cus <= 0) cus = 256;
        cus_cache.store(cus, std::memory_order_relaxed);
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, dyn_lds) != hipSuccess ||
        per_cu <= 0)
        per_cu = 1;
    if (max_per_cu > 0 && per_cu > max_per_cu) per_cu = max_per_cu;
    long long g = (long long)cus * per_cu;
    if (work_blocks < g) g = work_blocks;
    if (g < 1) g = 1;
    return (int)g;
}

}  // namespace vvh
