/* vvhip_cpu.c -- TEST INFRASTRUCTURE ONLY: CPU stand-ins for the vvhip_* shim
 * calls that vv-dsp_amd/csrc/host/dist.c makes, so the product's dist.c (linked
 * unchanged into tests/distsim/_build/libdistsim*.so) runs its gather on host
 * memory in 2-3 CPU processes over tests/distsim/fake_rccl.c
 * (tests/test_dist_rccl_sim.py).  "Device" pointers are host pointers and work
 * runs at once, so stream order is trivially kept; the stream waits dist.c asks
 * for are recorded (distsim_waits) so a test can check which stream waits for
 * which.  The STFT / FFT / FIR launches dist.c also references are not used by
 * the gather and report UNSUPPORTED.  Never part of the product library. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vv_dsp/vv_dsp_dist.h"
#include "vv_dsp_hip.h"

#define NDEV 8
#define STREAM_BASE ((uintptr_t)0x5000)

static __thread int g_dev;
static char g_err[256];
static int g_waits[256][2];
static int g_nwaits;
static long long g_mallocs, g_frees;

/* fake stream handle k (0..15) of device `dev`; NULL stays each device's null
 * stream.  Its id in the wait log is dev * 16 + k (-1 - dev for a null stream). */
void* distsim_stream(int dev, int k) { return (void*)(STREAM_BASE + 1 + 16 * (uintptr_t)(dev * 16 + k)); }

static int stream_slot(void* s) {
    const uintptr_t v = (uintptr_t)s;
    if (v < STREAM_BASE + 1 || v >= STREAM_BASE + 1 + 16 * NDEV * 16 || (v - STREAM_BASE - 1) % 16) return -1;
    return (int)((v - STREAM_BASE - 1) / 16);
}
static int stream_dev(void* s) {
    if (!s) return g_dev;
    const int k = stream_slot(s);
    return k < 0 ? -1 : k / 16;
}
static int stream_id(void* s) { return s ? stream_slot(s) : -1 - g_dev; }

int distsim_waits(int* out_pairs, int max_pairs) {
    const int n = g_nwaits < max_pairs ? g_nwaits : max_pairs;
    memcpy(out_pairs, g_waits, sizeof(int) * 2 * (size_t)n);
    return g_nwaits;
}
void distsim_reset(void) { g_nwaits = 0; g_mallocs = g_frees = 0; }
long long distsim_live_allocs(void) { return g_mallocs - g_frees; }

int vvhip_available(void) { return NDEV; }
const char* vvhip_last_error(void) { return g_err; }
void vvhip_set_error(const char* what) { snprintf(g_err, sizeof g_err, "%s", what ? what : ""); }

long long vvhip_debug_get(const char* name) {
    char key[96];
    snprintf(key, sizeof key, "VVHIP_%s", name);
    const char* v = getenv(key);
    return v ? atoll(v) : -1;
}

int vvhip_set_device(int device) {
    if (device < 0 || device >= NDEV) return VV_DSP_ERROR_OUT_OF_RANGE;
    g_dev = device;
    return 0;
}
int vvhip_get_device(int* device) {
    if (!device) return VV_DSP_ERROR_NULL_POINTER;
    *device = g_dev;
    return 0;
}
int vvhip_stream_device(void* stream, int* device) {
    if (!device) return VV_DSP_ERROR_NULL_POINTER;
    const int d = stream_dev(stream);
    if (d < 0) return VV_DSP_ERROR_INTERNAL;
    *device = d;
    return 0;
}
int vvhip_stream_wait(void* waiter, void* producer) {
    if (waiter == producer) return 0;
    if (g_nwaits < 256) {
        g_waits[g_nwaits][0] = stream_id(waiter);
        g_waits[g_nwaits][1] = stream_id(producer);
    }
    ++g_nwaits;
    return 0;
}
int vvhip_malloc_async(void** p, size_t bytes, void* stream) {
    (void)stream;
    if (!p) return VV_DSP_ERROR_NULL_POINTER;
    *p = malloc(bytes ? bytes : 16);
    if (!*p) return VV_DSP_ERROR_INTERNAL;
    ++g_mallocs;
    return 0;
}
int vvhip_free_async(void* p, void* stream) {
    (void)stream;
    if (p) {
        free(p);
        ++g_frees;
    }
    return 0;
}
int vvhip_memcpy_d2d_async(void* dst, const void* src, size_t bytes, void* stream) {
    (void)stream;
    if (bytes && dst != src) memmove(dst, src, bytes);
    return 0;
}
/* the pack / unpack rule of k_rows_half_pack / k_rows_half_unpack
 * (csrc/hip/stft_kernels.hip): pack keeps bins 0..n/2, unpack mirrors */
int vvhip_rows_half_device(const float* in, float* out, size_t rows, size_t n, int unpack, void* stream) {
    (void)stream;
    const size_t h = n / 2 + 1;
    for (size_t r = 0; r < rows; ++r) {
        if (unpack)
            for (size_t k = 0; k < n; ++k) out[r * n + k] = in[r * h + (k < h ? k : n - k)];
        else
            for (size_t k = 0; k < h; ++k) out[r * h + k] = in[r * n + k];
    }
    return 0;
}

size_t vvhip_stft_num_frames(size_t n, size_t nfft, size_t hop) { return n < nfft ? 1 : 1 + (n - nfft + hop) / hop; }

/* launches dist.c references but the gather does not use */
vv_dsp_status vv_dsp_stft_get_sizes(const vv_dsp_stft* h, size_t* a, size_t* b) {
    (void)h; (void)a; (void)b;
    return VV_DSP_ERROR_UNSUPPORTED;
}
vv_dsp_status vv_dsp_stft_channel_shard_device(vv_dsp_stft* h, int device, const vv_dsp_real* d_signal, size_t n,
                                               size_t count, size_t ch_stride, int out_kind, void* d_out,
                                               size_t out_ch_stride, void* stream, size_t* out_frames) {
    (void)h; (void)device; (void)d_signal; (void)n; (void)count; (void)ch_stride; (void)out_kind; (void)d_out;
    (void)out_ch_stride; (void)stream; (void)out_frames;
    return VV_DSP_ERROR_UNSUPPORTED;
}
vv_dsp_status vv_dsp_fft_make_plan_many(size_t n, vv_dsp_fft_type type, vv_dsp_fft_dir dir, size_t batch,
                                        vv_dsp_fft_plan** out) {
    (void)n; (void)type; (void)dir; (void)batch; (void)out;
    return VV_DSP_ERROR_UNSUPPORTED;
}
vv_dsp_status vv_dsp_fft_execute_device(const vv_dsp_fft_plan* p, const void* in, void* out, void* stream) {
    (void)p; (void)in; (void)out; (void)stream;
    return VV_DSP_ERROR_UNSUPPORTED;
}
vv_dsp_status vv_dsp_fft_destroy(vv_dsp_fft_plan* p) {
    (void)p;
    return VV_DSP_OK;
}
vv_dsp_status vv_dsp_fir_apply_fft_device(vv_dsp_fir_plan* p, const vv_dsp_real* x, vv_dsp_real* y, size_t n,
                                          size_t nch, size_t xs, size_t ys, void* stream) {
    (void)p; (void)x; (void)y; (void)n; (void)nch; (void)xs; (void)ys; (void)stream;
    return VV_DSP_ERROR_UNSUPPORTED;
}
