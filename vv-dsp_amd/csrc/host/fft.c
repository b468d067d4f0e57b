/* fft.c -- vv-dsp FFT front-end and backend dispatcher (C99).
 *
 * Replaces src/spectral/fft.c:9-124 of the reference with the same public
 * behaviour (argument validation order and status codes of :63-107, backend
 * snapshot per plan, NULL-safe destroy) plus:
 *   - a fourth vtable slot, VV_DSP_FFT_BACKEND_HIP, served by fft_hip.c;
 *   - the backend's free_plan is actually called on destroy (the reference's
 *     legacy shim fft_kiss.c:211-216 is a no-op);
 *   - thread-safe one-time registration (pthread_once);
 *   - the environment variable VV_DSP_BACKEND_FFT ("hip", "kiss", "fftw",
 *     "ffts") selects the initial backend (dead in the reference);
 *     otherwise HIP when a device is present.
 * The CPU backends are not part of this library: their vtables are weak
 * references, filled only when a program also links the reference's own
 * backend objects. */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include "fft_backend.h"
#include "vv_dsp/vv_dsp_amd.h"
#include "vv_dsp_hip.h"

extern const vv_dsp_fft_backend_vtable vv_dsp_fft_kiss_vtable __attribute__((weak));
extern const vv_dsp_fft_backend_vtable vv_dsp_fft_fftw_vtable __attribute__((weak));
extern const vv_dsp_fft_backend_vtable vv_dsp_fft_ffts_vtable __attribute__((weak));

const vv_dsp_fft_backend_vtable* g_fft_backends[VV_DSP_FFT_NUM_BACKENDS];
static vv_dsp_fft_backend g_current = VV_DSP_FFT_BACKEND_HIP;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* make_plan_many -> vtable->make_plan hand-off of the batch count (fft_backend.h) */
static __thread const struct vv_dsp_fft_plan* t_pending_spec;
static __thread size_t t_pending_batch;

size_t vv_amd_fft_pending_batch(const struct vv_dsp_fft_plan* spec) {
    return (spec && spec == t_pending_spec) ? t_pending_batch : 1;
}

static int slot_ok(int b) {
    return b >= 0 && b < VV_DSP_FFT_NUM_BACKENDS && g_fft_backends[b] && g_fft_backends[b]->is_available();
}

static void init_backends(void) {
    g_fft_backends[VV_DSP_FFT_BACKEND_KISS] = &vv_dsp_fft_kiss_vtable ? &vv_dsp_fft_kiss_vtable : NULL;
    g_fft_backends[VV_DSP_FFT_BACKEND_FFTW] = &vv_dsp_fft_fftw_vtable ? &vv_dsp_fft_fftw_vtable : NULL;
    g_fft_backends[VV_DSP_FFT_BACKEND_FFTS] = &vv_dsp_fft_ffts_vtable ? &vv_dsp_fft_ffts_vtable : NULL;
    g_fft_backends[VV_DSP_FFT_BACKEND_HIP] = &vv_dsp_fft_hip_vtable;

    int want = -1;
    const char* env = getenv("VV_DSP_BACKEND_FFT");
    if (env) {
        if (!strcasecmp(env, "hip") || !strcasecmp(env, "gfx950")) want = VV_DSP_FFT_BACKEND_HIP;
        else if (!strcasecmp(env, "kiss") || !strcasecmp(env, "kissfft")) want = VV_DSP_FFT_BACKEND_KISS;
        else if (!strcasecmp(env, "fftw")) want = VV_DSP_FFT_BACKEND_FFTW;
        else if (!strcasecmp(env, "ffts")) want = VV_DSP_FFT_BACKEND_FFTS;
    }
    if (want >= 0 && slot_ok(want)) g_current = (vv_dsp_fft_backend)want;
    else if (slot_ok(VV_DSP_FFT_BACKEND_HIP)) g_current = VV_DSP_FFT_BACKEND_HIP;
    else if (slot_ok(VV_DSP_FFT_BACKEND_KISS)) g_current = VV_DSP_FFT_BACKEND_KISS;
    else g_current = VV_DSP_FFT_BACKEND_HIP;   /* nothing usable: make_plan reports UNSUPPORTED */
}

static void ensure_init(void) { (void)pthread_once(&g_once, init_backends); }

vv_dsp_status vv_dsp_fft_set_backend(vv_dsp_fft_backend backend) {
    if ((int)backend < 0 || (int)backend >= VV_DSP_FFT_NUM_BACKENDS) return VV_DSP_ERROR_OUT_OF_RANGE;
    ensure_init();
    if (!slot_ok(backend)) return VV_DSP_ERROR_UNSUPPORTED;
    g_current = backend;
    return VV_DSP_OK;
}

vv_dsp_fft_backend vv_dsp_fft_get_backend(void) {
    ensure_init();
    return g_current;
}

int vv_dsp_fft_is_backend_available(vv_dsp_fft_backend backend) {
    if ((int)backend < 0 || (int)backend >= VV_DSP_FFT_NUM_BACKENDS) return 0;
    ensure_init();
    return slot_ok(backend);
}

/* FFTW planner knobs: no FFTW in this library (reference fft.c:55-62 behaviour). */
vv_dsp_status vv_dsp_fft_set_fftw_flag(vv_dsp_fftw_flag flag) {
    (void)flag;
    return VV_DSP_ERROR_UNSUPPORTED;
}
vv_dsp_status vv_dsp_fft_flush_fftw_cache(void) { return VV_DSP_ERROR_UNSUPPORTED; }

vv_dsp_status vv_dsp_fft_make_plan_many(size_t n, vv_dsp_fft_type type, vv_dsp_fft_dir dir, size_t batch,
                                        vv_dsp_fft_plan** out_plan) {
    if (!out_plan) return VV_DSP_ERROR_NULL_POINTER;
    *out_plan = NULL;
    if (n == 0 || batch == 0) return VV_DSP_ERROR_INVALID_SIZE;
    if (type != VV_DSP_FFT_C2C && type != VV_DSP_FFT_R2C && type != VV_DSP_FFT_C2R) return VV_DSP_ERROR_OUT_OF_RANGE;
    if (dir != VV_DSP_FFT_FORWARD && dir != VV_DSP_FFT_BACKWARD) return VV_DSP_ERROR_OUT_OF_RANGE;
    ensure_init();
    if (!slot_ok(g_current)) return VV_DSP_ERROR_UNSUPPORTED;
    vv_amd_fft_plan* w = (vv_amd_fft_plan*)calloc(1, sizeof(*w));
    if (!w) return VV_DSP_ERROR_INTERNAL;
    vv_dsp_fft_plan* p = &w->pub;
    p->n = n;
    p->type = type;
    p->dir = dir;
    p->backend = g_current;
    w->batch = batch;
    t_pending_spec = p;
    t_pending_batch = batch;
    vv_dsp_status st = g_fft_backends[p->backend]->make_plan(p, &p->backend_plan.generic);
    t_pending_spec = NULL;
    t_pending_batch = 1;
    if (st != VV_DSP_OK) {
        free(w);
        return st;
    }
    *out_plan = p;
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_fft_make_plan(size_t n, vv_dsp_fft_type type, vv_dsp_fft_dir dir, vv_dsp_fft_plan** out_plan) {
    return vv_dsp_fft_make_plan_many(n, type, dir, 1, out_plan);
}

static size_t in_stride_bytes(const vv_dsp_fft_plan* p) {
    return p->type == VV_DSP_FFT_C2C ? 8 * p->n : p->type == VV_DSP_FFT_R2C ? 4 * p->n : 8 * (p->n / 2 + 1);
}
static size_t out_stride_bytes(const vv_dsp_fft_plan* p) {
    return p->type == VV_DSP_FFT_C2C ? 8 * p->n : p->type == VV_DSP_FFT_R2C ? 8 * (p->n / 2 + 1) : 4 * p->n;
}

vv_dsp_status vv_dsp_fft_execute(const vv_dsp_fft_plan* plan, const void* in, void* out) {
    if (!plan || !in || !out) return VV_DSP_ERROR_NULL_POINTER;
    const vv_dsp_fft_backend_vtable* vt = g_fft_backends[plan->backend];
    if (!vt || !vt->is_available()) return VV_DSP_ERROR_UNSUPPORTED;
    if (plan->backend == VV_DSP_FFT_BACKEND_HIP || vv_amd_plan_batch(plan) == 1)
        return vt->execute(plan, plan->backend_plan.generic, in, out);
    /* CPU backends have no batch notion: one call per transform */
    for (size_t b = 0; b < vv_amd_plan_batch(plan); ++b) {
        vv_dsp_status st = vt->execute(plan, plan->backend_plan.generic,
                                       (const char*)in + b * in_stride_bytes(plan),
                                       (char*)out + b * out_stride_bytes(plan));
        if (st != VV_DSP_OK) return st;
    }
    return VV_DSP_OK;
}

vv_dsp_status vv_dsp_fft_execute_device(const vv_dsp_fft_plan* plan, const void* d_in, void* d_out, void* stream) {
    if (!plan || !d_in || !d_out) return VV_DSP_ERROR_NULL_POINTER;
    if (plan->backend != VV_DSP_FFT_BACKEND_HIP) return VV_DSP_ERROR_UNSUPPORTED;
    return (vv_dsp_status)vvhip_fft_exec_device((vvhip_fft*)plan->backend_plan.generic, d_in, d_out, vv_amd_plan_batch(plan),
                                                stream);
}

vv_dsp_status vv_dsp_fft_destroy(vv_dsp_fft_plan* plan) {
    if (!plan) return VV_DSP_OK;
    const vv_dsp_fft_backend_vtable* vt =
        ((int)plan->backend >= 0 && (int)plan->backend < VV_DSP_FFT_NUM_BACKENDS) ? g_fft_backends[plan->backend] : NULL;
    if (vt && vt->free_plan) vt->free_plan(plan->backend_plan.generic);
    free((vv_amd_fft_plan*)plan);
    return VV_DSP_OK;
}

int vv_dsp_amd_device_count(void) { return vvhip_available(); }
vv_dsp_status vv_dsp_amd_set_device(int device) { return (vv_dsp_status)vvhip_set_device(device); }
vv_dsp_status vv_dsp_amd_get_device(int* device) {
    if (!device) return VV_DSP_ERROR_NULL_POINTER;
    return (vv_dsp_status)vvhip_get_device(device);
}
const char* vv_dsp_amd_last_error(void) { return vvhip_last_error(); }
