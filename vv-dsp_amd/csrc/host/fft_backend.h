/* fft_backend.h -- internal plan object and backend vtable of the FFT front-end.
 * Same layout as the reference's src/spectral/fft_backend.h:17-38 so that a
 * backend object compiled against the reference header (e.g. its KissFFT
 * backend) can be registered in a slot and read spec->n/type/dir. */
#ifndef VV_AMD_FFT_BACKEND_H
#define VV_AMD_FFT_BACKEND_H
#include "vv_dsp/spectral/fft.h"

#define VV_DSP_FFT_NUM_BACKENDS 4

struct vv_dsp_fft_plan {
    size_t n;
    vv_dsp_fft_type type;
    vv_dsp_fft_dir dir;
    vv_dsp_fft_backend backend;
    union {
        void* generic;
    } backend_plan;
};

/* Plans made by THIS library's dispatcher carry a batch count.  It lives in a
 * wrapper around the reference-sized plan, never inside it: a backend vtable
 * must not read past struct vv_dsp_fft_plan, because the reference's
 * dispatcher mallocs exactly that struct (src/spectral/fft.c:76) before it
 * calls make_plan.  The HIP vtable learns the batch through
 * vv_amd_fft_pending_batch(), which answers 1 for any plan it did not
 * allocate itself (e.g. one made by the reference's own fft.c). */
typedef struct vv_amd_fft_plan {
    struct vv_dsp_fft_plan pub; /* first member: the opaque user handle points here */
    size_t batch;               /* transforms per execute (1 for the reference API) */
} vv_amd_fft_plan;

static inline size_t vv_amd_plan_batch(const struct vv_dsp_fft_plan* p) {
    return ((const vv_amd_fft_plan*)p)->batch;
}

/* Batch of the plan currently inside this thread's make_plan_many (fft.c), or 1
 * when `spec` is not that plan. */
__attribute__((visibility("hidden"))) size_t vv_amd_fft_pending_batch(const struct vv_dsp_fft_plan* spec);

typedef struct vv_dsp_fft_backend_vtable {
    vv_dsp_status (*make_plan)(const struct vv_dsp_fft_plan* spec, void** backend_data);
    vv_dsp_status (*execute)(const struct vv_dsp_fft_plan* spec, void* backend_data, const void* in, void* out);
    void (*free_plan)(void* backend_data);
    int (*is_available)(void);
    const char* name;
} vv_dsp_fft_backend_vtable;

extern const vv_dsp_fft_backend_vtable vv_dsp_fft_hip_vtable;
extern const vv_dsp_fft_backend_vtable* g_fft_backends[VV_DSP_FFT_NUM_BACKENDS];

#endif
