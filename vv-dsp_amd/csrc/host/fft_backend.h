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
    size_t batch; /* appended field: transforms per execute (1 for the reference API) */
};

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
