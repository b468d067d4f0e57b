/* refbench.c -- CPU-baseline driver for bench.py (TEST/BENCH INFRASTRUCTURE ONLY).
 *
 * Runs the REFERENCE's own public API (oracle/_ref/libvvref.so, the reference
 * sources compiled by oracle/Makefile) over many transforms in one C call, so
 * that bench.py's threaded cpu_baseline leg times the reference and not the
 * Python loop around it: ctypes releases the GIL for the whole call.
 * Never linked into or loaded by the product (vv-dsp_amd/).
 *
 *   refbench_fft_rows: `count` consecutive n-point C2C transforms through one
 *   plan, exactly as a caller of vv_dsp_fft_make_plan / vv_dsp_fft_execute
 *   (reference src/spectral/fft.c:63-100) would loop over a batch. */
#include <stddef.h>

typedef struct vv_dsp_fft_plan vv_dsp_fft_plan;
int vv_dsp_fft_make_plan(size_t n, int type, int dir, vv_dsp_fft_plan** out_plan);
int vv_dsp_fft_execute(const vv_dsp_fft_plan* plan, const void* in, void* out);
int vv_dsp_fft_destroy(vv_dsp_fft_plan* plan);

int refbench_fft_rows(const float* in, float* out, size_t n, size_t count, int dir) {
    vv_dsp_fft_plan* p = NULL;
    int st = vv_dsp_fft_make_plan(n, 0 /* C2C */, dir, &p);
    if (st) return st;
    for (size_t i = 0; i < count && !st; ++i) st = vv_dsp_fft_execute(p, in + 2 * n * i, out + 2 * n * i);
    vv_dsp_fft_destroy(p);
    return st;
}
