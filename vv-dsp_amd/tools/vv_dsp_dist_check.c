/* vv_dsp_dist_check.c -- the multi-GPU layer from plain C, no torch, no Python
 * (include/vv_dsp/vv_dsp_dist.h; SURVEY 8e, BASELINE config 5's "sharded across
 * GPUs, RCCL gather over xGMI").
 *
 *   vv_dsp_dist_check [ndev] [--loopback W]
 *
 * One process drives `ndev` GPUs (default: every visible one) through
 * vv_dsp_dist_init_all (ncclCommInitAll): a 7-channel x 20 s STFT is sharded by
 * channel (vv_dsp_shard_range: uneven shards), each device computes its shard on
 * its own stream (vv_dsp_dist_stft), and vv_dsp_dist_gather_rows collects every
 * rank's rows on a root -- roots 0 and ndev-1, full and half-spectrum rows.  Each
 * gathered spectrogram must equal the single-call rows of device 0 bit for bit.
 * With --loopback W the same runs on a W-rank loopback context on device 0
 * (transfers as device copies).  Prints one JSON line; exit status 0 iff every
 * comparison matched.  Reference semantics: src/spectral/stft.c:112-144.
 *
 * Built by vv-dsp_amd/Makefile (gcc; the HIP runtime's C API for device memory,
 * streams and events) into vv-dsp_amd/bin/. */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vv_dsp/spectral/stft.h"
#include "vv_dsp/vv_dsp_amd.h"
#include "vv_dsp/vv_dsp_dist.h"

#define MAXDEV 64
#define CHECK(x)                                                                      \
    do {                                                                              \
        int rc_ = (int)(x);                                                           \
        if (rc_ != 0) {                                                               \
            fprintf(stderr, "%s:%d: %s -> %d\n", __FILE__, __LINE__, #x, rc_);        \
            printf("{\"ok\": false, \"failed\": \"%s\"}\n", #x);                      \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

enum { NCH = 7, NFFT = 1024, HOP = 256 };
static const size_t N = 48000 * 20 + 333;

static float lcg(uint32_t* s) {   /* uniform [-1, 1) */
    *s = *s * 1664525u + 1013904223u;
    return (float)((*s >> 8) * (1.0 / 16777216.0)) * 2.0f - 1.0f;
}

int main(int argc, char** argv) {
    int ndev = 0, loop = 0;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--loopback") && i + 1 < argc) loop = atoi(argv[++i]);
        else ndev = atoi(argv[i]);
    }
    int visible = 0;
    CHECK(hipGetDeviceCount(&visible));
    if (ndev <= 0) ndev = visible;
    if (ndev > visible || ndev > MAXDEV || loop > MAXDEV) {
        printf("{\"ok\": false, \"error\": \"%d devices asked, %d visible\"}\n", ndev, visible);
        return 1;
    }
    const int world = loop > 0 ? loop : ndev;
    const size_t frames = 1 + (N - NFFT + HOP) / HOP, row = NFFT, rows_ch = frames * row;

    /* host signal, and the single-call reference rows from device 0 */
    float* h_sig = (float*)malloc(sizeof(float) * NCH * N);
    float* h_ref = (float*)malloc(sizeof(float) * NCH * rows_ch);
    float* h_got = (float*)malloc(sizeof(float) * NCH * rows_ch);
    if (!h_sig || !h_ref || !h_got) return 1;
    uint32_t seed = 12345u;
    for (size_t i = 0; i < (size_t)NCH * N; ++i) h_sig[i] = lcg(&seed);
    vv_dsp_stft_params prm = {NFFT, HOP, VV_DSP_STFT_WIN_HANN};
    vv_dsp_stft* st = NULL;
    CHECK(hipSetDevice(0));
    CHECK(vv_dsp_stft_create(&prm, &st));
    float *d_sig0 = NULL, *d_ref0 = NULL;
    CHECK(hipMalloc((void**)&d_sig0, sizeof(float) * NCH * N));
    CHECK(hipMalloc((void**)&d_ref0, sizeof(float) * NCH * rows_ch));
    CHECK(hipMemcpy(d_sig0, h_sig, sizeof(float) * NCH * N, hipMemcpyHostToDevice));
    size_t fr = 0;
    CHECK(vv_dsp_stft_spectrogram_device(st, d_sig0, N, NCH, N, d_ref0, rows_ch, NULL, &fr));
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(h_ref, d_ref0, sizeof(float) * NCH * rows_ch, hipMemcpyDeviceToHost));

    /* the context: every rank in this process */
    vv_dsp_dist* d = NULL;
    int devs[MAXDEV];
    for (int i = 0; i < ndev; ++i) devs[i] = i;
    if (loop > 0) CHECK(vv_dsp_dist_init_loopback(loop, 0, &d));
    else CHECK(vv_dsp_dist_init_all(ndev, devs, &d));
    const int slots = vv_dsp_dist_local_ranks(d);
    int count = 0;
    CHECK(vv_dsp_dist_comm_count(d, 0, &count));

    /* each rank's shard on its device: signal rows and output rows, one stream */
    const float* sig_p[MAXDEV];
    void* rows_p[MAXDEV];
    void* streams[MAXDEV];
    size_t first[MAXDEV], cnt[MAXDEV];
    int dev_of[MAXDEV];
    for (int s = 0; s < slots; ++s) {
        int r = 0, w = 0, dv = 0;
        CHECK(vv_dsp_dist_rank_info(d, s, &r, &w, &dv));
        CHECK(vv_dsp_shard_range(NCH, (size_t)w, (size_t)r, &first[s], &cnt[s]));
        dev_of[s] = dv;
        CHECK(hipSetDevice(dv));
        hipStream_t hs;
        CHECK(hipStreamCreateWithFlags(&hs, hipStreamNonBlocking));
        streams[s] = hs;
        float *ds = NULL, *dr = NULL;
        CHECK(hipMalloc((void**)&ds, sizeof(float) * (cnt[s] ? cnt[s] : 1) * N));
        CHECK(hipMalloc((void**)&dr, sizeof(float) * (cnt[s] ? cnt[s] : 1) * rows_ch));
        if (cnt[s]) CHECK(hipMemcpy(ds, h_sig + first[s] * N, sizeof(float) * cnt[s] * N, hipMemcpyHostToDevice));
        sig_p[s] = ds;
        rows_p[s] = dr;
    }
    CHECK(vv_dsp_dist_stft(d, st, sig_p, N, NCH, N, 0, rows_p, streams, &fr));
    for (int s = 0; s < slots; ++s) {
        CHECK(hipSetDevice(dev_of[s]));
        CHECK(hipStreamSynchronize((hipStream_t)streams[s]));
    }

    int ok = fr == frames, runs = 0, matched = 0;
    double gather_ms[4] = {0, 0, 0, 0};
    const int roots[2] = {0, world - 1};
    for (int ri = 0; ri < 2; ++ri) {
        const int root = roots[ri];
        int rs = -1;   /* the root's slot (every rank is local here) */
        for (int s = 0; s < slots; ++s) {
            int r = 0;
            CHECK(vv_dsp_dist_rank_info(d, s, &r, NULL, NULL));
            if (r == root) rs = s;
        }
        for (int half = 0; half < 2; ++half) {
            float* d_out = NULL;
            CHECK(hipSetDevice(dev_of[rs]));
            CHECK(hipMalloc((void**)&d_out, sizeof(float) * NCH * rows_ch));
            /* poison on the root's stream: the streams are non-blocking, so a memset on
             * the null stream would not be ordered before the gather's copies */
            CHECK(hipMemsetAsync(d_out, 0xff, sizeof(float) * NCH * rows_ch, (hipStream_t)streams[rs]));
            hipEvent_t e0, e1;
            CHECK(hipEventCreate(&e0));
            CHECK(hipEventCreate(&e1));
            CHECK(hipEventRecord(e0, (hipStream_t)streams[rs]));
            CHECK(vv_dsp_dist_gather_rows(d, (const vv_dsp_real* const*)rows_p, NCH, frames, row, half, d_out, root,
                                          streams));
            CHECK(hipSetDevice(dev_of[rs]));
            CHECK(hipEventRecord(e1, (hipStream_t)streams[rs]));
            for (int s = 0; s < slots; ++s) {
                CHECK(hipSetDevice(dev_of[s]));
                CHECK(hipStreamSynchronize((hipStream_t)streams[s]));
            }
            float ms = 0.0f;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            gather_ms[2 * ri + half] = ms;
            CHECK(hipSetDevice(dev_of[rs]));
            CHECK(hipMemcpy(h_got, d_out, sizeof(float) * NCH * rows_ch, hipMemcpyDeviceToHost));
            const int same = memcmp(h_got, h_ref, sizeof(float) * NCH * rows_ch) == 0;
            matched += same;
            ++runs;
            ok = ok && same;
            CHECK(hipFree(d_out));
            CHECK(hipEventDestroy(e0));
            CHECK(hipEventDestroy(e1));
        }
    }
    printf("{\"ok\": %s, \"mode\": \"%s\", \"world\": %d, \"rccl_ranks\": %d, \"devices\": %d, \"channels\": %d, "
           "\"frames\": %zu, \"gathers_bit_identical\": \"%d/%d\", \"gather_ms\": [%.3f, %.3f, %.3f, %.3f]}\n",
           ok ? "true" : "false", loop > 0 ? "loopback" : "init_all", world, count, loop > 0 ? 1 : ndev, NCH, frames,
           matched, runs, gather_ms[0], gather_ms[1], gather_ms[2], gather_ms[3]);
    for (int s = 0; s < slots; ++s) {
        CHECK(hipSetDevice(dev_of[s]));
        CHECK(hipFree((void*)sig_p[s]));
        CHECK(hipFree(rows_p[s]));
        CHECK(hipStreamDestroy((hipStream_t)streams[s]));
    }
    vv_dsp_dist_destroy(d);
    CHECK(hipSetDevice(0));
    vv_dsp_stft_destroy(st);
    CHECK(hipFree(d_sig0));
    CHECK(hipFree(d_ref0));
    free(h_sig);
    free(h_ref);
    free(h_got);
    return ok ? 0 : 1;
}
